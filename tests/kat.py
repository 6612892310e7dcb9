"""Shared loaders for tests/golden/kat_cases.json (used by the oracle and GPU tests)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
VDT = {0: "<i4", 1: "<f4", 3: "<f8"}


def load():
    with open(os.path.join(HERE, "golden", "kat_cases.json")) as f:
        return json.load(f)


def cases():
    return load()["cases"]


def expected_array(case, key="data_hex", dtype=None):
    dt = dtype or VDT[case["desc"]["value_type"]]
    rows = case["last"] - case["first"] + 1
    return np.frombuffer(bytes.fromhex(case["expected"][key]), dtype=dt).reshape(rows, case["cols"])


def init_array(case):
    dt = VDT[case["desc"]["value_type"]]
    rows = case["last"] - case["first"] + 1
    return np.frombuffer(bytes.fromhex(case["init_hex"]), dtype=dt).reshape(rows, case["cols"])


def pushes(case):
    return [bytes.fromhex(h) for h in case["pushes_hex"]]


def bits_equal(a, b) -> bool:
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()
