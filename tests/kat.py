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


def moments_within(got_data, got_alpha, got_delta, o, init, pushes, cols, what):
    """The two-moment AdaGrad path's bound: data within the
    summation-order bound of the plain sharded path and 1e-6 of sum|terms| from the
    exact sum; delta (a sum of squares, no cancellation), alpha = f(delta) and
    maxDelta within 1e-6 relative of the sequential oracle."""
    n = len(pushes) + 1
    terms = np.abs(init.astype(np.float64))
    exact = init.astype(np.float64)
    for h in pushes:
        rec = np.frombuffer(h, np.uint8).reshape(-1, 4 + 4 * cols)
        k = rec[:, :4].copy().view("<i4").ravel()
        g = rec[:, 4:].copy().view("<f4").astype(np.float64)
        np.add.at(terms, k, np.abs(g))
        np.add.at(exact, k, g)
    d = got_data.astype(np.float64)
    assert np.all(np.abs(d - o.data) <= 2 * (n - 1) * 2.0 ** -24 * terms), what
    assert float(np.max(np.abs(d - exact) / terms)) <= 1e-6, what
    od, oa = o.delta.astype(np.float64), o.alpha.astype(np.float64)
    assert float(np.max(np.abs(got_delta - od) / np.maximum(od, 1e-30))) <= 1e-6, what
    assert float(np.max(np.abs(got_alpha - oa) / np.maximum(np.abs(oa), 1e-30))) <= 1e-6, what
    assert (od > 1.0).any(), "the alpha update ran"
