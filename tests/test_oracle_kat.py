"""CPU: pin the oracle (oracle/dml_oracle.c) against the golden KATs.

The KAT expectations come from tests/golden/make_golden.py's independent
numpy restatement plus literal hand-computed values. Parity of the oracle
with the Java reference itself is UNPINNED (no JDK, no reference fixtures);
see DESIGN.md §Oracle.
"""
import numpy as np
import pytest

import kat


@pytest.mark.parametrize("case", kat.cases(), ids=lambda c: c["name"])
def test_oracle_matches_kat(oracle, case):
    d = case["desc"]
    s = oracle.OracleStore(d["data_type"], d["key_type"], d["value_type"], case["first"], case["last"],
                           case["cols"], d["dense_column"], d["ada_grad"], case["float_array_ref_stride"])
    s.data[:] = kat.init_array(case)
    if case["ada"]:
        s.set_alpha(*case["ada"])
    status = 0
    applied = 0
    for p in kat.pushes(case):
        status = s.push(p)
        applied += 1
        if status:
            break
    exp = case["expected"]
    assert status == exp["status"]
    assert applied == exp["pushes_applied"]
    if status:
        code, key, col = s.error()
        assert (code, key, col) == (exp["status"], exp["key"], exp["col"])
    assert kat.bits_equal(s.data, kat.expected_array(case))
    if case["ada"]:
        assert kat.bits_equal(s.alpha, kat.expected_array(case, "alpha_hex", "<f4"))
        assert kat.bits_equal(s.delta, kat.expected_array(case, "delta_hex", "<f4"))
        v, r, c = s.max_delta()
        assert [v, r, c] == exp["max_delta"]


def test_linear_split_kat(oracle):
    from distml_amd.datadesc import KeyRange
    for name, want in kat.load()["linear_split"].items():
        first, last, n = map(int, name.split("_"))
        assert [list(x) for x in oracle.linear_split(first, last, n)] == want
        assert [[r.firstKey, r.lastKey] for r in KeyRange(first, last).linearSplit(n)] == want


def test_oracle_fetch_and_checkpoint_layout(oracle):
    # FloatMatrixStore.handleFetch dense layout (:140-153) and writeAll big-endian (:74-81)
    s = oracle.OracleStore(1, 0, 1, 10, 12, 2)
    s.data[:] = np.array([[1.0, -2.0], [0.5, 3.0], [7.0, 8.0]], np.float32)
    out = s.fetch([12, 10])
    want = (np.array([12], "<i4").tobytes() + np.array([7.0, 8.0], "<f4").tobytes() +
            np.array([10], "<i4").tobytes() + np.array([1.0, -2.0], "<f4").tobytes())
    assert out == want
    assert s.write_all() == s.data.astype(">f4").tobytes()
    # FloatArrayStore fetch: 4 value bytes in an 8-byte zeroed slot (FloatArrayStore.java:92-105)
    a = oracle.OracleStore(0, 1, 1, 0, 3)
    a.data[:] = np.array([[1.0], [2.0], [3.0], [4.0]], np.float32)
    assert a.fetch([2]) == np.array([2], "<i8").tobytes() + np.array([3.0], "<f4").tobytes() + b"\0" * 4
    # readAll round trip
    b = oracle.OracleStore(1, 0, 3, 0, 1, 3)
    src = np.arange(6, dtype=np.float64).reshape(2, 3) / 7
    assert b.read_all(src.astype(">f8").tobytes()) == 0
    assert kat.bits_equal(b.data, src)


def test_oracle_synth_is_deterministic(oracle):
    a = oracle.synth_dense_bucket(0, 1, 0, 64, 64, 16, seed=1000, perm_a=5, perm_c=3)
    b = oracle.synth_dense_bucket(0, 1, 0, 64, 64, 16, seed=1000, perm_a=5, perm_c=3)
    assert a.tobytes() == b.tobytes()
    rec = a.reshape(64, 4 + 64)
    keys = rec[:, :4].copy().view("<i4").ravel()
    assert sorted(keys.tolist()) == list(range(64))  # a permutation of the shard's rows
    # values depend on (row, col) only: the permuted bucket carries the same row values
    c = oracle.synth_dense_bucket(0, 1, 0, 64, 64, 16, seed=1000, perm_a=1, perm_c=0).reshape(64, 68)
    for r in range(64):
        k = int(keys[r])
        assert rec[r, 4:].tobytes() == c[k, 4:].tobytes()
    vals = c[:, 4:].copy().view("<f4")
    assert 5e-4 < float(np.std(vals)) < 2e-3


def test_oracle_push_many_threads_matches_sequential(oracle):
    bufs = [oracle.synth_dense_bucket(0, 1, 0, 257, 257, 33, seed=1000 + b, perm_a=2 * b + 1, perm_c=b)
            for b in range(5)]
    s1 = oracle.OracleStore(1, 0, 1, 0, 256, 33)
    s1.synth_fill(7)
    s4 = oracle.OracleStore(1, 0, 1, 0, 256, 33)
    s4.synth_fill(7)
    assert s1.push_many(bufs, threads=1) == 0
    assert s4.push_many(bufs, threads=4) == 0
    assert kat.bits_equal(s1.data, s4.data)
