"""CPU: pin the oracle (oracle/dml_oracle.c) against the golden KATs.

The KAT expectations come from tests/golden/make_golden.py's independent
numpy restatement plus literal hand-computed values. Parity of the oracle
with the Java reference itself is UNPINNED (no JDK, no reference fixtures);
see DESIGN.md §Oracle.
"""
import math

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


def test_java_random_known_answers(oracle):
    """java.util.Random restated for DoubleMatrixStore.rand (DoubleMatrixStore.java:
    192-207), pinned by outputs the JDK prints for these seeds (widely published:
    new Random(42).nextInt() = -1170105035; nextGaussian() of seeds 42 / 0 / 1 =
    1.1419053154730547 / 0.8025330637390305 / 1.561581040188955). The gaussians go
    through the polar method's StrictMath.log, so they also pin the fdlibm log."""
    assert int(oracle.java_random_ints(42, 1)[0]) == -1170105035
    assert repr(float(oracle.java_random_gaussians(42, 1)[0])) == "1.1419053154730547"
    assert repr(float(oracle.java_random_gaussians(0, 1)[0])) == "0.8025330637390305"
    assert repr(float(oracle.java_random_gaussians(1, 1)[0])) == "1.561581040188955"
    # the second gaussian of a pair is the cached nextNextGaussian
    g = oracle.java_random_gaussians(1, 4)
    assert len(set(g.tolist())) == 4


def test_fdlibm_log(oracle):
    """StrictMath.log = fdlibm's __ieee754_log: specials, exact points, and within
    one ulp of the C library's log everywhere (it is not the same function: they
    differ in the last bit for a few percent of arguments)."""
    import math
    L = oracle.fdlibm_log
    assert L(1.0) == 0.0 and L(0.0) == -math.inf and L(-0.0) == -math.inf
    assert math.isnan(L(-1.0)) and L(math.inf) == math.inf and math.isnan(L(math.nan))
    assert L(2.0) == 0.6931471805599453 and L(5e-324) == -744.4400719213812
    rng = np.random.default_rng(4)
    xs = np.concatenate([rng.random(20000), rng.random(2000) * 1e-310, np.exp(rng.uniform(-700, 700, 20000))])
    diff = 0
    for x in xs.tolist():
        a, b = L(x), math.log(x)
        assert abs(a - b) <= math.ulp(b), x
        diff += a != b
    assert 0 < diff < len(xs) // 5


def test_oracle_double_matrix_rand(oracle):
    """orc_rand: one Random(1L) stream over the shard's rows (cols |g| each), rows of
    unit norm; the first row is exactly |gaussian| x 3 / norm in double."""
    s = oracle.OracleStore(1, 1, 3, 100, 109, 3)
    assert s.rand() == 0
    g = np.abs(oracle.java_random_gaussians(1, 30)).reshape(10, 3)
    for i in range(10):
        nrm = math.sqrt(g[i, 0] * g[i, 0] + g[i, 1] * g[i, 1] + g[i, 2] * g[i, 2])
        assert s.data[i].tolist() == [g[i, j] / nrm for j in range(3)]
    assert oracle.OracleStore(1, 0, 1, 0, 9, 3).rand() != 0  # float matrices: unseeded in the reference


def test_java_parse_float():
    """Float.parseFloat for DataStore.set(String): one rounding to float32."""
    from distml_amd.store import java_parse_float as pf
    assert pf("0.1") == float(np.float32(0.1)) and pf(" 3 ") == 3.0 and pf("2.5f") == 2.5 and pf("-0") == 0.0
    assert math.copysign(1, pf("-0.0")) == -1 and pf("Infinity") == math.inf and math.isnan(pf("NaN"))
    assert pf("0x1.8p1") == 3.0 and pf("1e-50") == 0.0 and pf("1e39") == math.inf
    # the exact float32 tie 1 + 2^-24 goes to the even side; one digit above it rounds up,
    # where a detour through double (which holds the tie exactly) would round down
    up = float(np.nextafter(np.float32(1), np.float32(2)))
    assert pf("1.000000059604644775390625") == 1.0 and pf("1.000000059604644775390626") == up
    assert pf(".5") == 0.5 and pf("1.") == 1.0 and pf("+1e2") == 100.0 and pf("1.e1") == 10.0
    # Float.parseFloat throws NumberFormatException on these (Fraction would take the first two)
    for bad in ("abc", "1/2", "1_0", "1e", "--1", ".", "1..2", ""):
        with pytest.raises(ValueError):
            pf(bad)


def test_row_subset_generators_match_full(oracle):
    """synth_dense_rows / synth_fill_rows (the full-size tests' sampled rows) hold
    exactly the values the full generators give those rows, whatever the push order."""
    rows, cols = 1000, 7
    pick = np.array([0, 5, 6, 999, 512, 3])
    for vt in (0, 1, 3):
        V = 8 if vt == 3 else 4
        dt = {0: "<i4", 1: "<f4", 3: "<f8"}[vt]
        full = oracle.synth_dense_bucket(0, vt, 0, rows, rows, cols, 77, 3, 11).reshape(rows, 4 + V * cols)
        keys = full[:, :4].copy().view("<i4").ravel()
        byrow = {int(k): full[i, 4:].tobytes() for i, k in enumerate(keys)}
        sub = oracle.synth_dense_rows(0, vt, pick, cols, 77).reshape(len(pick), 4 + V * cols)
        assert sub[:, :4].copy().view("<i4").ravel().tolist() == list(range(len(pick)))
        assert [sub[i, 4:].tobytes() for i in range(len(pick))] == [byrow[int(r)] for r in pick]
        s = oracle.OracleStore(1, 0, vt, 0, rows - 1, cols)
        s.synth_fill(9)
        t = oracle.OracleStore(1, 0, vt, 0, len(pick) - 1, cols)
        t.synth_fill_rows(pick, 9)
        assert t.data.view(dt).tobytes() == s.data[pick].tobytes()
