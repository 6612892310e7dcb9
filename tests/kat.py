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


def rs_parity(got, oracle_data, init, pushes, cols, what):
    """fp32 on the reduce-scatter path (north_star: within 1e-6 relative),
    against the sequential oracle's own values and the exact (fp64) sum.

    Asserted: |ours − oracle| <= 2(n−1)·2⁻²⁴·Σ|terms| per element (the two summation
    orders' bound); |ours − exact| <= 1e-6·Σ|terms|; ours no further from the exact sum
    than the oracle (+1 ulp of Σ|terms|); and, where the sum does not cancel
    (|oracle| >= Σ|terms|/4), ours within 1e-6 relative of the exact sum, and every
    element more than 1e-6 relative from the ORACLE's value one where the
    oracle is the further of the two from the exact sum: the excess is the sequential
    order's own rounding (n − 1 roundings at the shard value's magnitude; from ~40 terms
    a few elements in 10⁴, tests/test_group_gloo.py and DESIGN.md §2), never ours.
    Returns the per-case distribution — max relative deviation from the oracle's value
    and the count above 1e-6, over all elements with |oracle| > 0 and over the
    non-cancelling ones, and the same count for the oracle against the exact sum — and
    appends it to $DML_PARITY_LOG (JSON lines) when set."""
    n = len(pushes) + 1
    terms = np.abs(init.astype(np.float64))
    exact = init.astype(np.float64)
    for h in pushes:
        rec = np.frombuffer(bytes(h), np.uint8).reshape(-1, 4 + 4 * cols)
        k = rec[:, :4].copy().view("<i4").ravel()
        g = rec[:, 4:].copy().view("<f4").astype(np.float64)
        np.add.at(terms, k, np.abs(g))
        np.add.at(exact, k, g)
    d = got.astype(np.float64).reshape(exact.shape)
    ov = oracle_data.astype(np.float64).reshape(exact.shape)
    dev = np.abs(d - ov)
    assert np.all(dev <= 2 * (n - 1) * 2.0 ** -24 * terms), what
    err_ours = float(np.max(np.abs(d - exact) / terms))
    err_ref = float(np.max(np.abs(ov - exact) / terms))
    assert err_ours <= 1e-6, (what, err_ours, err_ref)
    assert err_ours <= err_ref + 2.0 ** -24, (what, err_ours, err_ref)
    nz = ov != 0
    rel = np.zeros_like(dev)
    rel[nz] = dev[nz] / np.abs(ov[nz])
    nc = np.abs(ov) >= 0.25 * terms
    stats = {"case": what, "elements": int(d.size), "terms_per_element": n,
             "max_rel_vs_oracle": float(rel[nz].max()) if nz.any() else 0.0,
             "above_1e-6_vs_oracle": int((rel[nz] > 1e-6).sum()),
             "noncancelling": int(nc.sum()),
             "max_rel_vs_oracle_noncancelling": float(rel[nc].max()) if nc.any() else 0.0,
             "above_1e-6_vs_oracle_noncancelling": int((rel[nc] > 1e-6).sum()),
             "max_rel_vs_exact_noncancelling": float((np.abs(d - exact)[nc] / np.abs(exact[nc])).max()) if nc.any() else 0.0,
             "oracle_above_1e-6_vs_exact_noncancelling": int((np.abs(ov - exact)[nc] > 1e-6 * np.abs(exact[nc])).sum()),
             "bit_equal_to_oracle": int((dev == 0).sum()),
             "max_abs_vs_exact_over_terms_ours": err_ours, "max_abs_vs_exact_over_terms_oracle": err_ref}
    log = os.environ.get("DML_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(stats) + "\n")
    assert nc.sum() > d.size // 4, (what, stats)
    assert stats["max_rel_vs_exact_noncancelling"] <= 1e-6, stats
    far = nc & (rel > 1e-6)
    assert np.all(np.abs(d - exact)[far] < np.abs(ov - exact)[far]), stats
    return stats
