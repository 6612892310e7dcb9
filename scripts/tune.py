"""Interleaved A/B of kernel variants on the config-2 workload (one process,
rounds x variants, median/min reported; MI355X guide §5.4 rule 24).

Variants are selected per launch by env vars read inside libdistml_ps:
  DML_REDUCE_VARIANT  0: G=8 plain  1: G=8 nt  2: G=16 plain  3: G=16 nt
  DML_INDEX_VARIANT   0: atomicExch index  1: plain-store index + verify
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from distml_amd import DataDesc, DataStore, KeyRange, _lib  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    variants = [(r, 0) for r in (3, 10, 13, 14, 15)]
    L = _lib.load()
    fmt = DataDesc(1, 0, 1)
    store = DataStore(fmt, KeyRange(0, bench.ROWS - 1), bench.COLS)
    store.synth_fill(7)
    bufs = bench.make_buckets(L, torch, fmt, bench.W, bench.ROWS)
    ptrs, lens = [b.data_ptr() for b in bufs], [b.numel() for b in bufs]
    algo = bench.W * bench.BUCKET + 2 * bench.SHARD
    res = {v: {"step_us": [], "reduce_us": []} for v in variants}
    for _ in range(rounds):
        for v in variants:
            os.environ["DML_REDUCE_VARIANT"], os.environ["DML_INDEX_VARIANT"] = str(v[0]), str(v[1])
            for _ in range(2):
                store.pushDevice(ptrs, lens)
            store.flush()
            store.set_timing(True)
            store.kernel_time(reset=True)
            n = 10
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                store.pushDevice(ptrs, lens)
            store.flush()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            ms, k = store.kernel_time(reset=True)
            store.set_timing(False)
            res[v]["step_us"].append(el / n * 1e6)
            res[v]["reduce_us"].append(ms / k * 1e3)
    out = []
    for v, d in res.items():
        st, rd = np.array(d["step_us"]), np.array(d["reduce_us"])
        out.append({"reduce_variant": v[0], "index_variant": v[1],
                    "step_us_median": round(float(np.median(st)), 1), "step_us_min": round(float(st.min()), 1),
                    "reduce_us_median": round(float(np.median(rd)), 1), "reduce_us_min": round(float(rd.min()), 1),
                    "reduce_TBps_median": round(algo / float(np.median(rd)) / 1e6, 3)})
    for o in out:
        print(json.dumps(o))


def order_test(L, store, algo, rounds):
    """All pushes in ascending row order vs all permuted (same bytes)."""
    import ctypes as C
    fmt = DataDesc(1, 0, 1)
    st = torch.cuda.current_stream().cuda_stream
    sets = {}
    for name, perm in (("ascending", lambda b: (1, 0)), ("permuted", lambda b: bench.perm_for(2 * b + 1))):
        bufs = []
        for b in range(bench.W):
            t = torch.empty(bench.BUCKET, dtype=torch.uint8, device="cuda")
            pa, pc = perm(b)
            assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, bench.ROWS, bench.ROWS, bench.COLS,
                                            1000 + b, pa, pc, C.c_void_p(st)) == 0
            bufs.append(t)
        sets[name] = bufs
    torch.cuda.synchronize()
    os.environ["DML_REDUCE_VARIANT"] = "3"
    res = {k: [] for k in sets}
    for _ in range(rounds):
        for name, bufs in sets.items():
            ptrs, lens = [b.data_ptr() for b in bufs], [b.numel() for b in bufs]
            store.pushDevice(ptrs, lens)
            store.flush()
            store.set_timing(True)
            store.kernel_time(reset=True)
            for _ in range(10):
                store.pushDevice(ptrs, lens)
                store.flush()
            ms, k = store.kernel_time(reset=True)
            store.set_timing(False)
            res[name].append(ms / k * 1e3)
    for name, v in res.items():
        print(json.dumps({"row_order": name, "reduce_us_median": round(float(np.median(v)), 1),
                          "reduce_TBps": round(algo / float(np.median(v)) / 1e6, 3)}))
    del sets


def stagger_test(L, store, algo, rounds):
    """Ascending-order pushes whose base addresses are staggered by b * step bytes."""
    import ctypes as C
    fmt = DataDesc(1, 0, 1)
    st = torch.cuda.current_stream().cuda_stream
    raw = [torch.empty(bench.BUCKET + 64 * 4096, dtype=torch.uint8, device="cuda") for _ in range(bench.W)]
    res = {}
    for _ in range(rounds):
        for step in (0, 256, 4096, 4100, 65536):
            ptrs = [r.data_ptr() + (b * step) % (64 * 4096) for b, r in enumerate(raw)]
            for b, p in enumerate(ptrs):
                assert L.dml_synth_dense_bucket(C.c_void_p(p), C.byref(fmt.to_c()), 0, bench.ROWS, bench.ROWS,
                                                bench.COLS, 1000 + b, 1, 0, C.c_void_p(st)) == 0
            torch.cuda.synchronize()
            lens = [bench.BUCKET] * bench.W
            store.pushDevice(ptrs, lens)
            store.flush()
            store.set_timing(True)
            store.kernel_time(reset=True)
            for _ in range(8):
                store.pushDevice(ptrs, lens)
            store.flush()
            ms, k = store.kernel_time(reset=True)
            store.set_timing(False)
            res.setdefault(step, []).append(ms / k * 1e3)
    for step, v in res.items():
        print(json.dumps({"stagger_bytes_per_push": step, "reduce_us_median": round(float(np.median(v)), 1),
                          "reduce_TBps": round(algo / float(np.median(v)) / 1e6, 3)}))


if __name__ == "__main__":
    main()
