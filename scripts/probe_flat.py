"""Config-4 kernel probe (diagnostic): the dense narrow-row reduce
(k_reduce_flat) of W full-range pushes into a rows x cols fp32 store, at several
model sizes, timed per launch with the store's HIP events; plus the box's measured
read / copy ceilings over the same byte count. One JSON line per case.

  python scripts/probe_flat.py --rows 10000000 1250000 --pushes 16 --reps 4
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[10_000_000, 1_250_000])
    ap.add_argument("--cols", type=int, default=200)
    ap.add_argument("--pushes", type=int, nargs="+", default=[16])
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--order", choices=["asc", "perm"], default="asc")
    ap.add_argument("--slab", action="store_true", help="pushes as slices of one allocation")
    ap.add_argument("--streams", action="store_true", help="also time read / copy ceilings")
    args = ap.parse_args()
    import torch
    from distml_amd import DataDesc, DataStore, KeyRange, _lib
    from distml_amd.store import DeviceBatch
    L = _lib.load()
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_FLOAT)
    st = torch.cuda.current_stream().cuda_stream
    cols = args.cols
    rec = 4 + 4 * cols
    for rows in args.rows:
        for w in args.pushes:
            if args.slab:
                slab = torch.empty(w * rows * rec, dtype=torch.uint8, device="cuda")
                bufs = [slab[b * rows * rec:(b + 1) * rows * rec] for b in range(w)]
            else:
                bufs = [torch.empty(rows * rec, dtype=torch.uint8, device="cuda") for _ in range(w)]
            for b, t in enumerate(bufs):
                pa, pc = (1, 0) if args.order == "asc" else ((2654435761 * (b + 1)) % rows | 1, b * 7919 % rows)
                while args.order == "perm" and __import__("math").gcd(pa, rows) != 1:
                    pa += 2
                assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows, rows, cols, 3000 + b,
                                                pa, pc, C.c_void_p(st)) == 0
            torch.cuda.synchronize()
            store = DataStore(fmt, KeyRange(0, rows - 1), cols, device=0)
            store.synth_fill(13)
            batch = DeviceBatch([t.data_ptr() for t in bufs], [t.numel() for t in bufs])
            store.pushDevice(batch)
            store.flush()
            store.set_timing(True)
            store.kernel_time(reset=True)
            for _ in range(args.reps):
                store.pushDevice(batch)
            store.flush()
            ms, n = store.kernel_time(reset=True)
            algo = w * rows * rec + 2 * rows * cols * 4
            us = ms / max(n, 1) * 1e3
            out = {"rows": rows, "cols": cols, "pushes": w, "order": args.order, "slab": args.slab,
                   "kernel": store.kernel_name(), "launches": n, "avg_kernel_us": round(us, 1),
                   "algo_bytes": algo, "GBps": round(algo / us / 1e3, 1), "frac": round(algo / us / 1e3 / 8000, 4),
                   "stats": store.stats()}
            store.close()
            del bufs, batch
            if args.slab:
                del slab
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            print(json.dumps(out), flush=True)
    if args.streams:
        for gb in (2, 8, 32):
            n = gb << 30
            src = torch.empty(n, dtype=torch.uint8, device="cuda")
            dst = torch.empty(n if gb <= 8 else 1 << 20, dtype=torch.uint8, device="cuda")
            res = {"stream_bytes": n}
            for copy in ((0, 1) if gb <= 8 else (0,)):
                best = 1e9
                for _ in range(3):
                    ms = C.c_float()
                    assert L.dml_diag_stream(copy, dst.data_ptr(), src.data_ptr(), n, C.c_void_p(st), C.byref(ms)) == 0
                    best = min(best, ms.value)
                res["copy_GBps" if copy else "read_GBps"] = round((2 if copy else 1) * n / best / 1e6, 1)
            print(json.dumps(res), flush=True)
            del src, dst
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
