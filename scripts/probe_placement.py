"""Config-2 buffer placement probe (diagnostic): the headline's
32-push reduce over bucket sets that differ only in where their pushes sit —
generated into their 32 buffers in allocation order or in a seeded order, and
allocated before or after the other sets — timed alternately on one store (k_reduce_rows
per launch, HIP events), so that allocation order and allocation position separate.
One JSON line per set and round.

  python scripts/probe_placement.py --rounds 3 --steps 100
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--slab", action="store_true")
    args = ap.parse_args()
    import torch
    import bench
    from distml_amd import DataDesc, DataStore, KeyRange, _lib
    from distml_amd.store import DeviceBatch
    L = _lib.load()
    bench.SLAB[0] = args.slab
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_FLOAT)
    sets = {}
    for name, seed in (("A_inorder_first", 0), ("B_shuffled", 7), ("C_inorder_after", 0), ("D_shuffled_after", 11)):
        bufs = bench.make_buckets(L, torch, fmt, bench.W, bench.ROWS, alloc_seed=seed)
        sets[name] = (bufs, DeviceBatch([b.data_ptr() for b in bufs], [b.numel() for b in bufs]))
    store = DataStore(fmt, KeyRange(0, bench.ROWS - 1), bench.COLS, device=0)
    store.synth_fill(7)
    algo = bench.W * bench.BUCKET + 2 * bench.SHARD
    for _, b in sets.values():
        for _ in range(10):
            store.pushDevice(b)
    store.flush()
    store.set_timing(True, every=1)
    for r in range(args.rounds):
        for name, (_, b) in sets.items():
            store.kernel_time(reset=True)
            for _ in range(args.steps):
                store.pushDevice(b)
            store.flush()
            ms, n = store.kernel_time(reset=True)
            us = ms / max(n, 1) * 1e3
            addrs = [t.data_ptr() for t in sets[name][0]]
            print(json.dumps({"set": name, "round": r, "slab": args.slab, "avg_kernel_us": round(us, 2),
                              "frac": round(algo / us / 1e3 / 8000, 4), "launches": n,
                              "push_addr_order_ascending": addrs == sorted(addrs),
                              "first_addr_gib": round(min(addrs) / 2**30, 3)}), flush=True)
    store.close()


if __name__ == "__main__":
    main()
