"""Interleaved A/B of k_reduce shapes on the bench's config-2 pushes (mixed row
order), one process: rounds x variants, median reduce time per variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from distml_amd import DataDesc, DataStore, KeyRange, _lib  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1].split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    L = _lib.load()
    fmt = DataDesc(1, 0, 1)
    store = DataStore(fmt, KeyRange(0, bench.ROWS - 1), bench.COLS)
    store.synth_fill(7)
    bufs = bench.make_buckets(L, torch, fmt, bench.W, bench.ROWS)
    ptrs, lens = [b.data_ptr() for b in bufs], [b.numel() for b in bufs]
    algo = bench.W * bench.BUCKET + 2 * bench.SHARD
    res = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            os.environ["DML_REDUCE_VARIANT"] = str(v)
            store.pushDevice(ptrs, lens)
            store.flush()
            store.set_timing(True)
            store.kernel_time(reset=True)
            for _ in range(10):
                store.pushDevice(ptrs, lens)
            store.flush()
            ms, k = store.kernel_time(reset=True)
            store.set_timing(False)
            res[v].append(ms / k * 1e3)
    for v, d in res.items():
        m = float(np.median(d))
        print(json.dumps({"variant": v, "reduce_us_median": round(m, 1), "reduce_us_min": round(min(d), 1),
                          "TBps": round(algo / m / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
