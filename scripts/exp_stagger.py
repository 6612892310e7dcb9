"""Ascending-order config-2 pushes whose base addresses are staggered by
b * step bytes inside one pool (do bank/channel offsets between the 32 pushes
matter?), default reduce launch shape."""
import ctypes as C
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    L = _lib.load()
    fmt = DataDesc(1, 0, 1)
    store = DataStore(fmt, KeyRange(0, bench.ROWS - 1), bench.COLS)
    store.synth_fill(7)
    st = torch.cuda.current_stream().cuda_stream
    span = (bench.BUCKET + (4 << 20) + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    pool = torch.empty(span * bench.W, dtype=torch.uint8, device="cuda")
    res = {}
    for _ in range(rounds):
        for step in (0, 4096, 4352, 65536 + 256, 1 << 20, 3 << 19):
            ptrs = [pool.data_ptr() + b * span + (b * step) % (4 << 20) for b in range(bench.W)]
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
    algo = bench.W * bench.BUCKET + 2 * bench.SHARD
    for step, v in res.items():
        print(json.dumps({"stagger_bytes_per_push": step, "span": span, "reduce_us_median": round(float(np.median(v)), 1),
                          "reduce_TBps": round(algo / float(np.median(v)) / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
