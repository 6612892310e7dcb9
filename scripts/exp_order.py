"""k_reduce time by push row order (config-2 shapes, default launch shape):
all ascending (the HashMap<Integer> order SparseMatrix.writeMap emits), all
permuted, and the bench's alternating mix; plus the measured read ceiling."""
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    L = _lib.load()
    fmt = DataDesc(1, 0, 1)
    store = DataStore(fmt, KeyRange(0, bench.ROWS - 1), bench.COLS)
    store.synth_fill(7)
    st = torch.cuda.current_stream().cuda_stream
    algo = bench.W * bench.BUCKET + 2 * bench.SHARD
    orders = {"ascending": lambda b: (1, 0), "permuted": lambda b: bench.perm_for(2 * b + 1), "mixed": bench.perm_for}
    sets = {}
    for name, perm in orders.items():
        bufs = []
        for b in range(bench.W):
            t = torch.empty(bench.BUCKET, dtype=torch.uint8, device="cuda")
            pa, pc = perm(b)
            assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, bench.ROWS, bench.ROWS, bench.COLS,
                                            1000 + b, pa, pc, C.c_void_p(st)) == 0
            bufs.append(t)
        sets[name] = bufs
    torch.cuda.synchronize()
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
        print(json.dumps({"row_order": name, "variant": os.environ.get("DML_REDUCE_VARIANT", "0"),
                          "reduce_us_median": round(float(np.median(v)), 1), "reduce_us_min": round(min(v), 1),
                          "reduce_TBps": round(algo / float(np.median(v)) / 1e6, 3)}), flush=True)
    del sets
    print(json.dumps({"stream_GBps": bench.stream_peaks(L, torch)}), flush=True)


if __name__ == "__main__":
    main()
