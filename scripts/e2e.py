"""End-to-end host-memory path: the config-2 pushes start in
host memory (pageable, then pinned), go through dml_store_push_batch (staging,
H2D, index, ordered reduce, error check), and the shard comes back with
handleFetch (KeyRange, D2H). Reports GiB/s end to end and per stage."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pyoracle  # noqa: E402
from distml_amd import DataDesc, DataStore, KeyRange  # noqa: E402

fmt = DataDesc(1, 0, 1)
W = bench.W
host = [pyoracle.synth_dense_bucket(0, 1, 0, bench.ROWS, bench.ROWS, bench.COLS, 1000 + b, *bench.perm_for(b))
        for b in range(W)]
algo = W * bench.BUCKET + 2 * bench.SHARD
res = {}
store = DataStore(fmt, KeyRange(0, bench.ROWS - 1), bench.COLS)
store.rand(7)
for kind in ("pageable", "pinned"):
    if kind == "pinned":
        pinned = [torch.from_numpy(h).pin_memory() for h in host]
        bufs = [p.numpy() for p in pinned]
    else:
        bufs = host
    ptrs = (C.c_void_p * W)(*[b.ctypes.data for b in bufs])
    lens = (C.c_int64 * W)(*[b.nbytes for b in bufs])
    from distml_amd import _lib
    L = _lib.load()
    assert L.dml_store_push_batch(store._h, ptrs, lens, W) == 0  # warm (staging alloc)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        assert L.dml_store_push_batch(store._h, ptrs, lens, W) == 0
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    res[kind] = {"push_batch_ms": round(t * 1e3, 2), "end_to_end_GiBps": round(algo / t / 2**30, 2),
                 "host_bytes_GBps": round(W * bench.BUCKET / t / 1e9, 2)}
# H2D alone (pinned, one 2 GiB DMA) for the per-stage split
dev = torch.empty(W * bench.BUCKET, dtype=torch.uint8, device="cuda")
src = torch.empty(W * bench.BUCKET, dtype=torch.uint8).pin_memory()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    dev.copy_(src, non_blocking=True)
torch.cuda.synchronize()
h2d = (time.perf_counter() - t0) / 3
res["h2d_pinned_GBps"] = round(W * bench.BUCKET / h2d / 1e9, 2)
del dev, src
# fetch the whole shard back (KeyRange -> [key][1024 f32] records, D2H)
t0 = time.perf_counter()
blob = store.handleFetch(fmt, KeyRange(0, bench.ROWS - 1))
tf = time.perf_counter() - t0
res["fetch_full_shard_ms"] = round(tf * 1e3, 2)
res["fetch_GBps"] = round(len(blob) / tf / 1e9, 2)
print(json.dumps(res))
