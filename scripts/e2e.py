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
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from distml_amd import DataDesc, DataStore, KeyRange, _lib  # noqa: E402

fmt = DataDesc(1, 0, 1)
W = bench.W
# the same synthetic pushes as bench.py, generated on the GPU and copied to host memory
host = [t.cpu().numpy() for t in bench.make_buckets(_lib.load(), torch, fmt, W, bench.ROWS)]
torch.cuda.empty_cache()
algo = W * bench.BUCKET + 2 * bench.SHARD
res = {}
store = DataStore(fmt, KeyRange(0, bench.ROWS - 1), bench.COLS)
store.synth_fill(7)
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
# fetch / checkpoint through the C-ABI (as the JNI shim calls it), pageable and pinned host buffers
from distml_amd import pinned_empty  # noqa: E402

L = _lib.load()
rec_bytes = bench.ROWS * (4 + 4 * bench.COLS)
shard_bytes = bench.SHARD


def best_ms(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


ln = C.c_int64()
for kind in ("pageable", "pinned"):
    fout = np.empty(rec_bytes, np.uint8) if kind == "pageable" else pinned_empty(rec_bytes)
    cout = np.empty(shard_bytes, np.uint8) if kind == "pageable" else pinned_empty(shard_bytes)
    t = best_ms(lambda: L.dml_store_fetch_range(store._h, 0, bench.ROWS - 1, fout.ctypes.data, rec_bytes,
                                                C.byref(ln)))
    res[f"fetch_range_full_shard_{kind}"] = {"ms": round(t, 3), "GBps": round(rec_bytes / t / 1e6, 2)}
    t = best_ms(lambda: L.dml_store_write_all(store._h, cout.ctypes.data, shard_bytes, C.byref(ln)))
    res[f"write_all_{kind}"] = {"ms": round(t, 3), "GBps": round(shard_bytes / t / 1e6, 2)}
    t = best_ms(lambda: L.dml_store_read_all(store._h, cout.ctypes.data, shard_bytes))
    res[f"read_all_{kind}"] = {"ms": round(t, 3), "GBps": round(shard_bytes / t / 1e6, 2)}
# random-key fetch: 4096 keys
keys = np.random.default_rng(1).integers(0, bench.ROWS, 4096).astype(np.int64)
kout = pinned_empty(4096 * (4 + 4 * bench.COLS))
t = best_ms(lambda: L.dml_store_fetch(store._h, keys.ctypes.data_as(C.POINTER(C.c_int64)), len(keys),
                                      kout.ctypes.data, kout.nbytes, C.byref(ln)))
res["fetch_4096_random_keys_pinned"] = {"ms": round(t, 3), "GBps": round(kout.nbytes / t / 1e6, 2)}
# Python mirror (adds the bytes object the Java-style API returns)
t0 = time.perf_counter()
blob = store.handleFetch(fmt, KeyRange(0, bench.ROWS - 1))
tf = time.perf_counter() - t0
res["handleFetch_python_bytes_ms"] = round(tf * 1e3, 2)
print(json.dumps(res))
