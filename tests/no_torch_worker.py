"""Runs in a fresh process that never imports torch (tests/test_gpu_runtime.py):
the C-ABI on the system ROCm runtime (/opt/rocm libamdhip64 + librccl, the
libraries the JNI deployment's libdistml_ps.so loads), not torch's bundled ones.

1. A config-2 batch: 32 pushes x 64 MiB from host memory through
   dml_store_push_batch into a 16 384 x 1 024 fp32 shard, bit-exact against the
   oracle (FloatMatrixStore.java:200-222).
2. dml_group_* at world 1 (the native RCCL communicator): int32 full-range pushes
   over device buffers from hipMalloc, two calls + flush, exact against the oracle.
Prints one JSON line with the runtime libraries the process mapped.
"""
import ctypes as C
import json
import os
import sys

sys.modules["torch"] = None  # any `import torch` now raises ImportError
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
from distml_amd import DataDesc, DataStore, KeyRange, _lib  # noqa: E402
from distml_amd.group import NativeShardGroup  # noqa: E402


def hip():
    # the HIP runtime libdistml_ps.so itself loaded (its rpath: /opt/rocm/lib)
    h = C.CDLL(mapped(["libamdhip64"])["libamdhip64"])
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipFree.argtypes = [C.c_void_p]
    h.hipDeviceSynchronize.argtypes = []
    return h


def config2_batch():
    rows, cols, W = 16384, 1024, 32
    fmt = DataDesc(1, 0, 1)
    s = DataStore(fmt, KeyRange(0, rows - 1), cols)
    s.synth_fill(7)
    perms = [(1, 0) if b % 2 == 0 else (((2 * b + 1) * 2654435761) % rows | 1, (b * 7919) % rows) for b in range(W)]
    host = [pyoracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 1000 + b, *perms[b]) for b in range(W)]
    s.handlePushBatch(fmt, host)
    got = s.values()
    s.close()
    o = pyoracle.OracleStore(1, 0, 1, 0, rows - 1, cols)
    o.synth_fill(7)
    assert o.push_many(host, threads=8) == 0
    assert got.tobytes() == o.data.tobytes(), "config-2 batch differs from the oracle"


def native_group_world1():
    H = hip()
    rows, cols, W = 1000, 256, 6
    fmt = DataDesc(1, 0, 0)
    pas = [1, 3, 7, 9, 11, 13]
    host = [pyoracle.synth_dense_bucket(0, 0, 0, rows, rows, cols, 70 + b, pas[b], 3 * b) for b in range(W)]
    dev = []
    for h in host:
        p = C.c_void_p()
        assert H.hipMalloc(C.byref(p), h.nbytes) == 0
        assert H.hipMemcpy(p, h.ctypes.data, h.nbytes, 1) == 0  # hipMemcpyHostToDevice
        dev.append(p.value)
    g = NativeShardGroup(fmt, rows, cols, 0, 1, NativeShardGroup.unique_id(), device=0)
    try:
        g.store.synth_fill(3)
        g.push_full_range(dev[:3], [h.nbytes for h in host[:3]])
        g.push_full_range(dev[3:], [h.nbytes for h in host[3:]])
        g.flush()
        got = g.store.values()
    finally:
        g.close()
        for p in dev:
            H.hipFree(C.c_void_p(p))
    o = pyoracle.OracleStore(1, 0, 0, 0, rows - 1, cols)
    o.synth_fill(3)
    for h in host:
        assert o.push(h) == 0
    assert np.array_equal(got, o.data), "native group differs from the oracle"


def mapped(names):
    out = {}
    for ln in open("/proc/self/maps"):
        for n in names:
            if n in ln and n not in out:
                out[n] = ln.split()[-1]
    return out


if __name__ == "__main__":
    _lib.load()
    assert _lib.torch is None and "torch" not in [m.split(".")[0] for m in sys.modules if sys.modules[m] is not None]
    config2_batch()
    native_group_world1()
    print(json.dumps({"ok": True, "libs": mapped(["libamdhip64", "librccl", "libdistml_ps"])}), flush=True)
