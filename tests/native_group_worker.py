"""One rank of the native shard group (dml_group_*, distml_amd/csrc/dml_group.hip —
what the JNI's GpuShardGroup binds) in a process that never imports torch, as the
PS JVM runs it. tests/test_native_group.py starts `world` of these.

--double: dlopen tests/rccl_double/librccl_double.so with RTLD_GLOBAL before
libdistml_ps.so, so the library's nccl* calls resolve to the test-only stand-in
(ranks sharing one GPU over host shared memory; RCCL refuses two ranks per
device). Without it the ranks use the system RCCL, one GPU each.

Cases (generators shared with tests/test_gpu_group.py):
  full      CALLS full-range calls back to back (call 2: rank 0's push 0 fails the
            speculation's verification and re-runs exactly), flush
  exchange  XCALLS exact exchange calls back to back (AdaGrad or int32), flush
  moments   XCALLS two-moment AdaGrad calls, flush
  local     int32: one full-range call then, without a flush, push_local of -(its
            sum) on the rank's own rows: exact only if the store applies them in order
  fault     int32 full-range calls; rank 0's second finished call fails its verdict
            (fault injection): it raises there, every rank finishes every call
  beginfail int32 full-range calls; rank 0's call 1 hands over a ragged push, so its
            _begin_ctx fails (no pieces, no host wait for the set's last apply): it
            raises at once, contributes zeros, every rank finishes every call
  asc       CALLS full-range calls whose pushes all list the rows in ascending order
            (Java HashMap<Integer> order, config 4's case): the pre-reduce pieces take
            the all-identity kernel (k_flat_ident) where no wave straddles a row block
  jni       int32 full-range calls and a pushLocal through the JNI shim's GpuShardGroup
            entry points (integration/jni/dml_jni.cc on the mock JNIEnv of tests/jni_mock)
Writes out/<case>_<rank>.npz and prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.modules["torch"] = None  # any `import torch` now raises ImportError
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
DOUBLE = os.path.join(ROOT, "tests", "rccl_double", "librccl_double.so")

import numpy as np  # noqa: E402


class Hip:
    """hipMalloc / hipMemcpy of the HIP runtime libdistml_ps.so loaded."""

    def __init__(self, device):
        path = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln][0]
        h = C.CDLL(path)
        h.hipSetDevice.argtypes = [C.c_int]
        h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        h.hipFree.argtypes = [C.c_void_p]
        assert h.hipSetDevice(device) == 0
        self.h, self.ptrs = h, []

    def put(self, arr: np.ndarray) -> int:
        arr = np.ascontiguousarray(arr)
        p = C.c_void_p()
        assert self.h.hipMalloc(C.byref(p), max(arr.nbytes, 1)) == 0
        assert self.h.hipMemcpy(p, arr.ctypes.data, arr.nbytes, 1) == 0  # host to device
        self.ptrs.append(p.value)
        return p.value

    def free(self):
        for p in self.ptrs:
            self.h.hipFree(C.c_void_p(p))
        self.ptrs = []


def read_uid(path, rank, timeout=120.0):
    from distml_amd.group import NativeShardGroup
    if rank == 0 and not os.path.exists(path):
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(NativeShardGroup.unique_id())
        os.replace(tmp, path)
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout:
            raise TimeoutError("no unique id from rank 0")
        time.sleep(0.05)
    return open(path, "rb").read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--uid-file", required=True)
    ap.add_argument("--case", required=True)
    ap.add_argument("--vt", type=int, default=1)
    ap.add_argument("--rows", type=int, default=1000)
    ap.add_argument("--cols", type=int, default=64)
    ap.add_argument("--pushes", type=int, default=5)
    ap.add_argument("--pieces", type=int, default=1)
    ap.add_argument("--out", required=True)
    ap.add_argument("--double", action="store_true")
    a = ap.parse_args()
    dbl = C.CDLL(DOUBLE, mode=C.RTLD_GLOBAL) if a.double else None  # before libdistml_ps.so
    from distml_amd import DataDesc, _lib
    from distml_amd.group import NativeShardGroup
    import pyoracle
    import test_gpu_group as G
    _lib.load()
    H = Hip(a.device)
    uid = read_uid(a.uid_file, a.rank)
    world, rank = a.world, a.rank
    errors, res = [], {}
    if a.case in ("full", "fault", "local", "beginfail", "asc"):
        vt = 0 if a.case in ("fault", "local", "beginfail") else a.vt
        rows, cols = a.rows, a.cols
        g = NativeShardGroup(DataDesc(1, 0, vt), rows, cols, rank, world, uid, device=a.device, pieces=a.pieces)
        sh = g.shard
        g.store.load_values(G._init(vt, rows, cols)[sh.firstKey:sh.lastKey + 1])
        if a.case == "fault" and rank == 0:
            g.debug_fail_verify(2)  # call 1's verdict (finished during call 2)
        calls = 1 if a.case == "local" else G.CALLS
        for call in range(calls):
            bufs = (G._asc_buckets(pyoracle, vt, rank, a.pushes, rows, cols, call) if a.case == "asc"
                    else G._buckets(pyoracle, vt, rank, a.pushes, rows, cols, call))
            ptrs = [H.put(b) for b in bufs]
            lens = [b.nbytes for b in bufs]
            if a.case == "beginfail" and rank == 0 and call == 1:
                lens[0] -= 1  # not whole records: DML_E_TRUNCATED from _begin_ctx
            try:
                g.push_full_range(ptrs, lens)
            except Exception as e:  # the fault case: rank 0's call-1 failure, raised at call 2
                errors.append([call, type(e).__name__, str(e)[:200]])
        if a.case == "local":
            # minus everything every rank pushed for this shard's rows, plus the init: the
            # counters end at exactly 0, but go negative if applied before the full-range sum
            tot = np.zeros((rows, cols), np.int64)
            for q in range(world):
                for b in G._buckets(pyoracle, vt, q, a.pushes, rows, cols, 0):
                    rec = b.reshape(rows, 4 + 4 * cols)
                    tot[rec[:, :4].copy().view("<i4").ravel()] += rec[:, 4:].copy().view("<i4")
            tot += G._init(vt, rows, cols)
            from distml_amd import encode_matrix_push
            keys = np.arange(sh.firstKey, sh.lastKey + 1)[::-1]
            p = np.frombuffer(encode_matrix_push(keys, (-tot[keys]).astype(np.int32), 0, 0), np.uint8).copy()
            g.push_local([H.put(p)], [p.nbytes])
        try:
            g.flush()
        except Exception as e:
            errors.append(["flush", type(e).__name__, str(e)[:200]])
        res["data"] = g.store.values()
        res["stats"] = np.array([g.prereduce_stats().get(k, 0) for k in ("spec_chunks", "spec_reruns", "ident_launches")])
    elif a.case == "jni":
        # the same full-range calls driven through the JNI shim's GpuShardGroup entry points
        # (integration/jni/dml_jni.cc linked with the in-process mock JNIEnv), int32, then
        # a pushLocal of this rank's own rows; the shard comes back through nativeWriteAll
        from test_jni_shim import MockJVM
        jvm = MockJVM()
        rows, cols = a.rows, a.cols
        uid_arr = jvm.bytes_(uid)
        g, exc = jvm.call("nativeGroupCreate", uid_arr, world, rank, a.device, 1, 0, 0, 0, 1, 0, rows, cols, a.pieces)
        assert exc is None and g, exc
        from distml_amd import KeyRange
        shard = KeyRange(0, rows - 1).linearSplit(world)[rank]
        st, exc = jvm.call("nativeGroupStore", g)
        init = G._init(0, rows, cols)[shard.firstKey:shard.lastKey + 1]
        jvm.call("nativeReadAll", st, jvm.bytes_(init.astype(">i4").tobytes()))
        for call in range(G.CALLS):
            bufs = G._buckets(pyoracle, 0, rank, a.pushes, rows, cols, call)
            ptrs = [H.put(b) for b in bufs]
            _, exc = jvm.call("nativeGroupPush", g, jvm.longs(ptrs), jvm.longs([b.nbytes for b in bufs]), 0)
            if exc:
                errors.append([call, exc[0], exc[1][:200]])
        from distml_amd import encode_matrix_push
        keys = np.arange(shard.firstKey, shard.lastKey + 1)
        lp = np.frombuffer(encode_matrix_push(keys, np.full((len(keys), cols), rank + 1, np.int32), 0, 0),
                           np.uint8).copy()
        _, exc = jvm.call("nativeGroupPush", g, jvm.longs([H.put(lp)]), jvm.longs([lp.nbytes]), 3)
        assert exc is None, exc
        _, exc = jvm.call("nativeGroupFlush", g)
        assert exc is None, exc
        wa, _ = jvm.call("nativeWriteAll", st)
        res["data"] = np.frombuffer(jvm.read(wa), ">i4").astype(np.int32)
        jvm.call("nativeGroupDestroy", g)
        g = None
    elif a.case in ("exchange", "moments"):
        vt = 1 if a.case == "moments" else a.vt
        fmt = DataDesc(1, 0, vt, False, True, vt == 1)
        g = NativeShardGroup(fmt, G.XR, G.XC, rank, world, uid, device=a.device)
        sh = g.shard
        g.store.load_values(G._init(vt, G.XR, G.XC)[sh.firstKey:sh.lastKey + 1])
        if vt == 1:
            g.store.setAlpha(*G.XADA)
        for call in range(G.XCALLS):
            bufs = G._xbuckets(vt, rank, call, repeat=a.case == "exchange")
            ptrs = [H.put(b) for b in bufs]
            (g.push_exchange if a.case == "exchange" else g.push_moments)(ptrs, [b.nbytes for b in bufs])
        g.flush()
        res["data"] = g.store.values()
        if vt == 1:
            res["alpha"], res["delta"] = g.store.adagrad_state()
            res["md"] = np.array(g.store.maxDelta(), np.float64)
    else:
        raise SystemExit(f"unknown case {a.case}")
    if g is not None:
        g.close()
    H.free()
    np.savez(os.path.join(a.out, f"{a.case}_{rank}.npz"), **res)
    calls, ctas = None, None
    if dbl is not None:
        dbl.rccl_double_calls.restype = C.c_int64
        calls = int(dbl.rccl_double_calls())
        dbl.rccl_double_ctas.restype = C.c_int32
        ctas = [int(dbl.rccl_double_ctas(0)), int(dbl.rccl_double_ctas(1))]
    libs = {n: ln.split()[-1] for ln in open("/proc/self/maps") for n in ("librccl", "libdistml_ps")
            if n in ln}
    print(json.dumps({"rank": rank, "errors": errors, "double_calls": calls, "ctas": ctas, "libs": libs}), flush=True)


if __name__ == "__main__":
    main()
