"""The JNI shim (integration/jni/dml_jni.cc) compiles: there is no JDK in this image,
so it is checked with g++ -fsyntax-only against tests/jni_stub/jni.h (the JNI
types and JNIEnv members it uses, JNI-spec signatures) and the real
include/distml_ps.h. Also: the shim's native methods are the ones
GpuDataStore.java / GpuShardGroup.java declare, and nativePush copies the
byte[] (GetByteArrayRegion) instead of holding a critical section across the
GPU apply. And the shim RUNS: linked with tests/jni_mock/mock_jvm.cc
(an in-process JNIEnv), its Java_* entry points are called as GpuDataStore.java /
GpuShardGroup.java would call them — exception mapping on the CPU, and on the GPU a
store driven only through JNI, bytes-equal against the oracle."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "integration", "jni")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_shim_compiles():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        os.path.join(JNI, "dml_jni.cc")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_native_methods_match():
    cc = open(os.path.join(JNI, "dml_jni.cc")).read()
    for cls, macro in (("GpuDataStore", "FN"), ("GpuShardGroup", "GFN")):
        java = open(os.path.join(JNI, cls + ".java")).read()
        declared = set(re.findall(r"native\s+[\w.\[\]]+\s+(\w+)\s*\(", java))
        defined = set(re.findall(r"\b" + macro + r"\((\w+)\)", cc)) - {"name"}  # the macro definitions
        assert declared == defined, (cls, declared ^ defined)


def test_push_does_not_pin_across_the_apply():
    cc = open(os.path.join(JNI, "dml_jni.cc")).read()
    assert "GetPrimitiveArrayCritical" not in cc


# ---- the shim RUN through an in-process mock JNIEnv (tests/jni_mock) -----------
class MockJVM:
    """integration/jni/dml_jni.cc linked with tests/jni_mock/mock_jvm.cc: the Java_*
    entry points called as the JVM calls them (JNIEnv*, jclass, args...), with Java
    byte[] / long[] / DirectByteBuffer objects from the mock."""

    def __init__(self):
        import ctypes as C
        sys.path.insert(0, ROOT)
        from distml_amd import _lib
        _lib.load()  # the product library first (and with it the HIP runtime the tests use)
        path = os.path.join(ROOT, "tests", "jni_mock", "libdml_jni_mock.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", os.path.dirname(path)], check=True)
        self.C = C
        L = self.L = C.CDLL(path)
        P, I, J, F, D = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_double
        L.mock_env.restype = P
        for n, a, r in [("mock_byte_array", [P, I], P), ("mock_long_array", [P, I], P),
                        ("mock_array_length", [P], I), ("mock_array_data", [P], P),
                        ("mock_direct_address", [P], P), ("mock_direct_capacity", [P], J), ("mock_free", [P], None),
                        ("mock_take_exception", [P, I, P, I], I), ("mock_calls", [], I),
                        ("mock_prim_array", [C.c_char, I], P), ("mock_object_array", [P, I], P),
                        ("mock_object_element", [P, I], P)]:
            getattr(L, n).argtypes, getattr(L, n).restype = a, r
        self.env = L.mock_env()
        sig = {
            "nativeCreate": ([I, I, I, I, I, I, J, J, I, I, I], J), "nativePush": ([J, P], None),
            "nativeRand": ([J, J], None), "nativeFetch": ([J, P], P), "nativeFetchRange": ([J, J, J], P),
            "nativeShardBytes": ([J], J), "nativeWriteAll": ([J], P), "nativeReadAll": ([J, P], None),
            "nativeSyncTo": ([J, I, I], P), "nativeSyncFrom": ([J, I, I, P], None), "nativeHostAlloc": ([J], P),
            "nativeHostFree": ([P], None), "nativePushDirect": ([J, P, I, I], None), "nativeFill": ([J, D], None),
            "nativeSetAlpha": ([J, F, F, F], None), "nativeDestroy": ([J], None),
            "nativeSnapshot": ([J, I, I, I, P], None), "nativeMaxDelta": ([J, P], F),
        }
        gsig = {
            "nativeUniqueId": ([], P), "nativeGroupCreate": ([P, I, I, I, I, I, I, I, I, I, J, I, I], J),
            "nativeGroupPush": ([J, P, P, I], None), "nativeGroupFlush": ([J], None),
            "nativeGroupStore": ([J], J), "nativeGroupDestroy": ([J], None),
        }
        self.fn = {}
        for cls, table in (("GpuDataStore", sig), ("GpuShardGroup", gsig)):
            for name, (args, res) in table.items():
                f = getattr(L, f"Java_com_intel_distml_util_store_{cls}_{name}")
                f.argtypes, f.restype = [P, P] + args, res
                self.fn[name] = f

    def call(self, name, *args):
        """Call a native method; returns (result, (exception class, message) or None)."""
        r = self.fn[name](self.env, None, *args)
        cls, msg = self.C.create_string_buffer(256), self.C.create_string_buffer(1024)
        exc = (cls.value.decode(), msg.value.decode()) if self.L.mock_take_exception(cls, 256, msg, 1024) else None
        return r, exc

    def bytes_(self, data: bytes):
        return self.L.mock_byte_array(data, len(data))

    def longs(self, vals):
        arr = (self.C.c_int64 * max(len(vals), 1))(*vals)
        return self.L.mock_long_array(arr, len(vals))

    def read(self, arr) -> bytes:
        n = self.L.mock_array_length(arr)
        return self.C.string_at(self.L.mock_array_data(arr), n) if n > 0 else b""

    def prim(self, kind: str, n: int):
        """A Java float[] / int[] / double[] ('F' / 'I' / 'D') of n zeros."""
        return self.L.mock_prim_array(kind.encode(), n)

    def matrix(self, kind: str, rows: int, cols: int):
        """A Java T[rows][cols] (an Object[] of T[] rows), as `new float[rows][cols]`."""
        elems = (self.C.c_void_p * max(rows, 1))(*[self.prim(kind, cols) for _ in range(rows)])
        return self.L.mock_object_array(elems, rows)

    def read_prim(self, arr, dtype):
        import numpy as np
        n = self.L.mock_array_length(arr)
        return np.frombuffer(self.C.string_at(self.L.mock_array_data(arr), n * np.dtype(dtype).itemsize), dtype)

    def read_matrix(self, arr, dtype):
        import numpy as np
        return np.stack([self.read_prim(self.L.mock_object_element(arr, i), dtype)
                         for i in range(self.L.mock_array_length(arr))])


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_mock_jvm_exception_mapping_cpu():
    """Runs the shim's create entry points without a GPU: DataStore.createStore's
    IllegalArgumentException for an unknown matrix type (DataStore.java:91), a
    RuntimeException for what the library does not support or cannot do (sparse-
    column matrices; no HIP device here), GpuShardGroup's id-length check."""
    import torch
    jvm = MockJVM()
    _, exc = jvm.call("nativeCreate", 7, 0, 1, 0, 1, 0, 0, 99, 4, 0, 0)  # data type 7
    assert exc and exc[0] == "java/lang/IllegalArgumentException" and "Unrecognized" in exc[1]
    _, exc = jvm.call("nativeCreate", 1, 0, 1, 0, 0, 0, 0, 99, 4, 0, 0)  # sparse-column matrix
    assert exc and exc[0] == "java/lang/RuntimeException"
    if not torch.cuda.is_available():
        h, exc = jvm.call("nativeCreate", 1, 0, 1, 0, 1, 0, 0, 99, 4, 0, 0)
        assert h == 0 and exc and exc[0] == "java/lang/RuntimeException" and "device" in exc[1]
    short = jvm.bytes_(b"\0" * 64)
    _, exc = jvm.call("nativeGroupCreate", short, 1, 0, 0, 1, 0, 1, 0, 1, 0, 100, 8, 1)
    assert exc == ("java/lang/IllegalArgumentException", "unique id must be 128 bytes")
    jvm.L.mock_free(short)
    assert jvm.L.mock_calls() > 0


@pytest.mark.gpu
def test_mock_jvm_store_on_gpu(oracle):
    """A FloatMatrixStore and an IntMatrixStore on cuda:0 driven only through the JNI
    shim's entry points, as GpuDataStore.java calls them: readAll of the oracle's
    writeAll bytes, byte[] pushes (PSAgent.handle, PSAgent.java:278-281), a push from
    a pinned DirectByteBuffer (nativeHostAlloc + nativePushDirect), fetch by keys and
    by range, writeAll; a key outside the shard (ArrayIndexOutOfBoundsException) and a
    negative counter (IllegalStateException, IntMatrixStore.java:174-176) leave the
    state the reference's store leaves. Then the native group at world 1 (unique id,
    create, two full-range device pushes, flush, its store's writeAll). Every result
    bytes-equal against the oracle."""
    import ctypes as C

    import numpy as np
    import torch
    from distml_amd import encode_matrix_push
    jvm = MockJVM()
    rng = np.random.default_rng(31)
    rows, cols = 1000, 64
    h, exc = jvm.call("nativeCreate", 1, 0, 1, 0, 1, 0, 0, rows - 1, cols, 0, 0)
    assert exc is None and h
    o = oracle.OracleStore(1, 0, 1, 0, rows - 1, cols)
    o.synth_fill(3)
    _, exc = jvm.call("nativeReadAll", h, jvm.bytes_(o.write_all()))
    assert exc is None
    n, _ = jvm.call("nativeShardBytes", h)
    assert n == len(o.write_all())
    for b in range(6):
        keys = rng.permutation(rows)[: rows - 37 * b]
        p = encode_matrix_push(keys, (rng.standard_normal((len(keys), cols)) * 0.01).astype(np.float32), 0, 1)
        _, exc = jvm.call("nativePush", h, jvm.bytes_(p))
        assert exc is None and o.push(p) == 0
    # a push the NIO channel read straight into pinned memory
    keys = rng.permutation(rows)[:300]
    p = encode_matrix_push(keys, (rng.standard_normal((300, cols)) * 0.01).astype(np.float32), 0, 1)
    buf, exc = jvm.call("nativeHostAlloc", len(p) + 64)
    assert exc is None and jvm.L.mock_direct_capacity(buf) == len(p) + 64
    C.memmove(jvm.L.mock_direct_address(buf) + 64, p, len(p))
    _, exc = jvm.call("nativePushDirect", h, buf, 64, len(p))
    assert exc is None and o.push(p) == 0
    jvm.call("nativeHostFree", buf)
    wa, exc = jvm.call("nativeWriteAll", h)
    assert exc is None and jvm.read(wa) == o.write_all()
    ks = [5, 999, 0, 500, 42]
    fa, exc = jvm.call("nativeFetch", h, jvm.longs(ks))
    assert exc is None and jvm.read(fa) == o.fetch(ks)
    fr, exc = jvm.call("nativeFetchRange", h, 10, 20)
    assert exc is None and jvm.read(fr) == o.fetch(list(range(10, 21)))
    # a key outside the shard: the adds before it stay, the store refuses later pushes
    keys = np.array([3, 4, rows + 5, 6])
    p = encode_matrix_push(keys, np.ones((4, cols), np.float32), 0, 1)
    _, exc = jvm.call("nativePush", h, jvm.bytes_(p))
    assert exc and exc[0] == "java/lang/ArrayIndexOutOfBoundsException"
    assert o.push(p) != 0
    wa, _ = jvm.call("nativeWriteAll", h)
    assert jvm.read(wa) == o.write_all()
    jvm.call("nativeDestroy", h)

    # IntMatrixStore: a counter below zero throws after the add (the add stays)
    hi, exc = jvm.call("nativeCreate", 1, 0, 0, 0, 1, 0, 0, 99, 8, 0, 0)
    assert exc is None
    oi = oracle.OracleStore(1, 0, 0, 0, 99, 8)
    oi.synth_fill(4)
    jvm.call("nativeReadAll", hi, jvm.bytes_(oi.write_all()))
    vals = rng.integers(-2, 3, size=(100, 8)).astype(np.int32)
    vals[37, 5] = -1000
    p = encode_matrix_push(rng.permutation(100), vals, 0, 0)
    _, exc = jvm.call("nativePush", hi, jvm.bytes_(p))
    assert exc and exc[0] == "java/lang/IllegalStateException"
    assert oi.push(p) != 0
    wa, _ = jvm.call("nativeWriteAll", hi)
    assert jvm.read(wa) == oi.write_all()
    jvm.call("nativeDestroy", hi)

    # GpuShardGroup at world 1: device-resident full-range int32 pushes (exact)
    uid, exc = jvm.call("nativeUniqueId")
    assert exc is None and jvm.L.mock_array_length(uid) == 128
    g, exc = jvm.call("nativeGroupCreate", uid, 1, 0, 0, 1, 0, 0, 0, 1, 0, rows, cols, 1)
    assert exc is None and g
    og = oracle.OracleStore(1, 0, 0, 0, rows - 1, cols)
    dev = []
    for b in range(4):
        p = encode_matrix_push(rng.permutation(rows), rng.integers(0, 3, size=(rows, cols)).astype(np.int32), 0, 0)
        assert og.push(p) == 0
        dev.append(torch.frombuffer(bytearray(p), dtype=torch.uint8).cuda())
    torch.cuda.synchronize()
    for pair in (dev[:2], dev[2:]):
        _, exc = jvm.call("nativeGroupPush", g, jvm.longs([t.data_ptr() for t in pair]),
                          jvm.longs([t.numel() for t in pair]), 0)
        assert exc is None
    # pushLocal (mode 3) right behind the full-range calls: applied after them, in order
    p = encode_matrix_push(rng.permutation(rows)[:rows // 2], rng.integers(0, 3, size=(rows // 2, cols)).astype(np.int32),
                           0, 0)
    assert og.push(p) == 0
    dl = torch.frombuffer(bytearray(p), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    _, exc = jvm.call("nativeGroupPush", g, jvm.longs([dl.data_ptr()]), jvm.longs([dl.numel()]), 3)
    assert exc is None
    # an unknown mode is refused with a Java exception (DML_E_INVALID_ARG)
    _, exc = jvm.call("nativeGroupPush", g, jvm.longs([dl.data_ptr()]), jvm.longs([dl.numel()]), 9)
    assert exc is not None
    _, exc = jvm.call("nativeGroupFlush", g)
    assert exc is None
    st, exc = jvm.call("nativeGroupStore", g)
    assert exc is None and st
    wa, _ = jvm.call("nativeWriteAll", st)
    assert jvm.read(wa) == og.write_all()
    jvm.call("nativeGroupDestroy", g)


@pytest.mark.gpu
def test_mock_jvm_snapshot_on_gpu(oracle):
    """The result-collect entry points through the shim, as the typed
    GPU stores call them: GpuDoubleArrayStore.iter() (LogisticRegression.scala:290-291)
    and GpuFloatMatrixStoreAdaGrad.iter() (Word2Vec.scala:814-817) fill the parent's
    localData (and alpha / delta, which the AdaGrad Iter prints) with nativeSnapshot,
    in bounded row chunks; the AdaGrad push reports maxDelta through nativeMaxDelta
    (FloatMatrixStoreAdaGrad.java:246). Keys and values bit-exact against the oracle.
    Also an IntMatrixStore snapshot (int[][]), a wrong-shape array and arrays of
    another element type than the store's (IllegalArgumentException), and a fetch past the Java array limit (OutOfMemoryError)."""
    import numpy as np
    from distml_amd import encode_array_push, encode_matrix_push
    jvm = MockJVM()
    rng = np.random.default_rng(41)

    # DoubleArrayStore shard [1000, 1999] (LR weights): sparse pushes with repeats
    first, n = 1000, 1000
    h, exc = jvm.call("nativeCreate", 0, 1, 3, 0, 1, 0, first, first + n - 1, 1, 0, 0)
    assert exc is None and h
    o = oracle.OracleStore(0, 1, 3, first, first + n - 1)
    for b in range(5):
        keys = rng.integers(first, first + n, size=700)
        p = encode_array_push(keys, rng.standard_normal(700), 1, 3)
        _, exc = jvm.call("nativePush", h, jvm.bytes_(p))
        assert exc is None and o.push(p) == 0
    arr = jvm.prim("D", n)  # DoubleArrayStore.localData = new double[rows]
    _, exc = jvm.call("nativeSnapshot", h, 0, 3, 1, arr)
    assert exc is None
    got = jvm.read_prim(arr, np.float64)
    assert got.tobytes() == o.data.reshape(-1).tobytes()
    # the Iter's (key, value) pairs: key = firstKey + p (keyOf), value = localData[p]
    pairs = [(first + i, float(v)) for i, v in enumerate(got)]
    assert pairs[0][0] == first and pairs[-1][0] == first + n - 1
    bad = jvm.prim("D", n - 1)
    _, exc = jvm.call("nativeSnapshot", h, 0, 3, 1, bad)
    assert exc and exc[0] == "java/lang/IllegalArgumentException"
    # an array of another element type than the store's, and the AdaGrad
    # side arrays on a store without them: refused, nothing written
    for which, elem in ((0, 1), (0, 0), (1, 1), (2, 1)):
        _, exc = jvm.call("nativeSnapshot", h, which, elem, 1, jvm.prim("F" if elem == 1 else "I", n))
        assert exc and exc[0] == "java/lang/IllegalArgumentException", (which, elem, exc)
    jvm.call("nativeDestroy", h)

    # FloatMatrixStoreAdaGrad shard (Word2Vec syn0): rows 0..2999 x 100, two pushes
    rows, cols = 3000, 100
    h, exc = jvm.call("nativeCreate", 1, 0, 1, 0, 1, 1, 0, rows - 1, cols, 0, 0)
    assert exc is None and h
    o = oracle.OracleStore(1, 0, 1, 0, rows - 1, cols, 1, 1)
    _, exc = jvm.call("nativeSetAlpha", h, 0.025, 0.0001, 1.5)
    o.set_alpha(0.025, 0.0001, 1.5)
    for b in range(2):
        keys = rng.permutation(rows)[:2500]
        p = encode_matrix_push(keys, rng.standard_normal((2500, cols)).astype(np.float32), 0, 1)
        _, exc = jvm.call("nativePush", h, jvm.bytes_(p))
        assert exc is None and o.push(p) == 0
        rc = jvm.prim("I", 2)
        v, exc = jvm.call("nativeMaxDelta", h, rc)
        assert exc is None
        assert (np.float32(v), *jvm.read_prim(rc, np.int32).tolist()) == tuple(o.max_delta())
    for which, want in ((0, o.data), (1, o.alpha), (2, o.delta)):
        m = jvm.matrix("F", rows, cols)  # new float[rows][rowSize]
        _, exc = jvm.call("nativeSnapshot", h, which, 1, 2, m)
        assert exc is None, exc
        assert jvm.read_matrix(m, np.float32).tobytes() == np.ascontiguousarray(want).tobytes(), which
        jvm.L.mock_free(m)
    m = jvm.matrix("D", rows, cols)  # alpha / delta are float, whatever array is passed
    _, exc = jvm.call("nativeSnapshot", h, 1, 3, 2, m)
    assert exc and exc[0] == "java/lang/IllegalArgumentException", exc
    jvm.L.mock_free(m)
    jvm.call("nativeDestroy", h)

    # IntMatrixStore: int[][], and rows large enough to take several 16 MiB chunks
    rows, cols = 40000, 256
    h, exc = jvm.call("nativeCreate", 1, 0, 0, 0, 1, 0, 0, rows - 1, cols, 0, 0)
    assert exc is None
    o = oracle.OracleStore(1, 0, 0, 0, rows - 1, cols)
    p = encode_matrix_push(rng.permutation(rows), rng.integers(0, 5, size=(rows, cols)).astype(np.int32), 0, 0)
    _, exc = jvm.call("nativePush", h, jvm.bytes_(p))
    assert exc is None and o.push(p) == 0
    m = jvm.matrix("I", rows, cols)
    _, exc = jvm.call("nativeSnapshot", h, 0, 0, 2, m)
    assert exc is None
    assert jvm.read_matrix(m, np.int32).tobytes() == o.data.tobytes()
    jvm.L.mock_free(m)
    # a fetch whose byte[] would pass the JVM's array limit: OutOfMemoryError, as `new byte[n]`
    _, exc = jvm.call("nativeFetchRange", h, 0, rows - 1)
    assert exc is None
    jvm.call("nativeDestroy", h)
    rows, cols = 3_000_000, 180  # 3 M x (8 + 16 x 180) B > 2^31
    h, exc = jvm.call("nativeCreate", 1, 0, 0, 0, 1, 0, 0, rows - 1, cols, 0, 0)
    assert exc is None
    _, exc = jvm.call("nativeFetchRange", h, 0, rows - 1)
    assert exc and exc[0] == "java/lang/OutOfMemoryError"
    jvm.call("nativeDestroy", h)
