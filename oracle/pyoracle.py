"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package `distml_amd`.
PARITY UNPINNED (no runnable reference, no reference fixtures): see
oracle/dml_oracle.h and DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

VALUE_DTYPE = {0: np.int32, 1: np.float32, 3: np.float64}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
        L.orc_create.restype = vp
        L.orc_create.argtypes = [i32, i32, i32, i32, i32, i64, i64, i32, i32]
        L.orc_destroy.argtypes = [vp]
        L.orc_elems.restype = i64
        L.orc_elems.argtypes = [vp]
        L.orc_data.restype = vp
        L.orc_data.argtypes = [vp]
        L.orc_alpha.restype = vp
        L.orc_alpha.argtypes = [vp]
        L.orc_delta.restype = vp
        L.orc_delta.argtypes = [vp]
        L.orc_push.restype = C.c_int
        L.orc_push.argtypes = [vp, C.c_char_p, i64]
        L.orc_push_many.restype = C.c_int
        L.orc_push_many.argtypes = [vp, C.POINTER(C.c_void_p), C.POINTER(i64), i32, i32]
        L.orc_error.restype = C.c_int
        L.orc_error.argtypes = [vp, C.POINTER(i64), C.POINTER(i32)]
        L.orc_set_alpha.argtypes = [vp, C.c_float, C.c_float, C.c_float]
        L.orc_max_delta.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(i32), C.POINTER(i32)]
        L.orc_fetch.restype = i64
        L.orc_fetch.argtypes = [vp, C.POINTER(i64), i64, vp, i64]
        L.orc_write_all.restype = i64
        L.orc_write_all.argtypes = [vp, vp, i64]
        L.orc_read_all.restype = C.c_int
        L.orc_read_all.argtypes = [vp, C.c_char_p, i64]
        L.orc_linear_split.argtypes = [i64, i64, i32, C.POINTER(i64), C.POINTER(i64)]
        L.orc_splitmix64.restype = u64
        L.orc_splitmix64.argtypes = [u64]
        L.orc_synth_dense_bucket.argtypes = [vp, i32, i32, i64, i64, i64, i32, u64, u64, u64]
        L.orc_synth_sparse_bucket.argtypes = [vp, i32, i32, i32, i64, i64, i64, u64, u64, u64]
        L.orc_synth_fill.argtypes = [vp, u64]
        L.orc_synth_dense_rows.argtypes = [vp, i32, i32, vp, i64, i32, u64]
        L.orc_synth_fill_rows.argtypes = [vp, vp, u64]
        L.orc_rand.restype = C.c_int
        L.orc_rand.argtypes = [vp]
        L.orc_java_random_ints.argtypes = [i64, i32, vp]
        L.orc_java_random_gaussians.argtypes = [i64, i32, vp]
        L.orc_fdlibm_log.restype = C.c_double
        L.orc_fdlibm_log.argtypes = [C.c_double]
        _lib = L
    return _lib


class OracleStore:
    """Sequential CPU store with the reference's handlePush semantics."""

    def __init__(self, data_type, key_type, value_type, first, last, cols=1,
                 dense_column=1, ada_grad=0, float_array_ref_stride=0):
        L = lib()
        self._h = L.orc_create(data_type, key_type, value_type, dense_column, ada_grad,
                               first, last, cols, float_array_ref_stride)
        if not self._h:
            raise ValueError("oracle rejected the store descriptor")
        self.data_type, self.key_type, self.value_type = data_type, key_type, value_type
        self.first, self.last = first, last
        self.rows = last - first + 1
        self.cols = cols if data_type == 1 else 1
        self.ada_grad = ada_grad and data_type == 1 and value_type == 1

    def close(self):
        if self._h:
            lib().orc_destroy(self._h)
            self._h = None

    __del__ = close

    def _view(self, ptr, dtype):
        n = self.rows * self.cols
        buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
        return np.frombuffer(buf, dtype=dtype).reshape(self.rows, self.cols)

    @property
    def data(self) -> np.ndarray:
        return self._view(lib().orc_data(self._h), VALUE_DTYPE[self.value_type])

    @property
    def alpha(self) -> np.ndarray:
        return self._view(lib().orc_alpha(self._h), np.float32)

    @property
    def delta(self) -> np.ndarray:
        return self._view(lib().orc_delta(self._h), np.float32)

    def push(self, data: bytes) -> int:
        data = bytes(data)
        return lib().orc_push(self._h, data, len(data))

    def push_many(self, bufs, threads=1) -> int:
        """bufs: list of numpy uint8 arrays (kept alive by the caller)."""
        n = len(bufs)
        ptrs = (C.c_void_p * n)(*[b.ctypes.data for b in bufs])
        lens = (C.c_int64 * n)(*[b.nbytes for b in bufs])
        return lib().orc_push_many(self._h, ptrs, lens, n, threads)

    def error(self):
        k, c = C.c_int64(), C.c_int32()
        code = lib().orc_error(self._h, C.byref(k), C.byref(c))
        return code, k.value, c.value

    def set_alpha(self, initial, minimum, factor):
        lib().orc_set_alpha(self._h, initial, minimum, factor)

    def max_delta(self):
        v, r, c = C.c_float(), C.c_int32(), C.c_int32()
        lib().orc_max_delta(self._h, C.byref(v), C.byref(r), C.byref(c))
        return v.value, r.value, c.value

    def fetch(self, keys) -> bytes:
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        cap = max(1, len(keys) * (8 + 16 * self.cols))
        out = np.zeros(cap, np.uint8)
        n = lib().orc_fetch(self._h, keys.ctypes.data_as(C.POINTER(C.c_int64)), len(keys),
                            out.ctypes.data, cap)
        if n < 0:
            raise IndexError("fetch key outside shard")
        return out[:n].tobytes()

    def write_all(self) -> bytes:
        cap = self.rows * self.cols * 8
        out = np.zeros(max(cap, 1), np.uint8)
        n = lib().orc_write_all(self._h, out.ctypes.data, cap)
        return out[:n].tobytes()

    def read_all(self, data: bytes) -> int:
        return lib().orc_read_all(self._h, bytes(data), len(data))

    def synth_fill(self, seed):
        lib().orc_synth_fill(self._h, seed)

    def synth_fill_rows(self, rows, seed):
        """orc_synth_fill's values of `rows` of a self.cols-wide store, as rows 0..n-1."""
        r = np.ascontiguousarray(rows, np.int64)
        assert len(r) == self.rows
        lib().orc_synth_fill_rows(self._h, r.ctypes.data, seed)

    def rand(self) -> int:
        """DoubleMatrixStore.rand() (DoubleMatrixStore.java:192-207), bit-exact."""
        return lib().orc_rand(self._h)


def java_random_ints(seed, n) -> np.ndarray:
    """new java.util.Random(seed).nextInt() x n."""
    out = np.empty(n, np.int32)
    lib().orc_java_random_ints(seed, n, out.ctypes.data)
    return out


def java_random_gaussians(seed, n) -> np.ndarray:
    """new java.util.Random(seed).nextGaussian() x n (StrictMath = fdlibm log)."""
    out = np.empty(n, np.float64)
    lib().orc_java_random_gaussians(seed, n, out.ctypes.data)
    return out


def fdlibm_log(x: float) -> float:
    return lib().orc_fdlibm_log(x)


def linear_split(first, last, n):
    f = (C.c_int64 * n)()
    l = (C.c_int64 * n)()
    lib().orc_linear_split(first, last, n, f, l)
    return [(f[i], l[i]) for i in range(n)]


def splitmix64(x):
    return lib().orc_splitmix64(x & 0xFFFFFFFFFFFFFFFF)


def synth_dense_bucket(key_type, value_type, first_key, shard_rows, nrec, cols, seed,
                       perm_a=1, perm_c=0) -> np.ndarray:
    K = 4 if key_type == 0 else 8
    V = 8 if value_type == 3 else 4
    out = np.empty(nrec * (K + V * cols), np.uint8)
    lib().orc_synth_dense_bucket(out.ctypes.data, key_type, value_type, first_key, shard_rows,
                                 nrec, cols, seed, perm_a, perm_c)
    return out


def synth_dense_rows(key_type, value_type, rows, cols, seed) -> np.ndarray:
    """The records synth_dense_bucket holds for `rows` (any push order), keyed 0..n-1."""
    r = np.ascontiguousarray(rows, np.int64)
    K = 4 if key_type == 0 else 8
    V = 8 if value_type == 3 else 4
    out = np.empty(len(r) * (K + V * cols), np.uint8)
    lib().orc_synth_dense_rows(out.ctypes.data, key_type, value_type, r.ctypes.data, len(r), cols, seed)
    return out


def synth_sparse_bucket(key_type, value_type, first_key, key_space, nrec, seed,
                        perm_a=1, perm_c=0, value_stride=None) -> np.ndarray:
    K = 4 if key_type == 0 else 8
    if value_stride is None:
        value_stride = 8 if value_type == 3 else 4
    out = np.empty(nrec * (K + value_stride), np.uint8)
    lib().orc_synth_sparse_bucket(out.ctypes.data, key_type, value_type, value_stride, first_key,
                                  key_space, nrec, seed, perm_a, perm_c)
    return out
