"""ctypes binding of libdistml_ps.so (include/distml_ps.h).

The HIP library is the product: there is no CPU fallback. Loading fails
loudly when the library is missing or was not built.

`torch` (when importable) is imported BEFORE the library so that one HIP
runtime serves the process: torch ships its own libamdhip64 with the same
soname, and the dynamic linker then reuses it for libdistml_ps.
"""
from __future__ import annotations

import ctypes as C
import os

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# The one shipped build, next to this file: nothing in the environment selects
# another (A/B runs of build-time variants load theirs through load(path) in scripts/).
LIB_PATH = os.path.join(_HERE, "libdistml_ps.so")
_lib = None


class dml_desc(C.Structure):
    """Mirror of DataDesc's six wire ints (DataDesc.java:62-69)."""
    _fields_ = [("data_type", C.c_int32), ("key_type", C.c_int32), ("value_type", C.c_int32),
                ("dense_row", C.c_int32), ("dense_column", C.c_int32), ("ada_grad", C.c_int32)]


class dml_store_counters(C.Structure):
    """Mirror of dml_store_counters (dml_store_stats)."""
    _fields_ = [("chunks", C.c_int64), ("spec_chunks", C.c_int64), ("spec_reruns", C.c_int64),
                ("identity_pushes", C.c_int64), ("reused_pushes", C.c_int64), ("indexed_pushes", C.c_int64),
                ("sparse_big_chunks", C.c_int64), ("sparse_replays", C.c_int64),
                ("ident_launches", C.c_int64)]


# Every symbol include/distml_ps.h declares, with its ctypes signature.
_vp, _i32, _i64, _u32, _u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
_P = C.POINTER
SIGNATURES = {
    "dml_store_create_range": (C.c_int, [_P(dml_desc), _i64, _i64, _i32, _i32, _u32, _P(_vp)]),
    "dml_store_destroy": (None, [_vp]),
    "dml_linear_split": (C.c_int, [_i64, _i64, _i32, _P(_i64), _P(_i64)]),
    "dml_store_push": (C.c_int, [_vp, _vp, _i64]),
    "dml_store_push_batch": (C.c_int, [_vp, _P(_vp), _P(_i64), _i32]),
    "dml_store_push_batch_device": (C.c_int, [_vp, _P(_vp), _P(_i64), _i32]),
    "dml_store_flush": (C.c_int, [_vp]),
    "dml_store_push_seq": (C.c_int, [_vp, _P(_u64)]),
    "dml_store_retire": (C.c_int, [_vp, _u64]),
    "dml_store_stats": (C.c_int, [_vp, _P(dml_store_counters), _i32]),
    "dml_store_error_state": (C.c_int, [_vp, _P(_i64), _P(_i32)]),
    "dml_store_clear_error": (None, [_vp]),
    "dml_store_shape": (C.c_int, [_vp, _P(_i64), _P(_i32)]),
    "dml_store_value_type": (C.c_int, [_vp, _P(_i32), _P(_i32)]),
    "dml_store_read_dense": (C.c_int, [_vp, _vp, _i64]),
    "dml_store_write_dense": (C.c_int, [_vp, _vp, _i64]),
    "dml_store_device_ptr": (C.c_int, [_vp, _P(_vp)]),
    "dml_store_read_adagrad": (C.c_int, [_vp, _vp, _vp, _i64]),
    "dml_store_read_rows": (C.c_int, [_vp, _i32, _i64, _i64, _vp, _i64]),
    "dml_store_fill": (C.c_int, [_vp, C.c_double]),
    "dml_store_set_alpha": (C.c_int, [_vp, C.c_float, C.c_float, C.c_float]),
    "dml_store_max_delta": (C.c_int, [_vp, _P(C.c_float), _P(_i32), _P(_i32)]),
    "dml_store_fetch": (C.c_int, [_vp, _P(_i64), _i64, _vp, _i64, _P(_i64)]),
    "dml_store_fetch_range": (C.c_int, [_vp, _i64, _i64, _vp, _i64, _P(_i64)]),
    "dml_store_write_all": (C.c_int, [_vp, _vp, _i64, _P(_i64)]),
    "dml_store_read_all": (C.c_int, [_vp, _vp, _i64]),
    "dml_store_sync_to": (C.c_int, [_vp, _i32, _i32, _vp, _i64, _P(_i64)]),
    "dml_store_sync_from": (C.c_int, [_vp, _i32, _i32, _vp, _i64]),
    "dml_host_alloc": (C.c_int, [_i64, _P(_vp)]),
    "dml_host_free": (None, [_vp]),
    "dml_store_stream": (C.c_int, [_vp, _P(_vp)]),
    "dml_store_set_timing": (C.c_int, [_vp, _i32]),
    "dml_store_kernel_time": (C.c_int, [_vp, _P(C.c_double), _P(_i64), _i32]),
    "dml_store_kernel_name": (C.c_int, [_vp, C.c_char_p, _i32]),
    "dml_store_apply_dense_device": (C.c_int, [_vp, _vp, _i64]),
    "dml_store_apply_adagrad_moments_device": (C.c_int, [_vp, _vp, _i64]),
    "dml_reduce_buckets_dense": (C.c_int, [_P(dml_desc), _i64, _i64, _i32, _P(_vp), _P(_i64), _i32, _vp, _vp]),
    "dml_prereduce_begin": (C.c_int, [_P(dml_desc), _i64, _i64, _i32, _P(_vp), _P(_i64), _i32, _vp, _P(_vp)]),
    "dml_prereduce_piece": (C.c_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    "dml_prereduce_end": (C.c_int, [_vp]),
    "dml_prereduce_moments_piece": (C.c_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    "dml_prereduce_stream_wait": (C.c_int, [_vp, _vp]),
    "dml_prereduce_timing": (C.c_int, [_i32]),
    "dml_prereduce_kernel_time": (C.c_int, [_P(C.c_double), _P(_i64), _i32]),
    "dml_prectx_create": (C.c_int, [_P(dml_desc), _i64, _i64, _i32, _i32, _P(_vp)]),
    "dml_prectx_destroy": (None, [_vp]),
    "dml_prectx_stats": (C.c_int, [_vp, _P(dml_store_counters), _i32]),
    "dml_prereduce_begin_ctx": (C.c_int, [_vp, _P(_vp), _P(_i64), _i32, _vp, _P(_vp)]),
    "dml_prereduce_verify": (C.c_int, [_vp, _P(_i32)]),
    "dml_shard_split": (C.c_int, [_P(dml_desc), _i32, _i64, _i32, _P(_vp), _P(_i64), _i32, _vp, _i64, _P(_i64), _vp]),
    "dml_group_unique_id": (C.c_int, [_vp, _i32]),
    "dml_group_push_exchange": (C.c_int, [_vp, _P(_vp), _P(_i64), _i32]),
    "dml_group_push_moments": (C.c_int, [_vp, _P(_vp), _P(_i64), _i32]),
    "dml_group_create": (C.c_int, [_vp, _i32, _i32, _i32, _P(dml_desc), _i64, _i32, _i32, _P(_vp)]),
    "dml_group_store": (C.c_int, [_vp, _P(_vp)]),
    "dml_group_prereduce_stats": (C.c_int, [_vp, _P(dml_store_counters), _i32]),
    "dml_group_push_full_range": (C.c_int, [_vp, _P(_vp), _P(_i64), _i32]),
    "dml_group_push_local": (C.c_int, [_vp, _P(_vp), _P(_i64), _i32]),
    "dml_group_debug_fail_verify": (C.c_int, [_vp, _i32]),
    "dml_group_flush": (C.c_int, [_vp]),
    "dml_group_destroy": (None, [_vp]),
    "dml_synth_dense_bucket": (C.c_int, [_vp, _P(dml_desc), _i64, _i64, _i64, _i32, _u64, _u64, _u64, _vp]),
    "dml_synth_sparse_bucket": (C.c_int, [_vp, _P(dml_desc), _i64, _i64, _i64, _u64, _u64, _u64, _vp]),
    "dml_synth_fill_store": (C.c_int, [_vp, _u64]),
    "dml_store_rand": (C.c_int, [_vp, _u64]),
    "dml_diag_stream": (C.c_int, [_i32, _vp, _vp, _i64, _vp, _P(C.c_float)]),
    "dml_diag_ring_rs": (C.c_int, [_i32, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp]),
    "dml_diag_rmw_floor": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _P(C.c_float)]),
    "dml_diag_gather_floor": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _i64, _vp, _P(C.c_float)]),
    "dml_diag_dense_floor": (C.c_int, [_vp, _vp, _vp, _i32, _vp, _P(C.c_float), _P(_i32)]),
    "dml_diag_store_knob": (C.c_int, [_vp, _i32, _i64]),
    "dml_last_error": (C.c_char_p, []),
    "dml_version": (C.c_char_p, []),
}

# Status codes (include/distml_ps.h)
DML_OK = 0
DML_E_BAD_DESC = 1
DML_E_KEY_OUT_OF_SHARD = 2
DML_E_TRUNCATED = 3
DML_E_NEGATIVE_COUNTER = 4
DML_E_INVALID_ARG = 16
DML_E_HIP = 17
DML_E_NOMEM = 18
DML_E_UNSUPPORTED = 19
DML_E_CAPACITY = 20

DML_FLAG_FLOAT_ARRAY_REF_STRIDE = 0x1
DML_FLAG_ASYNC = 0x2
DML_FLAG_NO_SPECULATION = 0x4


class NativeLibraryMissing(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libdistml_ps.so and bind every declared symbol (raises if absent)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} not found: build it with `make -C distml_amd/csrc` (or __graft_entry__.build())")
    L = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)  # AttributeError = a declared symbol is not exported
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _lib = L
    return L


def last_error() -> str:
    msg = load().dml_last_error()
    return msg.decode() if msg else ""
