"""Host mirror of DistML's server-store plugin interface over the HIP C-ABI.

`DataStore` mirrors `abstract class DataStore` (src/main/java/com/intel/distml/
util/DataStore.java:17-92): same method names, argument meaning and exception
behaviour, so code written against the reference's store reads the same here.
Every method routes to libdistml_ps (HBM-resident shard, HIP kernels); there
is no CPU fallback.

Exceptions mirror the Java ones the reference throws out of handlePush:
  IllegalStateException          negative int32 counter (IntMatrixStore.java:174-176)
  ArrayIndexOutOfBoundsException key outside the shard / truncated push
  IllegalArgumentException       unknown store type (DataStore.java:91)
"""
from __future__ import annotations

import ctypes as C
import re
import struct
import weakref
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (DML_E_BAD_DESC, DML_E_KEY_OUT_OF_SHARD, DML_E_NEGATIVE_COUNTER, DML_E_TRUNCATED,
                   DML_FLAG_ASYNC, DML_FLAG_FLOAT_ARRAY_REF_STRIDE, DML_OK)
from .datadesc import ALL, DataDesc, KeyCollection, KeyList, KeyRange

VALUE_DTYPE = {DataDesc.ELEMENT_TYPE_INT: np.int32, DataDesc.ELEMENT_TYPE_FLOAT: np.float32,
               DataDesc.ELEMENT_TYPE_DOUBLE: np.float64}


class DistMLException(Exception):
    """Base of the mirrored Java exceptions; carries the C-ABI status and position."""

    def __init__(self, msg, code=0, key=0, col=-1):
        super().__init__(msg)
        self.code, self.key, self.col = code, key, col


class IllegalStateException(DistMLException):
    pass


class ArrayIndexOutOfBoundsException(DistMLException):
    pass


class IllegalArgumentException(DistMLException):
    pass


class NativeError(DistMLException):
    pass


_EXC = {DML_E_NEGATIVE_COUNTER: IllegalStateException, DML_E_KEY_OUT_OF_SHARD: ArrayIndexOutOfBoundsException,
        DML_E_TRUNCATED: ArrayIndexOutOfBoundsException, DML_E_BAD_DESC: IllegalArgumentException}


def check(rc: int, store: Optional["DataStore"] = None):
    if rc == DML_OK:
        return
    key, col = 0, -1
    if store is not None and store._h and rc in _EXC:
        k, c = C.c_int64(), C.c_int32()
        _lib.load().dml_store_error_state(store._h, C.byref(k), C.byref(c))
        key, col = k.value, c.value
    raise _EXC.get(rc, NativeError)(_lib.last_error() or f"distml_ps status {rc}", rc, key, col)


def java_parse_float(text: str) -> float:
    """Float.parseFloat: the decimal (or hex) string rounded ONCE to the nearest
    float32, ties to even — not through a double, whose second rounding can differ.
    Leading/trailing whitespace and a trailing f/F/d/D are accepted, like Java's."""
    from fractions import Fraction
    t = text.strip(" \t\n\r\x0b\x0c\x00")
    if t[-1:] in ("f", "F", "d", "D") and not t.lower().endswith(("infinity", "nan")):
        t = t[:-1]
    body = t.lstrip("+-")
    neg = t.startswith("-")
    if body in ("NaN", "Infinity"):
        v = float("nan") if body == "NaN" else float("inf")
        return -v if neg else v
    if body.lower().startswith("0x"):
        exact = Fraction(float.fromhex(t)) if "p" in body.lower() else None
        if exact is None:
            raise ValueError(f"NumberFormatException: {text!r}")
    else:
        # Java's FloatingDecimal grammar: digits, one '.', an exponent — not Python's
        # Fraction extras ('1/2', '_' separators)
        if not re.fullmatch(r"[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?", t):
            raise ValueError(f"NumberFormatException: {text!r}")
        exact = Fraction(t)
    with np.errstate(over="ignore"):
        d = np.float32(float(exact))  # within one float32 ulp of the exact value
    if not np.isfinite(d):
        return float(d)
    best = d
    for c in (np.nextafter(d, np.float32(-np.inf)), np.nextafter(d, np.float32(np.inf))):
        if not np.isfinite(c):
            continue
        e0, e1 = abs(Fraction(float(best)) - exact), abs(Fraction(float(c)) - exact)
        if e1 < e0 or (e1 == e0 and int(c.view(np.uint32)) % 2 == 0):
            best = c
    if best == 0 and neg:
        return -0.0
    return float(best)


class DataStore:
    """One shard of one matrix, resident in HBM (a `dml_store`)."""

    def __init__(self, format: DataDesc, keys: KeyRange, cols: int = 1, device: int = 0,
                 float_array_ref_stride: bool = False, async_push: bool = False):
        if not isinstance(keys, KeyRange):
            # indexOf: "Only KeyRange or KeyHash is allowed in server storage" (FloatMatrixStore.java:185);
            # KeyHash shards (SURVEY defect 2) are not offered.
            raise RuntimeError("Only KeyRange is allowed in GPU server storage")
        self.format = format
        self.localRows = keys
        self.device = device
        L = _lib.load()
        flags = (DML_FLAG_FLOAT_ARRAY_REF_STRIDE if float_array_ref_stride else 0) | \
                (DML_FLAG_ASYNC if async_push else 0)
        h = C.c_void_p()
        self._h = None
        check(L.dml_store_create_range(C.byref(format.to_c()), keys.firstKey, keys.lastKey, int(cols), device,
                                       flags, C.byref(h)))
        self._h = h.value
        rows, c = C.c_int64(), C.c_int32()
        L.dml_store_shape(self._h, C.byref(rows), C.byref(c))
        self._rows, self._cols = rows.value, c.value
        self.dtype = VALUE_DTYPE[format.valueType]

    @classmethod
    def _wrap(cls, format: DataDesc, keys: KeyRange, cols: int, device: int, handle: int) -> "DataStore":
        """A view of a store owned elsewhere (a dml_group's shard): same API, no ownership."""
        self = cls.__new__(cls)
        self.format, self.localRows, self.device = format, keys, device
        self._h = handle
        self._owned = False
        rows, c = C.c_int64(), C.c_int32()
        _lib.load().dml_store_shape(self._h, C.byref(rows), C.byref(c))
        self._rows, self._cols = rows.value, c.value
        self.dtype = VALUE_DTYPE[format.valueType]
        return self

    # ---- lifecycle ----------------------------------------------------------
    def close(self):
        if not getattr(self, "_owned", True):
            self._h = None
            return
        if getattr(self, "_h", None):
            _lib.load().dml_store_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- DataStore API (DataStore.java:19-38) -------------------------------
    def rows(self) -> KeyRange:
        return self.localRows

    def rowSize(self) -> int:
        return self._cols

    def rand(self, seed: int = 1):
        """DataStore.rand (dml_store_rand). DoubleMatrixStore: the reference's values
        exactly (java.util.Random(1L) per shard, |nextGaussian()| rows scaled to unit
        norm, DoubleMatrixStore.java:192-207; `seed` unused). Float matrices draw from an
        unseeded Random in the reference (FloatMatrixStore.java:44), so here
        (a/100f - 0.5f)/rowSize with a uniform in 0..99 from a generator seeded by
        `seed` (FloatMatrixStore.java:39-51, FloatMatrixStoreAdaGrad.java:55-66); the
        other stores keep DataStore's no-op (DataStore.java:22)."""
        check(_lib.load().dml_store_rand(self._h, seed), self)

    def synth_fill(self, seed: int = 7):
        """Test/bench init with the counter-based generator the oracle restates
        (DESIGN.md §Synthetic data; pyoracle.OracleStore.synth_fill)."""
        check(_lib.load().dml_synth_fill_store(self._h, seed), self)

    def zero(self):
        """DataStore.zero(): a no-op on every store (DataStore.java:24). The float
        stores' zero(String) is an overload that PSActor's OP_ZERO never calls
        (FloatMatrixStore.java:57, PSActor.java:185-188). Use fill(0.0) to clear."""

    def set(self, value: str):
        """DataStore.set(String): FloatMatrixStore / FloatMatrixStoreAdaGrad fill every
        value with Float.parseFloat(value) (FloatMatrixStore.java:53-55,61-71,
        FloatMatrixStoreAdaGrad.java:69-71); a no-op on the other stores (DataStore.java:26)."""
        if self.format.dataType == DataDesc.DATA_TYPE_MATRIX and self.format.valueType == DataDesc.ELEMENT_TYPE_FLOAT:
            self.fill(java_parse_float(value))

    def fill(self, value: float):
        """Every value := value (dml_store_fill): test and tool access, not a reference API."""
        check(_lib.load().dml_store_fill(self._h, float(value)), self)

    @staticmethod
    def _host_view(data):
        """(pointer, length, keep-alive) of a push's bytes. A contiguous numpy uint8
        array (e.g. pinned_empty(), the wire-ingest buffer) is passed as is: the
        library DMAs pinned memory without staging. Anything else is copied to bytes."""
        if isinstance(data, np.ndarray) and data.dtype == np.uint8 and data.flags.c_contiguous:
            return data.ctypes.data, data.nbytes, data
        b = data if isinstance(data, bytes) else bytes(data)
        return C.cast(C.c_char_p(b), C.c_void_p).value, len(b), b

    def handlePush(self, format: DataDesc, data):
        """Apply one push (FloatMatrixStore.java:200-238 and the other typed stores).
        `data` is borrowed for the call (the reference's byte[]); with async_push the
        call returns once the bytes are captured."""
        self._check_format(format)
        p, n, keep = self._host_view(data)
        check(_lib.load().dml_store_push(self._h, C.c_void_p(p), n), self)
        del keep

    def handlePushBatch(self, format: DataDesc, datas: Sequence):
        """n sequential handlePush calls applied as one ordered multi-push reduce."""
        self._check_format(format)
        views = [self._host_view(d) for d in datas]
        n = len(views)
        ptrs = (C.c_void_p * max(n, 1))(*[v[0] for v in views])
        lens = (C.c_int64 * max(n, 1))(*[v[1] for v in views])
        check(_lib.load().dml_store_push_batch(self._h, ptrs, lens, n), self)
        del views

    def pushDevice(self, dev_ptrs, lens=None):
        """Device-resident pushes (pointers on this store's device), applied in order,
        asynchronously: a deferred error surfaces at a later call or flush().
        `dev_ptrs` may be a DeviceBatch (prebuilt argument arrays)."""
        b = dev_ptrs if isinstance(dev_ptrs, DeviceBatch) else DeviceBatch(dev_ptrs, lens)
        check(_lib.load().dml_store_push_batch_device(self._h, b.ptrs, b.lens, b.n), self)

    def flush(self):
        check(_lib.load().dml_store_flush(self._h), self)

    def push_seq(self) -> int:
        """Number of the last accepted push call (dml_store_push_seq)."""
        v = C.c_uint64()
        check(_lib.load().dml_store_push_seq(self._h, C.byref(v)), self)
        return v.value

    def retire(self, seq: int):
        """Finish the push calls up to `seq` on the host; their device buffers are
        no longer read afterwards (dml_store_retire). Raises their deferred error."""
        check(_lib.load().dml_store_retire(self._h, C.c_uint64(seq)), self)

    def stats(self, reset: bool = False) -> dict:
        """Pipeline counters (dml_store_stats): chunks, speculative chunks / re-runs,
        identity / reused / indexed pushes, counted as chunks retire."""
        c = _lib.dml_store_counters()
        check(_lib.load().dml_store_stats(self._h, C.byref(c), int(reset)), self)
        return {f: getattr(c, f) for f, _ in c._fields_}

    def handleFetch(self, format: DataDesc, rows: KeyCollection) -> bytes:
        """FloatMatrixStore.handleFetch dense-column layout (:113-174) and siblings."""
        self._check_format(format)
        keys = self.localRows.intersect(rows)
        L = _lib.load()
        out_len = C.c_int64()
        if isinstance(keys, KeyRange):
            cap = self._fetch_record_bytes() * max(keys.size(), 0)
            out = np.empty(max(cap, 1), np.uint8)
            check(L.dml_store_fetch_range(self._h, keys.firstKey, keys.lastKey, out.ctypes.data, cap,
                                          C.byref(out_len)), self)
        else:
            karr = np.fromiter(iter(keys), dtype=np.int64)
            cap = self._fetch_record_bytes() * len(karr)
            out = np.empty(max(cap, 1), np.uint8)
            check(L.dml_store_fetch(self._h, karr.ctypes.data_as(C.POINTER(C.c_int64)), len(karr),
                                    out.ctypes.data, cap, C.byref(out_len)), self)
        return out[:out_len.value].tobytes()

    def handleFetchInto(self, format: DataDesc, rows: KeyRange, out) -> int:
        """handleFetch of a KeyRange written into `out` (a writable buffer, e.g.
        pinned_empty()); returns the byte count. No intermediate copies."""
        self._check_format(format)
        keys = self.localRows.intersect(rows)
        if not isinstance(keys, KeyRange):
            raise TypeError("handleFetchInto takes a KeyRange")
        a = np.frombuffer(out, np.uint8) if not isinstance(out, np.ndarray) else out
        out_len = C.c_int64()
        check(_lib.load().dml_store_fetch_range(self._h, keys.firstKey, keys.lastKey, a.ctypes.data, a.nbytes,
                                                C.byref(out_len)), self)
        return out_len.value

    def writeAll(self, os=None) -> bytes:
        """Big-endian row-major dump (FloatMatrixStore.java:74-81); writes to `os` if given."""
        n = self._rows * self._cols * np.dtype(self.dtype).itemsize
        out = np.empty(max(n, 1), np.uint8)
        ln = C.c_int64()
        check(_lib.load().dml_store_write_all(self._h, out.ctypes.data, n, C.byref(ln)), self)
        b = out[:ln.value].tobytes()
        if os is not None:
            os.write(b)
        return b

    def readAll(self, is_) -> None:
        n = self._rows * self._cols * np.dtype(self.dtype).itemsize
        b = is_.read(n) if hasattr(is_, "read") else bytes(is_)
        check(_lib.load().dml_store_read_all(self._h, bytes(b), len(b)), self)

    def syncTo(self, os, fromRow: int, toRow: int):
        """Rows fromRow..toRow inclusive, big-endian (FloatMatrixStore.java:94-100);
        PSSync.java:131. Rows before a bad row are written before the error."""
        v = np.dtype(self.dtype).itemsize
        hi = min(toRow, self._rows - 1)
        cap = max(hi - fromRow + 1, 0) * self._cols * v
        out = np.empty(max(cap, 1), np.uint8)
        ln = C.c_int64()
        rc = _lib.load().dml_store_sync_to(self._h, fromRow, toRow, out.ctypes.data, cap, C.byref(ln))
        if ln.value and rc in (0, _lib.DML_E_KEY_OUT_OF_SHARD):
            os.write(out[:ln.value].tobytes())
        check(rc, self)

    def syncFrom(self, is_, fromRow: int, toRow: int):
        """Rows fromRow..toRow from big-endian bytes (PSSync.java:160). Follows the
        intended row layout; the reference's matrix syncFrom shadows rowSize with the
        row count (SURVEY defect 5), which this store does not reproduce."""
        v = np.dtype(self.dtype).itemsize
        hi = min(toRow, self._rows - 1)
        n = max(hi - fromRow + 1, 0) * self._cols * v
        if isinstance(is_, np.ndarray):  # e.g. pinned_empty(): handed to the DMA as is
            a = np.ascontiguousarray(is_.view(np.uint8).ravel()[:n])
            check(_lib.load().dml_store_sync_from(self._h, fromRow, toRow, a.ctypes.data, a.nbytes), self)
            return
        b = is_.read(n) if hasattr(is_, "read") else bytes(is_)[:n]
        check(_lib.load().dml_store_sync_from(self._h, fromRow, toRow, b, len(b)), self)

    # ---- AdaGrad ----------------------------------------------------------
    def setAlpha(self, initialAlpha: float, minAlpha: float, factor: float):
        check(_lib.load().dml_store_set_alpha(self._h, initialAlpha, minAlpha, factor), self)

    def maxDelta(self):
        v, r, c = C.c_float(), C.c_int32(), C.c_int32()
        check(_lib.load().dml_store_max_delta(self._h, C.byref(v), C.byref(r), C.byref(c)), self)
        return v.value, r.value, c.value

    def adagrad_state(self):
        n = self._rows * self._cols
        a = np.empty(n, np.float32)
        d = np.empty(n, np.float32)
        check(_lib.load().dml_store_read_adagrad(self._h, a.ctypes.data, d.ctypes.data, n), self)
        return a.reshape(self._rows, self._cols), d.reshape(self._rows, self._cols)

    # ---- raw access ---------------------------------------------------------
    def values(self) -> np.ndarray:
        a = np.empty((self._rows, self._cols), self.dtype)
        check(_lib.load().dml_store_read_dense(self._h, a.ctypes.data, a.nbytes), self)
        return a

    def load_values(self, a: np.ndarray):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        check(_lib.load().dml_store_write_dense(self._h, a.ctypes.data, a.nbytes), self)

    def error_state(self):
        k, c = C.c_int64(), C.c_int32()
        code = _lib.load().dml_store_error_state(self._h, C.byref(k), C.byref(c))
        return code, k.value, c.value

    def clear_error(self):
        _lib.load().dml_store_clear_error(self._h)

    def device_ptr(self) -> int:
        p = C.c_void_p()
        check(_lib.load().dml_store_device_ptr(self._h, C.byref(p)), self)
        return p.value

    def stream(self) -> int:
        p = C.c_void_p()
        check(_lib.load().dml_store_stream(self._h, C.byref(p)), self)
        return p.value or 0

    def set_timing(self, on, every: int = 1):
        """Kernel timing of the dominant reduce: every launch, or one chunk in `every`."""
        check(_lib.load().dml_store_set_timing(self._h, (max(int(every), 1) if on else 0)), self)

    def set_knob(self, knob: int, value: int):
        """Diagnostic tuning knob (dml_diag_store_knob), e.g. DML_KNOB_IDENT_FULL_MIN_BYTES = 1."""
        check(_lib.load().dml_diag_store_knob(self._h, int(knob), int(value)), self)

    def kernel_name(self) -> str:
        """Instantiation of the dominant kernel last launched (dml_store_kernel_name)."""
        buf = C.create_string_buffer(512)
        check(_lib.load().dml_store_kernel_name(self._h, buf, 512), self)
        return buf.value.decode()

    def kernel_time(self, reset=True):
        ms, n = C.c_double(), C.c_int64()
        check(_lib.load().dml_store_kernel_time(self._h, C.byref(ms), C.byref(n), int(reset)), self)
        return ms.value, n.value

    def iter(self):
        """(key, value-row) pairs in shard order (FloatMatrixStore.Iter, :241-269)."""
        vals = self.values()
        for i in range(self._rows):
            yield self.localRows.firstKey + i, (vals[i] if self._cols > 1 or self.format.dataType == 1 else vals[i, 0])

    # ---- helpers ------------------------------------------------------------
    def _check_format(self, format: DataDesc):
        if format is not None and not format.same_layout(self.format):
            raise IllegalArgumentException("push format differs from the store's DataDesc "
                                           "(PSAgent passes the server-side format, PSAgent.java:279)")

    def _fetch_record_bytes(self) -> int:
        f = self.format
        if f.dataType == DataDesc.DATA_TYPE_MATRIX:
            return f.keySize + self._cols * (8 if f.adaGrad and f.valueType == DataDesc.ELEMENT_TYPE_FLOAT
                                             else f.valueSize)
        return f.keySize + (8 if f.valueType == DataDesc.ELEMENT_TYPE_FLOAT else f.valueSize)

    # ---- factory (DataStore.java:41-92) -------------------------------------
    @staticmethod
    def createStore(serverIndex: int, matrix, device: Optional[int] = None, **kw) -> "DataStore":
        fmt: DataDesc = matrix.getFormat()
        if fmt.valueType not in VALUE_DTYPE or fmt.dataType not in (0, 1):
            raise IllegalArgumentException("Unrecognized matrix type: " + type(matrix).__name__)
        part = matrix.partitions[serverIndex]
        cols = matrix.getColKeys().size() if fmt.dataType == DataDesc.DATA_TYPE_MATRIX else 1
        return DataStore(fmt, part, cols, serverIndex if device is None else device, **kw)

    @staticmethod
    def createStores(model, serverIndex: int, device: Optional[int] = None):
        return {name: DataStore.createStore(serverIndex, m, device) for name, m in model.dataMap.items()}


def pinned_empty(nbytes: int) -> np.ndarray:
    """uint8 array over pinned host memory (dml_host_alloc); freed with the array."""
    L = _lib.load()
    p = C.c_void_p()
    check(L.dml_host_alloc(nbytes, C.byref(p)))
    buf = (C.c_uint8 * max(nbytes, 1)).from_address(p.value)
    weakref.finalize(buf, L.dml_host_free, p.value)
    return np.frombuffer(buf, np.uint8, count=nbytes)


class DeviceBatch:
    """ctypes argument arrays for a list of device-resident pushes (built once, reusable)."""

    def __init__(self, dev_ptrs: Sequence[int], lens: Sequence[int]):
        self.n = len(dev_ptrs)
        self.ptrs = (C.c_void_p * max(self.n, 1))(*dev_ptrs)
        self.lens = (C.c_int64 * max(self.n, 1))(*lens)


class DMatrix:
    """The parts of api/DMatrix.java the store factory reads: format, row keys, partitions."""

    def __init__(self, rows: int, cols: int, format: DataDesc, name: str = ""):
        self.rowKeys = KeyRange(0, rows - 1)            # DMatrix.java:27-31
        self.colKeys = KeyRange(0, cols - 1)
        self.format = format
        self.name = name
        self.partitions: List[KeyRange] = []

    def getFormat(self) -> DataDesc:
        return self.format

    def getRowKeys(self) -> KeyRange:
        return self.rowKeys

    def getColKeys(self) -> KeyRange:
        return self.colKeys if self.format.dataType == DataDesc.DATA_TYPE_MATRIX else KeyRange(0, 0)

    def partition(self, serverNum: int):
        self.partitions = self.rowKeys.linearSplit(serverNum)  # DMatrix.java:53-64
        return self.partitions


class Model:
    """api/Model.java: registerMatrix + autoPartition (Model.java:23-42)."""

    def __init__(self):
        self.dataMap = {}

    def registerMatrix(self, name: str, m: DMatrix):
        m.name = name
        self.dataMap[name] = m

    def autoPartition(self, psCount: int):
        for m in self.dataMap.values():
            m.partition(psCount)


# ---- record codec: the byte layout of the reference's writers ---------------
def encode_matrix_push(keys, values, key_type: int, value_type: int) -> bytes:
    """[key LE][cols x value LE] per row — SparseMatrix.writeMap dense branch
    (SparseMatrix.java:96-148). `values` is (n, cols)."""
    keys = np.asarray(keys, dtype=np.int64)
    vals = np.ascontiguousarray(values, dtype=VALUE_DTYPE[value_type])
    kdt = np.dtype("<i4") if key_type == DataDesc.KEY_TYPE_INT else np.dtype("<i8")
    rec = np.empty(len(keys), dtype=[("k", kdt), ("v", vals.dtype.newbyteorder("<"), (vals.shape[1],))])
    rec["k"] = keys
    rec["v"] = vals
    return rec.tobytes()


def encode_array_push(keys, values, key_type: int, value_type: int, value_stride: Optional[int] = None) -> bytes:
    """[key LE][value LE] per entry — SparseArray.writeMap (SparseArray.java:63-76).
    `value_stride` 8 for a float pads each value to FloatArrayStore's VALUE_SIZE."""
    keys = np.asarray(keys, dtype=np.int64)
    dt = VALUE_DTYPE[value_type]
    vs = value_stride or np.dtype(dt).itemsize
    kdt = np.dtype("<i4") if key_type == DataDesc.KEY_TYPE_INT else np.dtype("<i8")
    K = kdt.itemsize
    out = np.zeros(len(keys) * (K + vs), np.uint8).reshape(len(keys), K + vs)
    out[:, :K] = keys.astype(kdt).view(np.uint8).reshape(len(keys), K)
    v = np.asarray(values, dtype=np.dtype(dt).newbyteorder("<"))
    out[:, K:K + v.itemsize] = v.view(np.uint8).reshape(len(keys), v.itemsize)
    return out.tobytes()
