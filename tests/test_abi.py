"""CPU: the C-ABI library loads, exports every symbol include/distml_ps.h
declares, and the host-side mirror (DataDesc, KeyRange, codec) is correct.
No GPU compute here."""
import ctypes as C
import os
import re
import struct

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "distml_ps.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dml_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from distml_amd import _lib
    assert declared_symbols() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    from distml_amd import _lib
    L = _lib.load()  # binds every signature: AttributeError if one is missing
    raw = C.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(raw, name), name
    assert b"gfx950" in L.dml_version()


def test_library_is_built_for_gfx950_only():
    from distml_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_linear_split_cabi():
    from distml_amd import _lib
    L = _lib.load()
    f = (C.c_int64 * 4)()
    l = (C.c_int64 * 4)()
    assert L.dml_linear_split(0, 9, 4, f, l) == 0
    assert list(zip(f, l)) == [(0, 2), (3, 5), (6, 8), (9, 9)]


def test_create_without_gpu_fails_loudly():
    from distml_amd import _lib
    from distml_amd.datadesc import DataDesc
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    L = _lib.load()
    h = C.c_void_p()
    rc = L.dml_store_create_range(C.byref(DataDesc(1, 0, 1).to_c()), 0, 15, 4, 0, 0, C.byref(h))
    assert rc != 0 and h.value is None
    # a bad descriptor is rejected before any device work (IllegalArgumentException)
    rc = L.dml_store_create_range(C.byref(DataDesc(1, 0, 2).to_c()), 0, 15, 4, 0, 0, C.byref(h))
    assert rc == _lib.DML_E_BAD_DESC


def test_datadesc_wire_and_sizes():
    from distml_amd.datadesc import DataDesc
    d = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_LONG, DataDesc.ELEMENT_TYPE_DOUBLE,
                 False, True, False)
    assert (d.keySize, d.valueSize) == (8, 8)
    assert d.write() == struct.pack(">6i", 1, 1, 3, 0, 1, 0)
    assert DataDesc.read(d.write()).same_layout(d)
    assert (DataDesc(0, 0, 1).keySize, DataDesc(0, 0, 1).valueSize) == (4, 4)


def test_keyrange_intersect():
    from distml_amd.datadesc import ALL, EMPTY, KeyList, KeyRange
    r = KeyRange(10, 19)
    assert r.intersect(KeyRange(15, 30)) == KeyRange(15, 19)
    assert r.intersect(KeyRange(20, 30)) is EMPTY
    assert list(r.intersect(KeyList([3, 12, 19, 25]))) == [12, 19]
    assert r.intersect(ALL) is r
    assert r.size() == 10 and r.contains(10) and not r.contains(20)


def test_codec_matches_oracle_generator(oracle):
    from distml_amd.store import encode_array_push, encode_matrix_push
    b = oracle.synth_dense_bucket(1, 1, 5, 8, 8, 3, seed=3)
    rec = b.reshape(8, 8 + 12)
    keys = rec[:, :8].copy().view("<i8").ravel()
    vals = rec[:, 8:].copy().view("<f4").reshape(8, 3)
    assert encode_matrix_push(keys, vals, 1, 1) == b.tobytes()
    s = oracle.synth_sparse_bucket(0, 0, 100, 50, 10, seed=4, perm_a=7, perm_c=1)
    r = s.reshape(10, 8)
    assert encode_array_push(r[:, :4].copy().view("<i4").ravel(), r[:, 4:].copy().view("<i4").ravel(), 0, 0) \
        == s.tobytes()
    padded = encode_array_push([1], [2.0], 1, 1, value_stride=8)
    assert padded == struct.pack("<q", 1) + struct.pack("<f", 2.0) + b"\0" * 4


def test_dmatrix_partition_and_factory_dispatch():
    from distml_amd import DataDesc, DataStore, DMatrix, IllegalArgumentException
    m = DMatrix(1_000_000, 1000, DataDesc(1, 0, 0))
    parts = m.partition(8)
    assert parts[0].firstKey == 0 and parts[0].lastKey == 124999 and parts[7].lastKey == 999999
    bad = DMatrix(10, 2, DataDesc(1, 0, DataDesc.ELEMENT_TYPE_LONG))
    bad.partition(1)
    with pytest.raises(IllegalArgumentException):
        DataStore.createStore(0, bad)


def test_rccl_double_covers_the_library_imports():
    """tests/rccl_double (the stand-in the native group's N > 1 tests load ahead of
    libdistml_ps.so) defines every nccl* symbol the product library imports."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "tests", "rccl_double")], check=True)

    def syms(path, kind):
        out = subprocess.run(["nm", "-D", path], check=True, capture_output=True, text=True).stdout
        return {ln.split()[-1] for ln in out.splitlines() if ln.split()[-2:-1] == [kind] and "nccl" in ln}
    need = syms(os.path.join(root, "distml_amd", "libdistml_ps.so"), "U")
    have = syms(os.path.join(root, "tests", "rccl_double", "librccl_double.so"), "T")
    assert need and need <= have, need - have
