"""Generate tests/golden/kat_cases.json — known-answer tests for the push path.

Expected values come from THIS file's own pure-Python/numpy restatement of the
Java store loops (independent of oracle/dml_oracle.c), written from the Java
Language Specification: np.float32/np.float64 scalar `+`/`*` are single IEEE
roundings (JLS 15.18.2, 15.17.1; no FMA), int adds wrap mod 2^32, and a Java
exception stops the loop with every earlier add applied. A handful of cases
also carry literal, hand-computed expectations (`literal`), checked below.

Reference (no tests/fixtures of its own): the Java loops at
src/main/java/com/intel/distml/util/store/*.java cited per case.

Run: python tests/golden/make_golden.py   (rewrites kat_cases.json)
"""
from __future__ import annotations

import json
import math
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ARRAY, MATRIX = 0, 1
KINT, KLONG = 0, 1
VINT, VFLOAT, VDOUBLE = 0, 1, 3
OK, BAD_KEY, TRUNC, NEG = 0, 2, 3, 4
VDT = {VINT: np.int32, VFLOAT: np.float32, VDOUBLE: np.float64}


class JStore:
    """Pure-Python restatement of the typed stores' handlePush."""

    def __init__(self, dt, kt, vt, first, last, cols=1, ada=False, ref_stride=False):
        self.dt, self.kt, self.vt = dt, kt, vt
        self.first, self.rows = first, last - first + 1
        self.cols = cols if dt == MATRIX else 1
        self.K = 4 if kt == KINT else 8
        self.V = 4 if vt in (VINT, VFLOAT) else 8
        self.vs = 8 if (dt == ARRAY and vt == VFLOAT and ref_stride) else self.V
        self.data = np.zeros((self.rows, self.cols), VDT[vt])
        self.ada = ada and dt == MATRIX and vt == VFLOAT
        self.alpha = np.zeros((self.rows, self.cols), np.float32)
        self.delta = np.zeros((self.rows, self.cols), np.float32)
        self.ia, self.mina, self.factor = np.float32(0), np.float32(0), np.float32(1.5)
        self.maxd, self.maxr, self.maxc = np.float32(0), 0, 0

    def idx(self, key):
        i = (key - self.first) & 0xFFFFFFFF          # (int)(key - firstKey)
        i = i - (1 << 32) if i >= (1 << 31) else i
        return i if 0 <= i < self.rows else None     # else ArrayIndexOutOfBounds

    def rd(self, data, off, n):
        if off + n > len(data):
            raise IndexError
        return data[off:off + n]

    def key(self, data, off):
        b = self.rd(data, off, self.K)
        return struct.unpack("<i" if self.K == 4 else "<q", b)[0]

    def val(self, data, off):
        b = self.rd(data, off, self.V)
        return {VINT: lambda: np.int32(struct.unpack("<i", b)[0]),
                VFLOAT: lambda: np.frombuffer(b, "<f4")[0],
                VDOUBLE: lambda: np.frombuffer(b, "<f8")[0]}[self.vt]()

    def add(self, r, c, u):
        if self.vt == VINT:
            s = (int(self.data[r, c]) + int(u)) & 0xFFFFFFFF
            self.data[r, c] = np.int32(s - (1 << 32) if s >= (1 << 31) else s)
        else:
            self.data[r, c] = self.data[r, c] + u

    def push(self, data: bytes):
        """Returns (status, key, col)."""
        off, key = 0, 0
        while off < len(data):
            try:
                key = self.key(data, off)
            except IndexError:
                return TRUNC, 0, -1
            off += self.K
            if self.dt == MATRIX:
                r = self.idx(key)
                if r is None:
                    return BAD_KEY, key, -1
                for i in range(self.cols):
                    try:
                        u = self.val(data, off)
                    except IndexError:
                        return TRUNC, key, i
                    self.add(r, i, u)
                    if self.ada:
                        self.delta[r, i] = self.delta[r, i] + u * u
                        if float(self.delta[r, i]) > 1.0:
                            a = np.float32(float(self.ia) / (float(self.factor) * math.sqrt(float(self.delta[r, i]))))
                            self.alpha[r, i] = self.mina if a < self.mina else a
                        if self.delta[r, i] > self.maxd:
                            self.maxd, self.maxr, self.maxc = self.delta[r, i], np.int32(key).item(), i
                    if self.vt == VINT and self.data[r, i] < 0:
                        return NEG, key, i
                    off += self.V
            else:
                try:
                    u = self.val(data, off)
                except IndexError:
                    return TRUNC, key, -1
                off += self.vs
                r = self.idx(key)
                if r is None:
                    return BAD_KEY, key, -1
                self.add(r, 0, u)
                if self.vt == VINT and self.data[r, 0] < 0:
                    return NEG, key, -1
        return OK, 0, -1


def mrec(kt, vt, key, vals):
    kb = struct.pack("<i" if kt == KINT else "<q", key)
    return kb + np.asarray(vals, VDT[vt]).astype(np.dtype(VDT[vt]).newbyteorder("<")).tobytes()


def arec(kt, vt, key, v, vs=None):
    kb = struct.pack("<i" if kt == KINT else "<q", key)
    vb = np.asarray([v], VDT[vt]).astype(np.dtype(VDT[vt]).newbyteorder("<")).tobytes()
    pad = (vs or len(vb)) - len(vb)
    return kb + vb + b"\0" * pad


F = np.float32
cases = []
np.seterr(all="ignore")


def case(name, ref, dt, kt, vt, first, last, pushes, cols=1, init=None, ada=None, ref_stride=False, literal=None):
    s = JStore(dt, kt, vt, first, last, cols, ada is not None, ref_stride)
    if init is not None:
        s.data[:] = np.asarray(init, VDT[vt]).reshape(s.data.shape)
    if ada is not None:
        s.ia, s.mina, s.factor = F(ada[0]), F(ada[1]), F(ada[2])
        s.alpha[:] = s.ia
    init_hex = s.data.astype(s.data.dtype.newbyteorder("<")).tobytes().hex()
    status = (OK, 0, -1)
    applied = 0
    for p in pushes:
        status = s.push(p)
        applied += 1
        if status[0] != OK:
            break
    exp = {"status": status[0], "key": int(status[1]), "col": int(status[2]), "pushes_applied": applied,
           "data_hex": s.data.astype(s.data.dtype.newbyteorder("<")).tobytes().hex()}
    if s.ada:
        exp["alpha_hex"] = s.alpha.astype("<f4").tobytes().hex()
        exp["delta_hex"] = s.delta.astype("<f4").tobytes().hex()
        exp["max_delta"] = [float(s.maxd), int(s.maxr), int(s.maxc)]
    if literal is not None:
        got = s.data.reshape(-1).tolist()
        for i, want in literal.items():
            g = got[i]
            assert (g == want and math.copysign(1, g) == math.copysign(1, want)) or \
                (isinstance(want, float) and math.isnan(want) and math.isnan(g)), (name, i, g, want)
    cases.append({"name": name, "ref": ref,
                  "desc": {"data_type": dt, "key_type": kt, "value_type": vt, "dense_column": 1,
                           "ada_grad": int(ada is not None)},
                  "first": first, "last": last, "cols": cols if dt == MATRIX else 1,
                  "float_array_ref_stride": int(ref_stride), "ada": list(ada) if ada else None,
                  "init_hex": init_hex, "pushes_hex": [p.hex() for p in pushes], "expected": exp})


FMS = "FloatMatrixStore.java:200-222"
IMS = "IntMatrixStore.java:154-178"
FAS = "FloatArrayStore.java:110-122"
IAS = "IntArrayStore.java:97-113"
DAS = "DoubleArrayStore.java:115-127"
DMS = "DoubleMatrixStore.java:153-175"
ADA = "FloatMatrixStoreAdaGrad.java:239-284"
e24 = float(2.0 ** -24)

# --- fp32 ordered rounding: 1 + 2^-24 rounds to 1 (ties-to-even); order matters
case("f32_ordered_rounding", FMS, MATRIX, KINT, VFLOAT, 0, 1,
     [mrec(KINT, VFLOAT, 0, [1.0, 0.0]), mrec(KINT, VFLOAT, 0, [e24, e24]), mrec(KINT, VFLOAT, 0, [e24, e24])],
     cols=2, literal={0: 1.0, 1: 2.0 ** -23})
# --- same row twice inside one push (sequential within the push)
case("f32_row_twice_in_push", FMS, MATRIX, KINT, VFLOAT, 10, 13,
     [mrec(KINT, VFLOAT, 11, [1.0, 2.0]) + mrec(KINT, VFLOAT, 12, [3.0, 4.0]) + mrec(KINT, VFLOAT, 11, [e24, 0.5])],
     cols=2, literal={2: 1.0, 3: 2.5})
# --- signed zeros, denormals, Inf/NaN
case("f32_zero_denormal_inf_nan", FMS, MATRIX, KINT, VFLOAT, 0, 0,
     [mrec(KINT, VFLOAT, 0, [-0.0, -0.0, 2.0 ** -149, 3e38, float("inf"), 1.0]),
      mrec(KINT, VFLOAT, 0, [-0.0, 0.0, 2.0 ** -149, 3e38, float("-inf"), float("nan")])],
     cols=6, init=[0.0, -0.0, 0.0, 0.0, 0.0, 0.0],
     literal={0: 0.0, 1: 0.0, 2: 2.0 ** -148, 3: float("inf"), 4: float("nan"), 5: float("nan")})
# --- long keys, permuted record order
case("f32_long_keys_permuted", FMS, MATRIX, KLONG, VFLOAT, 1 << 33, (1 << 33) + 3,
     [b"".join(mrec(KLONG, VFLOAT, (1 << 33) + r, [r + 0.25, -r]) for r in (3, 0, 2, 1)),
      b"".join(mrec(KLONG, VFLOAT, (1 << 33) + r, [0.125, 1.0]) for r in (1, 3))], cols=2)
# --- key outside the shard: earlier records applied, the failing record not
case("f32_key_out_of_shard", FMS, MATRIX, KINT, VFLOAT, 100, 103,
     [mrec(KINT, VFLOAT, 100, [1.0]), mrec(KINT, VFLOAT, 101, [2.0]) + mrec(KINT, VFLOAT, 99, [5.0]) +
      mrec(KINT, VFLOAT, 102, [3.0]), mrec(KINT, VFLOAT, 103, [4.0])], cols=1, literal={0: 1.0, 1: 2.0, 2: 0.0, 3: 0.0})
# --- (int)(key - firstKey) narrowing: key = first + 2^32 lands on row 0 (reference quirk)
case("f32_key_narrowing_quirk", FMS, MATRIX, KLONG, VFLOAT, 0, 3,
     [mrec(KLONG, VFLOAT, (1 << 32) + 1, [7.0])], cols=1, literal={1: 7.0})
# --- truncated push: values before the cut are applied
case("f32_truncated_value", FMS, MATRIX, KINT, VFLOAT, 0, 1,
     [mrec(KINT, VFLOAT, 0, [1.0, 1.0, 1.0]) + mrec(KINT, VFLOAT, 1, [2.0, 2.0, 2.0])[:4 + 8 + 2]], cols=3,
     literal={0: 1.0, 3: 2.0, 4: 2.0, 5: 0.0})
case("f32_truncated_key", FMS, MATRIX, KINT, VFLOAT, 0, 1,
     [mrec(KINT, VFLOAT, 1, [1.0, 1.0]) + b"\x00\x00"], cols=2, literal={2: 1.0, 3: 1.0})
# --- int32 wrap and the negativity check (the failing add is applied, then the throw)
case("i32_wrap_negative", IMS, MATRIX, KINT, VINT, 0, 1,
     [mrec(KINT, VINT, 0, [2147483647, 5]), mrec(KINT, VINT, 1, [3, 4]) + mrec(KINT, VINT, 0, [1, 6]),
      mrec(KINT, VINT, 1, [1, 1])], cols=2, literal={0: -2147483648, 1: 5, 2: 3, 3: 4})
case("i32_intermediate_negative", IMS, MATRIX, KINT, VINT, 0, 0,
     [mrec(KINT, VINT, 0, [2, 2]), mrec(KINT, VINT, 0, [-1, -3]), mrec(KINT, VINT, 0, [5, 5])], cols=2,
     literal={0: 1, 1: -1})
case("i32_counts_ok", IMS, MATRIX, KINT, VINT, 5, 8,
     [mrec(KINT, VINT, 6, [1, 2, 3]) + mrec(KINT, VINT, 8, [4, 5, 6]), mrec(KINT, VINT, 6, [-1, -2, 0])],
     cols=3, init=[[3, 3, 3]] * 4)
# --- arrays
case("f32_array_writer_stride", FAS, ARRAY, KLONG, VFLOAT, 0, 9,
     [arec(KLONG, VFLOAT, 3, 1.5) + arec(KLONG, VFLOAT, 7, -2.0), arec(KLONG, VFLOAT, 3, 0.25)],
     literal={3: 1.75, 7: -2.0})
case("f32_array_reference_stride", FAS, ARRAY, KLONG, VFLOAT, 0, 9,
     [arec(KLONG, VFLOAT, 3, 1.5, 8) + arec(KLONG, VFLOAT, 7, -2.0, 8)[:12]], ref_stride=True,
     literal={3: 1.5, 7: -2.0})
case("i32_array_negative", IAS, ARRAY, KINT, VINT, 0, 3,
     [arec(KINT, VINT, 1, 4) + arec(KINT, VINT, 2, 1), arec(KINT, VINT, 1, -5) + arec(KINT, VINT, 2, 9)],
     literal={1: -1, 2: 1})
case("f64_array", DAS, ARRAY, KINT, VDOUBLE, 1000, 1003,
     [arec(KINT, VDOUBLE, 1001, 0.1) + arec(KINT, VDOUBLE, 1003, 1e-300), arec(KINT, VDOUBLE, 1001, 0.2)],
     literal={1: 0.1 + 0.2})
case("f64_matrix", DMS, MATRIX, KLONG, VDOUBLE, 0, 2,
     [mrec(KLONG, VDOUBLE, 2, [1.0, 2.0 ** -53]), mrec(KLONG, VDOUBLE, 2, [2.0 ** -53, 1.0])], cols=2,
     literal={4: 1.0, 5: 1.0})
# --- AdaGrad: delta crosses 1.0, alpha in double then clamped to minAlpha; maxDelta
case("adagrad_alpha_clamp", ADA, MATRIX, KINT, VFLOAT, 0, 2,
     [mrec(KINT, VFLOAT, 1, [0.5, 2.0, 0.0]) + mrec(KINT, VFLOAT, 0, [1.5, 0.1, 3.0]),
      mrec(KINT, VFLOAT, 1, [1.0, 0.0, 0.75]), mrec(KINT, VFLOAT, 2, [3.0, 0.0, 0.0])],
     cols=3, ada=(0.025, 0.0001, 1.5))
case("adagrad_minalpha_hit", ADA, MATRIX, KINT, VFLOAT, 0, 0,
     [mrec(KINT, VFLOAT, 0, [100.0, 1.01])], cols=2, ada=(0.025, 0.001, 1.5))

# --- linearSplit (KeyRange.java:68-80)
splits = {"0_9_4": [[0, 2], [3, 5], [6, 8], [9, 9]], "0_4_4": [[0, 1], [2, 3], [4, 4], [6, 4]],
          "0_16383_1": [[0, 16383]], "0_9999999_8": [[i * 1250000, i * 1250000 + 1249999] for i in range(8)],
          "0_999999_8": [[i * 125000, i * 125000 + 124999] for i in range(8)]}

if __name__ == "__main__":
    np.seterr(all="ignore")
    with open(os.path.join(HERE, "kat_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": cases, "linear_split": splits}, f, indent=1)
    print(f"wrote {len(cases)} cases")
