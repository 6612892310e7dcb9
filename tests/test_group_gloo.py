"""CPU, multi-process (gloo): the sharded full-range push path of distml_amd.group.

ShardGroup's orchestration (linearSplit shard plan, ordered local pre-reduce,
reduce-scatter of the partials, owner apply) runs for real over torch.distributed
with world_size 2, 3, 4 and 8; only the two device ops are replaced by oracle-backed
CPU stand-ins injected by this test (the product ops are the HIP kernels).

Tolerance: the sharded path sums each element as p0 + (P_0 + P_1 + ...) where
P_r is rank r's ordered partial, the reference as p0 + g_0 + g_1 + ... . For
int32 the two are identical (exact, mod 2^32). For fp32 both orders are within
Higham's recursive-summation bound of the exact sum, so
    |ours - oracle| <= 2 (n-1) 2^-24 sum|terms|,   n = number of terms,
and the test also checks the north-star's 1e-6 relative bound (to sum|terms|)
against the exact sum. It does not check that bound against the oracle: with
|init| >> |gradient| the sequential order rounds n-1 times at the shard value's
magnitude and the sharded order once, so at n ~ 30 the reference's own error
reaches 1e-6 of sum|terms| while ours stays near 2^-24.
"""
import ctypes as C
import os
import socket
import sys

import numpy as np
import pytest

import kat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleShard:
    def __init__(self, pyoracle, fmt, shard, cols, init):
        self.o = pyoracle.OracleStore(fmt.dataType, fmt.keyType, fmt.valueType, shard.firstKey, shard.lastKey, cols)
        self.o.data[:] = init

    def flush(self):
        pass


class OracleOps:
    def __init__(self, pyoracle):
        self.po = pyoracle

    def prereduce(self, fmt, first, rows, cols, ptrs, lens, out_ptr, stream):
        dt = {0: np.int32, 1: np.float32, 3: np.float64}[fmt.valueType]
        out = np.frombuffer((C.c_char * (rows * cols * np.dtype(dt).itemsize)).from_address(out_ptr), dtype=dt)
        if fmt.valueType == 0:  # partial sums of count deltas may be negative: plain wrapping adds
            acc = np.zeros((rows, cols), np.int64)
            for p, n in zip(ptrs, lens):
                rec = np.frombuffer(C.string_at(p, n), np.uint8).reshape(-1, 4 + 4 * cols)
                keys = rec[:, :4].copy().view("<i4").ravel() - first
                acc[keys] += rec[:, 4:].copy().view("<i4")
            out[:] = (acc.reshape(-1) & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
            return
        o = self.po.OracleStore(fmt.dataType, fmt.keyType, fmt.valueType, first, first + rows - 1, cols)
        for p, n in zip(ptrs, lens):
            assert o.push(C.string_at(p, n)) == 0
        out[:] = o.data.reshape(-1)

    def apply(self, store, src_ptr, elems):
        d = store.o.data
        src = np.frombuffer((C.c_char * (elems * d.itemsize)).from_address(src_ptr), dtype=d.dtype)
        if d.dtype == np.int32:
            d[:] = (d.reshape(-1).astype(np.int64) + src).astype(np.int32).reshape(d.shape)
        else:
            d += src.reshape(d.shape)


def _buckets(pyoracle, vt, rank, W, rows, cols):
    return [pyoracle.synth_dense_bucket(0, vt, 0, rows, rows, cols, 100 * rank + b, (2 * b + 1) % rows or 1, b)
            for b in range(W)]


def _worker(rank, world, port, vt, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    import pyoracle
    from distml_amd.datadesc import DataDesc
    from distml_amd.group import ShardGroup

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows, cols, W = 101, 37, 4
    fmt = DataDesc(1, 0, vt)
    rng = np.random.default_rng(5)
    dt = {0: np.int32, 1: np.float32}[vt]
    init_full = (rng.integers(50, 60, size=(rows, cols)) if vt == 0 else rng.standard_normal((rows, cols))).astype(dt)

    holder = {}

    def factory():
        shard = holder["g"].shard
        return OracleShard(pyoracle, fmt, shard, cols, init_full[shard.firstKey:shard.lastKey + 1])

    class G(ShardGroup):
        def __init__(self, *a, **k):
            holder["g"] = self
            super().__init__(*a, **k)

    g = G(fmt, rows, cols, rank, world, device=None, ops=OracleOps(pyoracle), store_factory=factory)
    bufs = [torch.from_numpy(b) for b in _buckets(pyoracle, vt, rank, W, rows, cols)]
    g.push_full_range([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
    g.flush()
    np.save(os.path.join(out_dir, f"shard{rank}.npy"), g.store.o.data)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# world 4 and 8 (the driver's node sizes): linearSplit(8) of 101 rows is 7 shards of 13
# and a short last shard of 10 (padded in the reduce-scatter)
@pytest.mark.parametrize("world,vt", [(2, 1), (2, 0), (3, 1), (4, 1), (8, 1), (8, 0)])
def test_sharded_full_range_push_gloo(tmp_path, oracle, world, vt):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), vt, str(tmp_path)), nprocs=world, join=True)
    rows, cols, W = 101, 37, 4
    from distml_amd.datadesc import KeyRange
    parts = KeyRange(0, rows - 1).linearSplit(world)
    got = np.concatenate([np.load(tmp_path / f"shard{r}.npy") for r in range(world)])
    # reference: one sequential store, every rank's pushes in rank-major push order
    rng = np.random.default_rng(5)
    dt = {0: np.int32, 1: np.float32}[vt]
    init = (rng.integers(50, 60, size=(rows, cols)) if vt == 0 else rng.standard_normal((rows, cols))).astype(dt)
    o = oracle.OracleStore(1, 0, vt, 0, rows - 1, cols)
    o.data[:] = init
    all_b = [b for r in range(world) for b in _buckets(oracle, vt, r, W, rows, cols)]
    for b in all_b:
        assert o.push(b.tobytes()) == 0
    assert got.shape == o.data.shape and sum(p.size() for p in parts) == rows
    if vt == 0:
        assert np.array_equal(got, o.data)
        return
    kat.rs_parity(got, o.data, init, [b.tobytes() for b in all_b], cols, f"gloo world {world}")
