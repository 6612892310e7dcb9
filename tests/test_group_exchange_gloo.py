"""CPU, multi-process (gloo): the exact exchange path of distml_amd.group
(ShardGroup.push_exchange) at world_size 2, 3, 4 and 8.

Each rank pushes key-subset buckets; ShardGroup splits them by owner shard,
exchanges the slices all-to-all over torch.distributed, and each owner applies
its slices in rank-major push order through the store's ordered push. Only the
split kernel and the store are CPU stand-ins here (numpy split; the oracle as
the store), injected by this test — the product ops are dml_shard_split and the
HIP DataStore (tests/test_gpu_parity.py covers both on the GPU).

Two exchange calls run back to back without a flush (the pipelined path hands a
call's slices to the store at the next call). Expected: bit-exact against ONE
oracle store applying every call's buckets, each call in rank-major order — AdaGrad data, alpha and delta, and int32 counts — because the
split keeps each push's record order and rows are independent.
"""
import ctypes as C
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS, COLS, W = 97, 24, 3
ADA = (0.025, 0.0001, 1.5)


def _fmt(vt):
    from distml_amd.datadesc import DataDesc
    return DataDesc(1, 0, vt, False, True, vt == 1)


CALLS = 2  # back-to-back exchange calls without a flush between them (pipelined path)


def _buckets(vt, rank, call=0):
    from distml_amd import encode_matrix_push
    out = []
    for b in range(W):
        rng = np.random.default_rng(1000 * rank + 100 * call + b)
        keys = rng.permutation(ROWS)[: rng.integers(ROWS // 3, ROWS)]
        if vt == 1:
            vals = (rng.standard_normal((len(keys), COLS)) * 0.6).astype(np.float32)
        else:
            vals = rng.integers(-2, 3, size=(len(keys), COLS)).astype(np.int32)
        out.append(np.frombuffer(encode_matrix_push(keys, vals, 0, vt), np.uint8).copy())
    return out


def _init(vt):
    rng = np.random.default_rng(9)
    return (rng.standard_normal((ROWS, COLS)).astype(np.float32) if vt == 1
            else rng.integers(50, 60, size=(ROWS, COLS)).astype(np.int32))


class OracleStoreShard:
    """The oracle behind DataStore.pushDevice (host pointers stand in for device ones)."""

    def __init__(self, pyoracle, fmt, shard, init):
        self.o = pyoracle.OracleStore(1, 0, fmt.valueType, shard.firstKey, shard.lastKey, COLS, 1, int(fmt.adaGrad))
        if fmt.adaGrad:
            self.o.set_alpha(*ADA)
        self.o.data[:] = init

    def pushDevice(self, ptrs, lens):
        for p, n in zip(ptrs, lens):
            assert self.o.push(C.string_at(p, n)) == 0, self.o.error()

    def flush(self):
        pass


class SplitOps:
    """numpy restatement of dml_shard_split (stable per-owner partition, dest-major)."""

    def split(self, fmt, cols, total_rows, world, ptrs, lens, out_ptr, out_cap, stream):
        from distml_amd.datadesc import KeyRange
        parts = KeyRange(0, total_rows - 1).linearSplit(world)
        step = parts[0].size()
        stride = fmt.keySize + fmt.valueSize * cols
        recs = [np.frombuffer(C.string_at(p, n), np.uint8).reshape(-1, stride) for p, n in zip(ptrs, lens)]
        owners = [r[:, :4].copy().view("<i4").ravel() // step for r in recs]
        out = np.frombuffer((C.c_char * out_cap).from_address(out_ptr), np.uint8)
        off = 0
        for d in range(world):
            for r, o in zip(recs, owners):
                sel = r[o == d].reshape(-1)
                out[off:off + sel.size] = sel
                off += sel.size
        return [[int((o == d).sum()) for d in range(world)] for o in owners]


def _worker(rank, world, port, vt, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    import pyoracle
    from distml_amd.group import ShardGroup

    dist.init_process_group("gloo", rank=rank, world_size=world)
    fmt = _fmt(vt)
    init = _init(vt)
    holder = {}

    def factory():
        sh = holder["g"].shard
        return OracleStoreShard(pyoracle, fmt, sh, init[sh.firstKey:sh.lastKey + 1])

    class G(ShardGroup):
        def __init__(self, *a, **k):
            holder["g"] = self
            super().__init__(*a, **k)

    g = G(fmt, ROWS, COLS, rank, world, device=None, ops=SplitOps(), store_factory=factory, exchange_only=True)
    with pytest.raises(RuntimeError):
        g.push_full_range([], [])  # an exchange-only group holds no partial buffers
    keep = []  # push buffers stay allocated until flush() (the group's contract)
    for call in range(CALLS):
        bufs = [torch.from_numpy(b) for b in _buckets(vt, rank, call)]
        g.push_exchange([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
        keep.append(bufs)
    g.flush()
    del keep
    o = g.store.o
    np.save(os.path.join(out_dir, f"data{rank}.npy"), o.data)
    if fmt.adaGrad:
        np.save(os.path.join(out_dir, f"alpha{rank}.npy"), o.alpha)
        np.save(os.path.join(out_dir, f"delta{rank}.npy"), o.delta)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# world 4 and 8 (the driver's node sizes): linearSplit(8) of 97 rows is 7 shards of 13
# and a short last shard of 6
@pytest.mark.parametrize("world,vt", [(2, 1), (3, 1), (2, 0), (3, 0), (4, 1), (8, 1), (8, 0)])
def test_exchange_push_gloo_bit_exact(tmp_path, oracle, world, vt):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), vt, str(tmp_path)), nprocs=world, join=True)
    o = oracle.OracleStore(1, 0, vt, 0, ROWS - 1, COLS, 1, int(vt == 1))
    if vt == 1:
        o.set_alpha(*ADA)
    o.data[:] = _init(vt)
    for call in range(CALLS):
        for r in range(world):
            for b in _buckets(vt, r, call):
                assert o.push(b.tobytes()) == 0
    got = np.concatenate([np.load(tmp_path / f"data{r}.npy") for r in range(world)])
    assert got.tobytes() == o.data.tobytes()
    if vt == 1:
        for name, ref in (("alpha", o.alpha), ("delta", o.delta)):
            g = np.concatenate([np.load(tmp_path / f"{name}{r}.npy") for r in range(world)])
            assert g.tobytes() == ref.tobytes()
        assert (o.delta > 1.0).any()  # the alpha update ran
