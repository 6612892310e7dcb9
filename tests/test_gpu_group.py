"""GPU, multi-process: ShardGroup's full-range push path on the real HIP kernels.

World 2 and 3 ranks share cuda:0, and the reduce-scatter runs over gloo. The
default ShardGroup reduce-scatter under gloo copies the partial to the host,
all_reduces it and copies the rank's chunk back. This exercises everything
except RCCL itself: the piecewise pre-reduce with its [rank][row] row map, the
padding rows of linearSplit's short last shard, the comm-stream ordering and
the owner apply. RCCL needs one GPU per rank, so its reduce-scatter is covered
only at world 1 (tests/test_gpu_parity.py) and by bench.py at N>1.

Tolerance as in tests/test_group_gloo.py: fp32 within 2(n-1)2^-24 sum|terms| of
the sequential oracle, and within 1e-6 relative (to sum|terms|) of the exact sum;
int32 exact.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _buckets(pyoracle, vt, rank, W, rows, cols, call=0):
    # multipliers coprime with 1000: every push lists each row once, in a permuted order
    # (push 0 ascending); call 2: rank 0's push 0 has two records swapped where the
    # speculative pre-reduce's sample cannot see them (its pieces fail verification and
    # the call re-runs with the key index; the sums are unchanged)
    out = [pyoracle.synth_dense_bucket(0, vt, 0, rows, rows, cols, 1000 * call + 100 * rank + b,
                                       (1, 3, 7, 9, 11)[b % 5], 13 * b) for b in range(W)]
    if call == 2 and rank == 0:
        sampled = {t * (rows - 1) // 31 for t in range(32)} | {pyoracle.splitmix64(t) % rows for t in range(32, 64)}
        free = sorted(set(range(rows)) - sampled)
        rec = out[0].reshape(rows, -1)
        i, j = free[len(free) // 2], free[len(free) // 2 + 1]
        rec[[i, j]] = rec[[j, i]]
    return out


def _asc_buckets(pyoracle, vt, rank, W, rows, cols, call=0):
    """W full-range pushes listing every row in ascending order (record r = row r)."""
    return [pyoracle.synth_dense_bucket(0, vt, 0, rows, rows, cols, 1000 * call + 100 * rank + b + 7, 1, 0)
            for b in range(W)]


def _init(vt, rows, cols):
    rng = np.random.default_rng(5)
    dt = {0: np.int32, 1: np.float32}[vt]
    return (rng.integers(50, 60, size=(rows, cols)) if vt == 0 else rng.standard_normal((rows, cols))).astype(dt)


def _worker(rank, world, port, vt, rows, cols, W, pieces, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    import pyoracle
    from distml_amd.datadesc import DataDesc
    from distml_amd.group import ShardGroup

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fmt = DataDesc(1, 0, vt)
    g = ShardGroup(fmt, rows, cols, rank, world, device=0, pieces=pieces)
    sh = g.shard
    g.store.load_values(_init(vt, rows, cols)[sh.firstKey:sh.lastKey + 1])
    keep = []
    pipelined = g.step_rows % pieces == 0
    for call in range(CALLS):  # back to back: workspaces and kept slot tables are reused
        bufs = [torch.from_numpy(b).cuda() for b in _buckets(pyoracle, vt, rank, W, rows, cols, call)]
        keep.append(bufs)
        torch.cuda.synchronize()
        g.push_full_range([b.data_ptr() for b in bufs], [b.numel() for b in bufs],
                          torch.cuda.current_stream().cuda_stream)
    g.flush()
    if pipelined and cols % 4 == 0:
        st = g.prereduce_stats()
        assert st["spec_chunks"] == CALLS and st["spec_reruns"] == (1 if rank == 0 else 0), st
    np.save(os.path.join(out_dir, f"shard{rank}.npy"), g.store.values())
    with open(os.path.join(out_dir, f"path{rank}.txt"), "w") as f:
        f.write("pipelined" if pipelined else "plain")
    g.store.close()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CALLS = 4


# (world, vt, rows, pieces): step_rows = ceil-ish linearSplit step
#   2, 1000 rows -> step 500, pieces 4: pipelined, no padding
#   3, 1000 rows -> step 334, pieces 2: pipelined, last shard 332 rows (2 padding rows)
#   3, 1000 rows -> step 334, pieces 4: 334 % 4 != 0 -> one-shot pre-reduce path
#   2, 1000 rows int32, pieces 4: exact
#   cols 64: the speculative pre-reduce (whole vectors); 67: ragged rows, key index
@pytest.mark.parametrize("world,vt,rows,pieces,path,cols", [
    (2, 1, 1000, 4, "pipelined", 67), (3, 1, 1000, 2, "pipelined", 67), (3, 1, 1000, 4, "plain", 67),
    (2, 0, 1000, 4, "pipelined", 67), (2, 1, 1000, 1, "pipelined", 64), (3, 0, 1000, 2, "pipelined", 64)])
def test_shard_group_hip_multiprocess(tmp_path, oracle, world, vt, rows, pieces, path, cols):
    """ShardGroup.push_full_range with the HIP kernels at world 2-3 (ranks share cuda:0,
    gloo reduce-scatter): four calls back to back; call 2 has rank 0 fail the
    speculative pre-reduce's verification (re-run exactly)."""
    import torch.multiprocessing as mp
    W = 5
    mp.spawn(_worker, args=(world, _free_port(), vt, rows, cols, W, pieces, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"path{r}.txt").read_text() == path
    got = np.concatenate([np.load(tmp_path / f"shard{r}.npy") for r in range(world)]).reshape(rows, cols)
    init = _init(vt, rows, cols)
    o = oracle.OracleStore(1, 0, vt, 0, rows - 1, cols)
    o.data[:] = init
    all_b = [b for c in range(CALLS) for r in range(world) for b in _buckets(oracle, vt, r, W, rows, cols, c)]
    for b in all_b:
        assert o.push(b.tobytes()) == 0
    if vt == 0:
        assert np.array_equal(got, o.data)
        return
    check_full_range(got, o, init, all_b, rows, cols, f"torch group world {world} pieces {pieces} cols {cols}")


def check_full_range(got, o, init, all_b, rows, cols, what="full range"):
    """fp32 sharded sums against the sequential oracle `o` (kat.rs_parity)."""
    import kat
    return kat.rs_parity(got, o.data, init, [b.tobytes() for b in all_b], cols, what)


# ---------------------------------------------------------------- exact exchange path
XR, XC, XW = 2000, 200, 4
XADA = (0.025, 0.0001, 1.5)


# back-to-back exchange calls, no flush between them (the pipelined path); the pooled
# receive buffers are reused from the third call on, after the store retired the call
# that read them (call 1 repeats a row: its chunk replays that row at retire)
XCALLS = 4


def _xbuckets(vt, rank, call=0, repeat=True):
    from distml_amd import encode_matrix_push
    out = []
    for b in range(XW):
        rng = np.random.default_rng(500 * rank + 50 * call + b)
        keys = rng.permutation(XR)[: rng.integers(XR // 4, XR)]
        if repeat and call == 1 and b == 0 and rank == 0:
            keys[5] = keys[17]  # one row listed twice (the exact replay)
        vals = ((rng.standard_normal((len(keys), XC)) * 0.6).astype(np.float32) if vt == 1
                else rng.integers(-2, 3, size=(len(keys), XC)).astype(np.int32))
        out.append(np.frombuffer(encode_matrix_push(keys, vals, 0, vt), np.uint8).copy())
    return out


def _xworker(rank, world, port, vt, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    from distml_amd.datadesc import DataDesc
    from distml_amd.group import ShardGroup

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fmt = DataDesc(1, 0, vt, False, True, vt == 1)
    g = ShardGroup(fmt, XR, XC, rank, world, device=0, exchange_only=(world == 3))  # no partial buffers
    sh = g.shard
    g.store.load_values(_init(vt, XR, XC)[sh.firstKey:sh.lastKey + 1])
    if vt == 1:
        g.store.setAlpha(*XADA)
    keep = []  # push buffers stay allocated until flush() (the group's contract)
    for call in range(XCALLS):
        bufs = [torch.from_numpy(b).cuda() for b in _xbuckets(vt, rank, call)]
        torch.cuda.synchronize()
        g.push_exchange([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
        keep.append(bufs)
    g.flush()
    del keep
    np.save(os.path.join(out_dir, f"data{rank}.npy"), g.store.values())
    if vt == 1:
        a, d = g.store.adagrad_state()
        np.save(os.path.join(out_dir, f"alpha{rank}.npy"), a)
        np.save(os.path.join(out_dir, f"delta{rank}.npy"), d)
        np.save(os.path.join(out_dir, f"md{rank}.npy"), np.array(g.store.maxDelta(), np.float64))
    g.store.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,vt", [(2, 1), (3, 1), (2, 0)])
def test_exchange_hip_multiprocess(tmp_path, oracle, world, vt):
    """push_exchange with the real dml_shard_split and HIP stores (ranks share cuda:0,
    all-to-all over gloo through the host), four calls back to back without a flush:
    bit-exact against one oracle store fed every call's pushes, rank-major per call; each shard's maxDelta against an oracle
    shard fed the same pushes restricted to its keys."""
    import torch.multiprocessing as mp
    mp.spawn(_xworker, args=(world, _free_port(), vt, str(tmp_path)), nprocs=world, join=True)
    check_exchange(tmp_path, oracle, world, vt, lambda n, r: np.load(tmp_path / f"{n}{r}.npy"))


def check_exchange(tmp_path, oracle, world, vt, load):
    """Exchange-path shards (load(name, rank): data / alpha / delta / md) bit-exact against
    one oracle store fed every call's pushes rank-major, maxDelta per shard."""
    from distml_amd.datadesc import KeyRange
    init = _init(vt, XR, XC)
    allb = [b for call in range(XCALLS) for r in range(world) for b in _xbuckets(vt, r, call)]
    o = oracle.OracleStore(1, 0, vt, 0, XR - 1, XC, 1, int(vt == 1))
    if vt == 1:
        o.set_alpha(*XADA)
    o.data[:] = init
    for b in allb:
        assert o.push(b.tobytes()) == 0
    got = np.concatenate([load("data", r) for r in range(world)]).reshape(XR, XC)
    assert got.tobytes() == o.data.tobytes()
    if vt != 1:
        return
    for name, ref in (("alpha", o.alpha), ("delta", o.delta)):
        g = np.concatenate([load(name, r) for r in range(world)]).reshape(XR, XC)
        assert g.tobytes() == ref.tobytes()
    for r, sh in enumerate(KeyRange(0, XR - 1).linearSplit(world)):
        so = oracle.OracleStore(1, 0, 1, sh.firstKey, sh.lastKey, XC, 1, 1)
        so.set_alpha(*XADA)
        so.data[:] = init[sh.firstKey:sh.lastKey + 1]
        for b in allb:
            rec = b.reshape(-1, 4 + 4 * XC)
            k = rec[:, :4].copy().view("<i4").ravel()
            assert so.push(rec[(k >= sh.firstKey) & (k <= sh.lastKey)].tobytes()) == 0
        assert tuple(load("md", r).tolist()) == tuple(float(x) for x in so.max_delta())


# ---------------------------------------------------------------- two-moment AdaGrad path
def _mworker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    from distml_amd.datadesc import DataDesc
    from distml_amd.group import ShardGroup

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fmt = DataDesc(1, 0, 1, False, True, True)
    g = ShardGroup(fmt, XR, XC, rank, world, device=0, exchange_only=True)
    sh = g.shard
    g.store.load_values(_init(1, XR, XC)[sh.firstKey:sh.lastKey + 1])
    g.store.setAlpha(*XADA)
    keep = []
    for call in range(XCALLS):
        bufs = [torch.from_numpy(b).cuda() for b in _xbuckets(1, rank, call, repeat=False)]
        torch.cuda.synchronize()
        g.push_moments([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
        keep.append(bufs)
    g.flush()
    np.save(os.path.join(out_dir, f"data{rank}.npy"), g.store.values())
    a, d = g.store.adagrad_state()
    np.save(os.path.join(out_dir, f"alpha{rank}.npy"), a)
    np.save(os.path.join(out_dir, f"delta{rank}.npy"), d)
    g.store.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_moments_hip_multiprocess(tmp_path, oracle, world):
    """ShardGroup.push_moments (the two-moment AdaGrad path) with the HIP kernels at
    world 2-3 (ranks share cuda:0, gloo reduce-scatter), four calls of key-subset
    pushes: within 1e-6 of one oracle store fed every call's pushes, rank-major."""
    import torch.multiprocessing as mp
    import kat
    mp.spawn(_mworker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    init = _init(1, XR, XC)
    allb = [b for call in range(XCALLS) for r in range(world) for b in _xbuckets(1, r, call, repeat=False)]
    o = oracle.OracleStore(1, 0, 1, 0, XR - 1, XC, 1, 1)
    o.set_alpha(*XADA)
    o.data[:] = init
    for b in allb:
        assert o.push(b.tobytes()) == 0
    cat = {n: np.concatenate([np.load(tmp_path / f"{n}{r}.npy") for r in range(world)]).reshape(XR, XC)
           for n in ("data", "alpha", "delta")}
    kat.moments_within(cat["data"], cat["alpha"].astype(np.float64), cat["delta"].astype(np.float64), o, init,
                       [b.tobytes() for b in allb], XC, f"world {world}")


# ---------------------------------------------------------------- local failure, torch binding
def _fworker(rank, world, port, rows, cols, W, out_dir, mode="verify"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    import pyoracle
    from distml_amd.datadesc import DataDesc
    from distml_amd.group import HipOps, ShardGroup

    class FailOnce(HipOps):
        """rank 0's verdict of its second call fails, as a local HIP error would"""
        n = 0

        def verify(self, h):
            FailOnce.n += 1
            if mode == "verify" and rank == 0 and FailOnce.n == 2:
                raise RuntimeError("injected verify failure")
            return super().verify(h)

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = ShardGroup(DataDesc(1, 0, 0), rows, cols, rank, world, device=0, ops=FailOnce())
    sh = g.shard
    g.store.load_values(_init(0, rows, cols)[sh.firstKey:sh.lastKey + 1])
    keep, errors = [], []
    for call in range(CALLS):
        bufs = [torch.from_numpy(b).cuda() for b in _buckets(pyoracle, 0, rank, W, rows, cols, call)]
        keep.append(bufs)
        torch.cuda.synchronize()
        lens = [b.numel() for b in bufs]
        if mode == "begin" and rank == 0 and call == 1:
            lens[0] -= 1  # a ragged push: begin_ctx fails before any piece
        try:
            g.push_full_range([b.data_ptr() for b in bufs], lens, torch.cuda.current_stream().cuda_stream)
        except Exception:
            errors.append(call)
    g.flush()
    np.save(os.path.join(out_dir, f"shard{rank}.npy"), g.store.values())
    np.save(os.path.join(out_dir, f"err{rank}.npy"), np.array(errors, np.int64))
    g.store.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["verify", "begin"])
def test_shard_group_local_failure_keeps_collectives(tmp_path, oracle, mode):
    """ShardGroup (torch binding) at world 2: rank 0's call 1 fails locally — its verdict
    (raised at call 2, which finishes call 1) or its begin_ctx on a ragged
    push (raised at call 1 itself). Rank 0 still enters call 1's
    reduce-scatter with a zeroed partial and skips its own apply; nobody hangs. int32,
    exact: rank 1's shard lacks only rank 0's call-1 pushes, rank 0's lacks all of call 1."""
    import torch.multiprocessing as mp
    from distml_amd.datadesc import KeyRange
    world, rows, cols, W = 2, 1000, 64, 3
    mp.spawn(_fworker, args=(world, _free_port(), rows, cols, W, str(tmp_path), mode), nprocs=world, join=True)
    assert np.load(tmp_path / "err0.npy").tolist() == ([2] if mode == "verify" else [1])
    assert np.load(tmp_path / "err1.npy").tolist() == []
    init = _init(0, rows, cols)
    for r, sh in enumerate(KeyRange(0, rows - 1).linearSplit(world)):
        o = oracle.OracleStore(1, 0, 0, 0, rows - 1, cols)
        o.data[:] = init
        for c in range(CALLS):
            for q in range(world):
                if c == 1 and (r == 0 or q == 0):
                    continue
                for b in _buckets(oracle, 0, q, W, rows, cols, c):
                    assert o.push(b.tobytes()) == 0
        got = np.load(tmp_path / f"shard{r}.npy").reshape(-1, cols)
        assert np.array_equal(got, o.data[sh.firstKey:sh.lastKey + 1]), r
