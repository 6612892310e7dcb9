"""GPU, multi-process: the native shard group (dml_group_*, what the JNI's
GpuShardGroup binds) at world 2-4, in torch-free worker processes
(tests/native_group_worker.py) — its N > 1 schedule: the padded
ncclReduceScatter slices, the grouped count exchange and all-to-all
(ncclSend/ncclRecv), the two-moment reduce-scatter, buffer rotation over
back-to-back calls, a failed speculation, a short last shard (1000 rows over 3
or 4 ranks) and a local failure on one rank.

RCCL refuses two ranks on one GPU, so the ranks run the library's unchanged
nccl* calls against tests/rccl_double (a test-only stand-in over host shared
memory, loaded before libdistml_ps.so). test_native_group_rccl_all_devices runs
the same cases over the real RCCL, one GPU per rank, where the box has more than
one GPU (skipped on one).

Checks as tests/test_gpu_group.py: fp32 within the reduce-scatter bound of
DESIGN.md §2 (check_full_range), int32 and the exchange path bit-exact, the
two-moment path within 1e-6 (kat.moments_within).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import kat
import test_gpu_group as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "native_group_worker.py")
DOUBLE = os.path.join(ROOT, "tests", "rccl_double", "librccl_double.so")
pytestmark = pytest.mark.gpu


# Every collective of the stand-in runs this long after its inputs are ready (helper
# thread, asynchronous to the caller's streams): a stream dependency the library
# forgets shows up as wrong sums.
DELAY_US = 20000


def run_ranks(tmp_path, world, case, double=True, delay_us=DELAY_US, **kw):
    """Start `world` workers, wait for all, return their JSON lines (rank order)."""
    uid = tmp_path / f"uid_{case}"
    if double:
        # the stand-in's id names its shared-memory segment (rccl_double.cc's format);
        # written here without loading the stand-in, whose HIP runtime (/opt/rocm) must
        # not join torch's in this process
        name = ("dml-rccl-double:/dmlrccl_" + os.urandom(12).hex()).encode()
        uid.write_bytes(name + b"\0" * (128 - len(name)))
    args = [f"--{k.replace('_', '-')}={v}" for k, v in kw.items()]
    env = dict(os.environ, DML_RCCL_DOUBLE_DELAY_US=str(delay_us))
    procs = []
    for r in range(world):
        cmd = [sys.executable, "-u", WORKER, f"--world={world}", f"--rank={r}", f"--uid-file={uid}",
               f"--case={case}", f"--out={tmp_path}", f"--device={0 if double else r}"] + args
        procs.append(subprocess.Popen(cmd + (["--double"] if double else []), stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, env=env))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            assert p.returncode == 0, f"rank {procs.index(p)} rc {p.returncode}:\n{e[-3000:]}"
            outs.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for d in outs:
        assert "libdistml_ps" in d["libs"], d
        if double:
            assert d["double_calls"] > 0, d  # the collectives ran through the stand-in
            # the communicator pins RCCL's channel count (ncclCommInitRankConfig)
            assert d["ctas"] == [128, 128], d
    return outs


def shards(tmp_path, case, world, name="data", shape=None):
    a = np.concatenate([np.load(tmp_path / f"{case}_{r}.npz")[name] for r in range(world)])
    return a.reshape(shape) if shape else a


def full_expected(oracle, vt, world, rows, cols, W, calls, skip=lambda r, c: False):
    init = G._init(vt, rows, cols)
    o = oracle.OracleStore(1, 0, vt, 0, rows - 1, cols)
    o.data[:] = init
    all_b = [b for c in range(calls) for r in range(world) if not skip(r, c)
             for b in G._buckets(oracle, vt, r, W, rows, cols, c)]
    for b in all_b:
        assert o.push(b.tobytes()) == 0
    return o, init, all_b


@pytest.mark.parametrize("world,vt,rows,cols,pieces", [
    (2, 1, 1000, 64, 1), (3, 1, 1000, 64, 2), (4, 1, 1000, 67, 1), (2, 0, 1000, 64, 4), (3, 0, 1000, 67, 1)])
def test_native_group_full_range(tmp_path, oracle, world, vt, rows, cols, pieces):
    """dml_group_push_full_range at world 2-4 (1000 rows: step 334 / 250 at world 3 / 4,
    the last shard short by 2 rows at world 3), four calls back to back; call 2 fails
    rank 0's speculation (exact re-run). fp32 within the bound, int32 exact."""
    W = 5
    run_ranks(tmp_path, world, "full", vt=vt, rows=rows, cols=cols, pushes=W, pieces=pieces)
    got = shards(tmp_path, "full", world, shape=(rows, cols))
    o, init, all_b = full_expected(oracle, vt, world, rows, cols, W, G.CALLS)
    if cols % 4 == 0:  # whole 16-B vectors: the speculative pre-reduce runs
        for r in range(world):
            st = np.load(tmp_path / f"full_{r}.npz")["stats"].tolist()
            assert st[:2] == [G.CALLS, 1 if r == 0 else 0], (r, st)
    if vt == 0:
        assert np.array_equal(got, o.data)
    else:
        G.check_full_range(got, o, init, all_b, rows, cols, f"native world {world} pieces {pieces} cols {cols}")


# (world, vt, rows, pieces, ident): 200 columns (800-B rows, the flat kernels, 10 rows per
# k_flat_ident wave); 1198 rows over 3 ranks: step 400, the last shard 2 rows short;
# pieces 2: 200-row blocks; 999 rows over 2: step 500, pieces 4: 125-row blocks, which a
# 10-row wave would straddle, so the pieces fall back to k_reduce_flat
@pytest.mark.parametrize("world,vt,rows,pieces,ident", [
    (3, 1, 1198, 1, True), (3, 0, 1198, 2, True), (2, 1, 999, 4, False)])
def test_native_group_ascending_flat_ident(tmp_path, oracle, world, vt, rows, pieces, ident):
    """full-range calls whose pushes all list the rows in ascending order at a
    flat width take the all-identity kernel in the pre-reduce pieces (row map: strided
    row blocks, [rank][row] output, the short last shard's padding rows) — asserted
    through the pre-reduce counters — or, where a wave would straddle two row blocks,
    k_reduce_flat. int32 bit-exact, fp32 within the reduce-scatter bound (kat.rs_parity)."""
    cols, W = 200, 4
    run_ranks(tmp_path, world, "asc", vt=vt, rows=rows, cols=cols, pushes=W, pieces=pieces)
    for r in range(world):
        st = np.load(tmp_path / f"asc_{r}.npz")["stats"].tolist()
        assert st[:2] == [G.CALLS, 0], (r, st)
        assert st[2] == (G.CALLS * pieces if ident else 0), (r, st)
    got = shards(tmp_path, "asc", world, shape=(rows, cols))
    init = G._init(vt, rows, cols)
    o = oracle.OracleStore(1, 0, vt, 0, rows - 1, cols)
    o.data[:] = init
    all_b = [b for c in range(G.CALLS) for r in range(world) for b in G._asc_buckets(oracle, vt, r, W, rows, cols, c)]
    for b in all_b:
        assert o.push(b.tobytes()) == 0
    if vt == 0:
        assert np.array_equal(got, o.data)
    else:
        G.check_full_range(got, o, init, all_b, rows, cols, f"native ascending world {world} pieces {pieces}")


@pytest.mark.parametrize("world,vt", [(2, 1), (3, 1), (4, 1), (3, 0)])
def test_native_group_exchange(tmp_path, oracle, world, vt):
    """dml_group_push_exchange at world 2-4: split, grouped count exchange, all-to-all,
    owner apply in rank-major push order; four calls back to back without a flush
    (the double-buffered send / receive sets rotate; call 1 repeats a row): data,
    alpha, delta and every shard's maxDelta bit-exact against the oracle."""
    run_ranks(tmp_path, world, "exchange", vt=vt)
    G.check_exchange(tmp_path, oracle, world, vt,
                     lambda n, r: np.load(tmp_path / f"exchange_{r}.npz")[n if n != "md" else "md"])


@pytest.mark.parametrize("world", [2, 3, 4])
def test_native_group_moments(tmp_path, oracle, world):
    """dml_group_push_moments at world 2-4: Σu and Σu² reduce-scattered, the owner's
    AdaGrad apply; four calls: within 1e-6 of the sequential oracle."""
    run_ranks(tmp_path, world, "moments")
    init = G._init(1, G.XR, G.XC)
    allb = [b for call in range(G.XCALLS) for r in range(world) for b in G._xbuckets(1, r, call, repeat=False)]
    o = oracle.OracleStore(1, 0, 1, 0, G.XR - 1, G.XC, 1, 1)
    o.set_alpha(*G.XADA)
    o.data[:] = init
    for b in allb:
        assert o.push(b.tobytes()) == 0
    cat = {n: shards(tmp_path, "moments", world, n, (G.XR, G.XC)) for n in ("data", "alpha", "delta")}
    kat.moments_within(cat["data"], cat["alpha"].astype(np.float64), cat["delta"].astype(np.float64), o, init,
                       [b.tobytes() for b in allb], G.XC, f"native world {world}")


@pytest.mark.parametrize("world", [2, 3])
def test_native_group_local_after_full_range(tmp_path, world):
    """dml_group_push_local right after a full-range call, no flush between:
    the local push subtracts init + every rank's sum from the rank's rows, so the int32
    counters end at exactly 0 only if the store applies it after the full-range call;
    before it, they would go negative and the store would raise."""
    outs = run_ranks(tmp_path, world, "local", rows=1000, cols=64, pushes=3)
    assert all(not d["errors"] for d in outs), outs
    assert not shards(tmp_path, "local", world).any()


def test_native_group_local_failure_keeps_collectives(tmp_path, oracle):
    """A local failure on one rank (rank 0's verdict for call 1, injected) at world 3:
    rank 0 raises once, nobody waits for a collective it skipped, every rank finishes
    its calls. int32, exact: rank 0 contributed zeros to call 1's
    reduce-scatter and skipped its own apply of call 1."""
    world, rows, cols, W = 3, 1000, 64, 4
    outs = run_ranks(tmp_path, world, "fault", rows=rows, cols=cols, pushes=W)
    assert [len(d["errors"]) for d in outs] == [1, 0, 0], outs
    assert outs[0]["errors"][0][0] == 2 and "injected" in outs[0]["errors"][0][2], outs[0]
    from distml_amd.datadesc import KeyRange
    parts = KeyRange(0, rows - 1).linearSplit(world)
    o0, _, _ = full_expected(oracle, 0, world, rows, cols, W, G.CALLS, skip=lambda r, c: c == 1)
    on, _, _ = full_expected(oracle, 0, world, rows, cols, W, G.CALLS, skip=lambda r, c: (r, c) == (0, 1))
    for r, sh in enumerate(parts):
        got = np.load(tmp_path / f"fault_{r}.npz")["data"].reshape(-1, cols)
        want = (o0 if r == 0 else on).data[sh.firstKey:sh.lastKey + 1]
        assert np.array_equal(got, want), r


def test_native_group_begin_failure_keeps_collectives(tmp_path, oracle):
    """A call that fails in dml_prereduce_begin_ctx (rank 0's call 1: a ragged push) at
    world 3: it skipped the host wait for its buffer set's last apply, so
    its zero contribution orders after that apply on the device, and the set stays
    busy until the zero-contribution scatter has run: call 3 reuses it while the
    stand-in still delays call 1's scatter. Rank 0 raises at call 1; every shard exact."""
    world, rows, cols, W = 3, 1000, 64, 4
    outs = run_ranks(tmp_path, world, "beginfail", rows=rows, cols=cols, pushes=W)
    assert [len(d["errors"]) for d in outs] == [1, 0, 0], outs
    assert outs[0]["errors"][0][0] == 1 and outs[0]["errors"][0][1] == "ArrayIndexOutOfBoundsException", outs[0]
    from distml_amd.datadesc import KeyRange
    o0, _, _ = full_expected(oracle, 0, world, rows, cols, W, G.CALLS, skip=lambda r, c: c == 1)
    on, _, _ = full_expected(oracle, 0, world, rows, cols, W, G.CALLS, skip=lambda r, c: (r, c) == (0, 1))
    for r, sh in enumerate(KeyRange(0, rows - 1).linearSplit(world)):
        got = np.load(tmp_path / f"beginfail_{r}.npz")["data"].reshape(-1, cols)
        want = (o0 if r == 0 else on).data[sh.firstKey:sh.lastKey + 1]
        assert np.array_equal(got, want), r


def test_native_group_rccl_all_devices(tmp_path, oracle):
    """The same schedule over the system RCCL, one GPU per rank, at world = the box's
    GPU count (xGMI): full-range fp32 and int32, exchange (AdaGrad), moments."""
    import torch
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU: RCCL refuses two ranks per device (the stand-in tests cover N > 1)")
    world = min(n, 8)
    rows, cols, W = 1000, 64, 5
    for vt in (1, 0):
        run_ranks(tmp_path, world, "full", double=False, vt=vt, rows=rows, cols=cols, pushes=W)
        got = shards(tmp_path, "full", world, shape=(rows, cols))
        o, init, all_b = full_expected(oracle, vt, world, rows, cols, W, G.CALLS)
        if vt == 0:
            assert np.array_equal(got, o.data)
        else:
            G.check_full_range(got, o, init, all_b, rows, cols)
    run_ranks(tmp_path, world, "exchange", double=False, vt=1)
    G.check_exchange(tmp_path, oracle, world, 1, lambda n, r: np.load(tmp_path / f"exchange_{r}.npz")[n])


@pytest.mark.parametrize("world", [2, 3])
def test_native_group_through_jni(tmp_path, oracle, world):
    """The JNI's multi-GPU binding itself at world 2-3: GpuShardGroup's entry points in
    integration/jni/dml_jni.cc (nativeGroupCreate / nativeGroupPush mode 0 and 3 /
    nativeGroupFlush / nativeGroupStore) on the mock JNIEnv, in torch-free ranks over
    the RCCL stand-in; int32 full-range calls then a pushLocal of each rank's rows,
    every shard read back through nativeWriteAll (big-endian), exact."""
    rows, cols, W = 1000, 64, 3
    outs = run_ranks(tmp_path, world, "jni", rows=rows, cols=cols, pushes=W)
    assert all(not d["errors"] for d in outs), outs
    from distml_amd.datadesc import KeyRange
    o, _, _ = full_expected(oracle, 0, world, rows, cols, W, G.CALLS)
    for r, sh in enumerate(KeyRange(0, rows - 1).linearSplit(world)):
        got = np.load(tmp_path / f"jni_{r}.npz")["data"].reshape(-1, cols)
        assert np.array_equal(got, o.data[sh.firstKey:sh.lastKey + 1] + (r + 1)), r
