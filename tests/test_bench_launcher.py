"""bench.py's own rank launcher: `python bench.py --gpus N` with no
WORLD_SIZE starts its N rank processes itself and prints rank 0's one JSON line.
Rehearsed on CPU with --launcher-check: the same env, 127.0.0.1 rendezvous, barrier
and max-over-ranks as the GPU run, over gloo (no GPU call)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launcher-check"],
                          env=env, capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_bench_self_launch_ranks(n):
    r = _run(n)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks_seen"] == n and d["local_rank"] == 0
    # max over ranks: the slowest rank sleeps 0.02 * n s before the barrier
    assert d["value"] >= 0.02 * n - 1e-3


def test_bench_launcher_propagates_failure():
    """A failing rank fails the launch (non-zero exit) instead of hanging."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "4"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0


def test_hbm_footprint_check():
    """bench.py refuses (exit 3, with a message) a leg whose per-rank HBM footprint
    exceeds the device before it allocates anything."""
    sys.path.insert(0, ROOT)
    import bench

    class NoGpu:  # get_device_properties fails without a GPU: the 288 GB spec applies
        class cuda:
            @staticmethod
            def current_device():
                raise RuntimeError("no GPU")

    bench.hbm_check(NoGpu, "fits", {"pushes": 128.6e9, "store": bench.store_bytes(10_000_000, 200, 4, spec=True)})
    with pytest.raises(SystemExit) as ei:
        bench.hbm_check(NoGpu, "too big", {"pushes": 40 * 8.04e9})
    assert ei.value.code == 3
    # the config-4 leg at N = 8: 16 pushes of the full model per rank + the sharded path's buffers
    s4 = bench.store_bytes(1_250_000, 200, 4, spec=True) + bench.group_bytes(8, 10_000_000, 200, 4)
    assert 16 * 10_000_000 * 804 + s4 < 0.97 * bench.HBM_BYTES


@pytest.mark.parametrize("mode", ["raise", "hang", "ok"])
def test_guarded_leg_keeps_the_line(mode):
    """bench.guarded_leg: a secondary leg (the native group at N > 1) that raises or
    never returns costs only itself — rank 0 prints the line so far with the leg's
    error and the rank exits 0; a leg that returns is reported as is."""
    code = f"""
import json, sys, time
sys.path.insert(0, {ROOT!r})
import bench
class Ctx: rank = 0
def leg():
    if {mode!r} == "raise": raise RuntimeError("boom")
    if {mode!r} == "hang": time.sleep(30)
    return {{"value": 1.0}}
line = {{"metric": "m", "value": 5.0}}
line["native_group"] = bench.guarded_leg(Ctx(), line, sys.stdout, "native_group", leg, seconds=1.0)
print(json.dumps(line), flush=True)
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["value"] == 5.0
    if mode == "ok":
        assert d["native_group"] == {"value": 1.0}
    else:
        assert "error" in d["native_group"] and ("boom" in d["native_group"]["error"] or "within" in d["native_group"]["error"])


class _FakeCuda:
    def __init__(self, free, total):
        self._m = (free, total)

    def mem_get_info(self):
        return self._m


class _FakeCtx:
    """bench.Ctx's surface c4_fit_rows uses: torch.cuda.mem_get_info, world and a max
    over ranks (here: over the other ranks' values given up front)."""

    def __init__(self, free, total, world=1, others=()):
        self.torch = type("T", (), {"cuda": _FakeCuda(free, total)})()
        self.world, self._others = world, list(others)

    def max(self, x):
        return max([x] + self._others)


def test_config4_w32_rows_fit_and_agree():
    """The config-4 W = 32 leg's model size (bench.c4_fit_rows): whole 100 000s, at most
    10 M, its pushes + store (+ group buffers at N > 1) within the free HBM less the 1/8
    headroom the store keeps before it allocates its speculative buffer (dml_store.hip), and
    the same on every rank (the smallest fit: a different size per rank would desynchronise
    the collectives)."""
    sys.path.insert(0, ROOT)
    import bench
    total = 309 * 2**30
    for world in (1, 2, 8):
        free = total - 3 * 2**30
        rows = bench.c4_fit_rows(_FakeCtx(free, total, world), 32)
        assert rows % 100_000 == 0 and 0 < rows <= bench.C4_ROWS
        per_row = 32 * 804 + 2 * 800 + 3 * bench.WS_BYTES_PER_ROW
        if world == 1:
            assert rows * per_row <= 0.97 * free - total / 8
            assert (rows + 100_000) * per_row > 0.97 * free - total / 8  # the most that fit
        assert bench.c4_fit_rows(_FakeCtx(free, total, world), 8) == bench.C4_ROWS  # W = 8 fits at 10 M
    # another rank with less free memory settles the size for all
    small = bench.c4_fit_rows(_FakeCtx(200 * 2**30, total, 2), 32)
    assert bench.c4_fit_rows(_FakeCtx(300 * 2**30, total, 2, others=[-small]), 32) == small


def test_push_buffers_layouts():
    """bench.push_buffers: the config-4 legs' pushes as slices of one receive slab
    (consecutive, non-overlapping views of one allocation) or one allocation each
    (--push-layout separate), the same sizes either way."""
    sys.path.insert(0, ROOT)
    import bench
    import torch

    class _CpuTorch:  # torch with the device argument dropped (no GPU here)
        uint8 = torch.uint8

        @staticmethod
        def empty(n, dtype, device):
            return torch.empty(n, dtype=dtype)

    keep = bench.SLAB4[0]
    try:
        bench.SLAB4[0] = True
        bufs = bench.push_buffers(_CpuTorch, 4, 1000)
        assert [b.numel() for b in bufs] == [1000] * 4
        base = bufs[0].data_ptr()
        assert [b.data_ptr() - base for b in bufs] == [0, 1000, 2000, 3000]
        assert len({b.untyped_storage().data_ptr() for b in bufs}) == 1
        bench.SLAB4[0] = False
        bufs = bench.push_buffers(_CpuTorch, 4, 1000)
        assert [b.numel() for b in bufs] == [1000] * 4
        assert len({b.untyped_storage().data_ptr() for b in bufs}) == 4
    finally:
        bench.SLAB4[0] = keep
