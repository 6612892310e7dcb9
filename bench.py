"""Benchmark: device-resident gradient-bucket reduce GiB/s (BASELINE.json metric).

N=1 (default) — config 2 of BASELINE.json: a 16 384 x 1 024 fp32 shard (64 MiB,
DataDesc MATRIX/INT/FLOAT dense) receives 32 pushes of 64 MiB each
([int32 key][1 024 x f32] x 16 384 records = 67 174 400 B), resident in HBM.
One step = dml_store_push_batch_device(32 pushes): slot-table reset, key
index kernel (side stream, overlapping the previous batch's reduce), the
ordered multi-push reduce kernel, the error check; the timed region ends with
flush() (every batch applied and error-checked) and a device synchronize.
Algorithmic bytes per step = 32 x 67 174 400 + 2 x 67 108 864 = 2 283 798 528.

N>1 (torchrun, one rank per GPU, RCCL) — weak scaling: every rank holds 32
full-range pushes of the same 64 MiB model, whose rows are linearSplit over
the N ranks; step = ordered pre-reduce of the 32 local pushes, RCCL
reduce-scatter of the partials, owner apply.

Also reported: the dominant kernel's HBM roofline (achieved from HIP events
around every k_reduce launch, on the store's stream) and the CPU baseline
(the oracle's restatement of FloatMatrixStore.updateRow, 1 thread, timed on
this host on the same pushes).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# One hardware queue per stream: the store (apply / index / copy), torch's default
# stream and the group path's index / comm streams each need their own queue, or
# HIP multiplexes them onto HIP's default 4 and work meant to overlap serializes
# (measured on the --group path: the next call's key index queued behind the pieces).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

ROWS, COLS, W = 16384, 1024, 32
REC = 4 + 4 * COLS
BUCKET = ROWS * REC                      # 67 174 400 B
SHARD = ROWS * COLS * 4                  # 67 108 864 B
HBM_PEAK_GBS = 8000.0                    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def perm_for(b: int):
    # even pushes list rows ascending (Java HashMap<Integer> order), odd ones a seeded permutation
    return (1, 0) if b % 2 == 0 else (((2 * b + 1) * 2654435761) % ROWS | 1, (b * 7919) % ROWS)


def make_buckets(L, torch, fmt, n, rows_total):
    st = torch.cuda.current_stream().cuda_stream
    bufs = []
    for b in range(n):
        t = torch.empty(rows_total * REC, dtype=torch.uint8, device="cuda")
        pa, pc = perm_for(b)
        rc = L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows_total, rows_total, COLS,
                                      1000 + b, pa % rows_total, pc % rows_total, C.c_void_p(st))
        assert rc == 0, rc
        bufs.append(t)
    torch.cuda.synchronize()
    return bufs


def cpu_baseline(budget_s: float = 12.0):
    """Oracle (C restatement of FloatMatrixStore.updateRow, single thread) on the
    same 32 x 64 MiB pushes, repeated until `budget_s` of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    bufs = [pyoracle.synth_dense_bucket(0, 1, 0, ROWS, ROWS, COLS, 1000 + b, *perm_for(b)) for b in range(W)]
    o = pyoracle.OracleStore(1, 0, 1, 0, ROWS - 1, COLS)
    o.synth_fill(7)
    reps, t0 = 0, time.perf_counter()
    while True:
        assert o.push_many(bufs, threads=1) == 0
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 50:
            break
    algo = W * BUCKET + 2 * SHARD
    return {"value": round(reps * algo / el / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"full config-2 workload (32 x 64 MiB pushes -> 16384x1024 fp32 shard) x{reps} reps, "
                      f"{el:.1f} s, oracle/dml_oracle.c single thread"}


def sparse_leg(L, torch, steps: int):
    """Config 3 (reported beside the headline): 1e9-dim fp32 FloatArrayStore shard
    (4 GB), 32 device-resident pushes x 1e6 unique keys ([int64 key][f32] = 12 B),
    ordered per-push scatter-add. Algorithmic bytes per step = 32 x 12e6 + 2 x 4 x 32e6."""
    from distml_amd import DataDesc, DataStore, KeyRange
    from distml_amd.store import DeviceBatch
    dim, nnz, w = 10**9, 10**6, 32
    fmt = DataDesc(DataDesc.DATA_TYPE_ARRAY, DataDesc.KEY_TYPE_LONG, DataDesc.ELEMENT_TYPE_FLOAT)
    store = DataStore(fmt, KeyRange(0, dim - 1))
    bufs = []
    st = torch.cuda.current_stream().cuda_stream
    for b in range(w):
        pa = (2 * b + 3) * 999_999_937 % dim
        while pa % 2 == 0 or pa % 5 == 0:
            pa += 1
        t = torch.empty(nnz * 12, dtype=torch.uint8, device="cuda")
        assert L.dml_synth_sparse_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, dim, nnz, 2000 + b, pa,
                                         (b * 12_345_701) % dim, C.c_void_p(st)) == 0
        bufs.append(t)
    torch.cuda.synchronize()
    batch = DeviceBatch([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
    for _ in range(max(2, steps)):  # warmup: as many untimed steps as timed ones
        store.pushDevice(batch)
    store.flush()
    store.set_timing(True)
    store.kernel_time(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        store.pushDevice(batch)
    store.flush()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k_ms, k_n = store.kernel_time(reset=True)
    algo = w * nnz * 12 + 2 * 4 * w * nnz
    out = {"workload": "config3: 1e9-dim fp32 array shard, 32 pushes x 1e6 unique int64 keys, ordered scatter-add",
           "value": round(steps * algo / el / 2**30, 2), "unit": "GiB/s (algorithmic)", "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 3), "algorithmic_bytes_per_step": algo,
           "apply_kernel_us_avg": round(k_ms / max(k_n, 1) * 1e3, 2), "apply_launches": k_n}
    store.close()
    del bufs
    return out


def stream_peaks(L, torch, nbytes: int = 1 << 31, reps: int = 5):
    """Measured streaming ceilings on this box, GB/s: best of `reps` runs of the
    library's 16-B nt-load kernels (dml_diag_stream) over `nbytes` — a pure read
    (k_reduce moves 97 % of its bytes as reads) and a copy (read + write counted).
    SURVEY §8(d) asks for fractions against both the spec and a measured peak."""
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    src.fill_(1)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for mode, name, moved in ((0, "read", nbytes), (1, "copy", 2 * nbytes)):
        best, ms = float("inf"), C.c_float()
        for _ in range(reps + 1):
            assert L.dml_diag_stream(mode, dst.data_ptr(), src.data_ptr(), nbytes, st, C.byref(ms)) == 0
            best = min(best, ms.value / 1e3)
        out[name] = moved / best / 1e9
    del src, dst
    return out


# ---------------------------------------------------------------- configs 4 and 5
# One GPU's shard of BASELINE.json configs 4 and 5 (8-GPU configs):
# the rows linearSplit(8) gives one rank, device-resident pushes of the named
# shapes, the store's ordered batch reduce. `python bench.py --config 5|4`.
SHARD_CONFIGS = {
    "5": dict(name="config5: LDA IntMatrixStore shard 125000x1000 int32 (negativity check), "
                   "32 pushes x 8192 distinct rows ([int32][1000 x int32])",
              rows=125_000, cols=1000, W=32, nrec=8192, vt=0, ada=None, seed0=4000, mult=331, init=11, steps=20),
    # config 4's metric is the plain sum (FloatMatrixStore), W = 8 and 32; AdaGrad is its variant
    "4": dict(name="config4: Word2Vec rows, FloatMatrixStore shard 1250000x200 fp32, 8 full-range pushes "
                   "([int32][200 x f32])",
              rows=1_250_000, cols=200, W=8, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919, init=13,
              steps=10),
    "4-32": dict(name="config4 (W=32): Word2Vec rows, FloatMatrixStore shard 1250000x200 fp32, 32 full-range pushes",
                 rows=1_250_000, cols=200, W=32, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919, init=13,
                 steps=5),
    "4-asc": dict(name="config4 with every push in ascending row order (Java HashMap<Integer> iteration): "
                       "FloatMatrixStore shard 1250000x200 fp32, 8 full-range pushes",
                  rows=1_250_000, cols=200, W=8, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919, init=13,
                  steps=10, asc=True),
    "4-256": dict(name="config4 shape probe: FloatMatrixStore shard 1250000x256 fp32 (whole 1-KiB rows), 8 full-range "
                       "pushes", rows=1_250_000, cols=256, W=8, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919,
                  init=13, steps=10),
    "4-ada": dict(name="config4 AdaGrad variant: FloatMatrixStoreAdaGrad shard 1250000x200 fp32 (data + alpha + "
                       "delta), 8 full-range pushes",
                  rows=1_250_000, cols=200, W=8, nrec=1_250_000, vt=1, ada=(0.025, 0.0001, 1.0), seed0=3000,
                  mult=7919, init=13, steps=5),
}


def _coprime(a, n):
    import math
    while math.gcd(a, n) != 1:
        a += 1
    return a


def _shard_perms(c):
    if c.get("asc"):
        return [(1, 0)] * c["W"]
    return [(_coprime((c["seed0"] + b) * 2654435761 % c["rows"] | 1, c["rows"]), b * c["mult"] % c["rows"])
            for b in range(c["W"])]


def shard_cpu_baseline(c, budget_s: float):
    """The oracle (1 thread) on the first pushes of the same workload (int32: each push
    alternating with its negation, as on the GPU, so counts stay >= 0)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    perms = _shard_perms(c)
    rows, cols, nrec = c["rows"], c["cols"], c["nrec"]
    host = [pyoracle.synth_dense_bucket(0, c["vt"], 0, rows, nrec, cols, c["seed0"] + b, *perms[b]) for b in range(4)]
    if c["vt"] == 0:
        negs = []
        for h in host:
            t = h.view(np.int32).reshape(nrec, 1 + cols).copy()
            t[:, 1:] = -t[:, 1:]
            negs.append(t.view(np.uint8).reshape(-1))
        host = [x for pair in zip(host, negs) for x in pair]
    o = pyoracle.OracleStore(1, 0, c["vt"], 0, rows - 1, cols, ada_grad=1 if c["ada"] else 0)
    if c["ada"]:
        o.set_alpha(*c["ada"])
    o.synth_fill(c["init"])
    nb, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        assert o.push(host[nb % len(host)]) == 0
        nb += 1
    el = time.perf_counter() - t0
    return {"value": round(nb * nrec * (4 + 4 * cols) / el / 2**30, 3), "unit": "GiB/s of push bytes", "cores": 1,
            "kind": "port", "sample": f"{nb} pushes of the same shapes in {el:.1f} s, oracle/dml_oracle.c"}


def run_shard_config(which: str, cpu_s: float, no_cpu: bool) -> dict:
    import torch
    from distml_amd import DataDesc, DataStore, KeyRange, _lib
    c = SHARD_CONFIGS[which]
    L = _lib.load()
    rows, cols, W, nrec = c["rows"], c["cols"], c["W"], c["nrec"]
    fmt = DataDesc(1, 0, c["vt"], False, True, c["ada"] is not None)
    store = DataStore(fmt, KeyRange(0, rows - 1), cols)
    if c["ada"]:
        store.setAlpha(*c["ada"])
    store.rand(c["init"])
    st = torch.cuda.current_stream().cuda_stream
    bufs = []
    for b, (pa, pc) in enumerate(_shard_perms(c)):
        t = torch.empty(nrec * (4 + 4 * cols), dtype=torch.uint8, device="cuda")
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows, nrec, cols, c["seed0"] + b,
                                        pa, pc, C.c_void_p(st)) == 0
        bufs.append(t)
    torch.cuda.synchronize()
    sets = [([b.data_ptr() for b in bufs], [b.numel() for b in bufs])]
    if c["vt"] == 0:  # alternate with the negated pushes: repeated steps keep the counts >= 0
        neg = []
        for b in bufs:
            t = b.clone().view(torch.int32).view(nrec, 1 + cols)
            t[:, 1:] = -t[:, 1:]
            neg.append(t.view(torch.uint8).view(-1))
        bufs = bufs + neg
        sets.append(([b.data_ptr() for b in neg], [b.numel() for b in neg]))
    torch.cuda.synchronize()
    # every push byte once + the touched shard rows read and written once
    # (AdaGrad: alpha and delta too)
    touched = rows if nrec >= rows else int(round(rows * (1 - (1 - nrec / rows) ** W)))
    algo = W * nrec * (4 + 4 * cols) + 2 * (3 if c["ada"] else 1) * 4 * cols * touched
    steps = c["steps"]
    for i in range(max(4, steps)):
        store.pushDevice(*sets[i % len(sets)])
    store.flush()
    store.set_timing(True)
    store.kernel_time(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        store.pushDevice(*sets[i % len(sets)])
    store.flush()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k_ms, k_n = store.kernel_time(reset=True)
    store.set_timing(False)
    assert store.error_state()[0] == 0, store.error_state()
    store.close()
    del bufs, sets
    torch.cuda.empty_cache()
    k_s = k_ms / max(k_n, 1) / 1e3
    line = {"metric": "device-resident push reduce GiB/s (one GPU's shard)", "value": round(steps * algo / el / 2**30, 1),
            "unit": "GiB/s", "n_gpus": 1, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
            "higher_is_better": True, "dtype": "i32" if c["vt"] == 0 else "f32", "data": "synthetic",
            "config": {"workload": c["name"], "rows": rows, "cols": cols, "pushes": W, "records_per_push": nrec,
                       "algorithmic_bytes_per_step": algo},
            "roofline": {"bound": "hbm", "achieved": round(algo / k_s / 1e9, 1) if k_n else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / k_s / 1e9 / HBM_PEAK_GBS, 4) if k_n else None,
                         "kernel_us_avg": round(k_s * 1e6, 1), "traffic": None}}
    if not no_cpu:
        line["cpu_baseline"] = shard_cpu_baseline(c, cpu_s)
    return line


def _pre_time(L, enable: bool, reset: bool):
    """Pre-reduce piece timing of the sharded path (dml_prereduce_timing / _kernel_time)."""
    ms, n = C.c_double(0.0), C.c_int64(0)
    assert L.dml_prereduce_kernel_time(C.byref(ms), C.byref(n), 1 if reset else 0) == 0
    assert L.dml_prereduce_timing(1 if enable else 0) == 0
    return ms.value, n.value


def load_traffic():
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~0.2 s of warmup and ~0.4 s timed at N=1: a few-ms window on a GPU that sat idle
    # through process start-up measured 5 % slow (clocks still ramping)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-timing", action="store_true", help="no kernel timing events in the timed region")
    ap.add_argument("--sparse-steps", type=int, default=20, help="config-3 sparse leg steps (0 = skip)")
    ap.add_argument("--pieces", type=int, default=4, help="pre-reduce row slices per call (sharded path)")
    ap.add_argument("--group", action="store_true",
                    help="use the sharded pre-reduce/reduce-scatter path even at N=1 (path check)")
    ap.add_argument("--config", choices=["2", "4", "4-32", "4-asc", "4-256", "4-ada", "5"], default="2",
                    help="2 = the headline (default); 4, 4-32, 4-ada, 5 = one GPU's shard of those 8-GPU configs")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline budget for --config 4/5")
    args = ap.parse_args()
    # stdout carries exactly the one JSON line: RCCL and other native libraries print
    # banners to fd 1 (e.g. "RCCL version : ..."), so fd 1 goes to stderr for the run
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.config != "2":
        print(json.dumps(run_shard_config(args.config, args.cpu_seconds, args.no_cpu)), file=out, flush=True)
        return

    import torch
    import torch.distributed as dist
    from distml_amd import DataDesc, DataStore, KeyRange, _lib
    from distml_amd.group import ShardGroup
    from distml_amd.store import DeviceBatch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif args.group:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
    L = _lib.load()
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_FLOAT)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    if world == 1 and not args.group:
        store = DataStore(fmt, KeyRange(0, ROWS - 1), COLS, device=local)
        store.rand(7)
        bufs = make_buckets(L, torch, fmt, W, ROWS)
        batch = DeviceBatch([b.data_ptr() for b in bufs], [b.numel() for b in bufs])

        def step():
            # async: ack once captured; the store keeps <= 2 batches in flight and the
            # key index of batch k+1 overlaps the reduce of batch k
            store.pushDevice(batch)

        def finish():
            store.flush()  # every pushed batch applied and error-checked
        timed_store = store
        algo_per_rank = W * BUCKET + 2 * SHARD
    else:
        group = ShardGroup(fmt, ROWS, COLS, rank, world, device=local, pieces=args.pieces)
        bufs = make_buckets(L, torch, fmt, W, ROWS)
        ptrs, lens = [b.data_ptr() for b in bufs], [b.numel() for b in bufs]
        st = torch.cuda.current_stream().cuda_stream

        def step():
            group.push_full_range(ptrs, lens, st)

        def finish():
            group.flush()
        timed_store = group.store
        algo_per_rank = W * BUCKET + 2 * group.shard.size() * COLS * 4

    sharded = not (world == 1 and not args.group)
    for _ in range(args.warmup):
        step()
    finish()
    timed_store.set_timing(not args.no_timing)
    timed_store.kernel_time(reset=True)
    if sharded and not args.no_timing:
        _pre_time(L, enable=True, reset=True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    finish()
    barrier()
    el = time.perf_counter() - t0
    k_ms, k_n = timed_store.kernel_time(reset=True)
    timed_store.set_timing(False)
    pre_ms, pre_n = _pre_time(L, enable=False, reset=True) if sharded else (0.0, 0)
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())

    total_bytes = algo_per_rank * world * args.steps
    value = total_bytes / el / 2**30
    line = {
        "metric": "device-resident gradient-bucket reduce GiB/s (dense fp32 + sparse scatter-add)",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "config2: dense fp32 reduce, 32 device-resident pushes x 64 MiB "
                               "([int32 key][1024 x f32] x 16384) -> 16384x1024 fp32 shard per model",
                   "pushes_per_gpu": W, "push_bytes": BUCKET, "model_rows": ROWS, "cols": COLS,
                   "parallelism": ("single shard" if world == 1 and not args.group
                                   else f"linearSplit({world}) + RCCL reduce-scatter"),
                   "algorithmic_bytes_per_step_per_gpu": algo_per_rank},
    }
    if rank == 0:
        if world == 1 and k_n > 0 and not args.group:
            avg_s = k_ms / k_n / 1e3
            achieved = algo_per_rank / avg_s / 1e9
            traffic = load_traffic()
            pk = stream_peaks(L, torch)
            line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                                "kernel": "k_reduce_rows<float,kAdd> (2 rows x 4 KiB per wave)", "avg_kernel_us": round(avg_s * 1e6, 2),
                                "launches": k_n, "measured_read_peak": round(pk["read"], 1),
                                "frac_of_measured_read": round(achieved / pk["read"], 4),
                                "measured_copy_peak": round(pk["copy"], 1)}
        elif pre_n > 0:
            # sharded path: the pre-reduce pieces (k_reduce_rows in pre-reduce mode) are the
            # dominant kernel; per call they read the W pushes and write the full-model partial
            pre_bytes = W * BUCKET + world * group.step_rows * COLS * 4
            calls = pre_n / args.pieces
            avg_s = pre_ms / calls / 1e3
            achieved = pre_bytes / avg_s / 1e9
            line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                                "kernel": f"k_reduce_rows pre-reduce ({args.pieces} pieces per call, rank 0)",
                                "avg_kernel_us": round(avg_s * 1e6, 2), "launches": pre_n,
                                "algorithmic_bytes_per_call": pre_bytes}
        if world == 1 and not args.group and args.sparse_steps > 0:
            del bufs
            line["sparse"] = sparse_leg(L, torch, args.sparse_steps)
        if world == 1 and not args.no_cpu and not args.group:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), file=out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
