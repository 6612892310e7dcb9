"""Benchmark: device-resident gradient-bucket reduce GiB/s (BASELINE.json metric).

Headline (every N) — config 2 of BASELINE.json: a 16 384 x 1 024 fp32 model
(64 MiB, DataDesc MATRIX/INT/FLOAT dense) receives 32 pushes of 64 MiB per GPU
([int32 key][1 024 x f32] x 16 384 records = 67 174 400 B), resident in HBM.
  N=1: one shard; one step = dml_store_push_batch_device(32 pushes): key index
       (side stream, overlapping the previous batch's reduce), the ordered
       multi-push reduce, the error check; the timed region ends with flush().
       Algorithmic bytes per step = 32 x 67 174 400 + 2 x 67 108 864.
  N>1: weak scaling, one process per GPU, RCCL: every rank holds 32 full-range
       pushes of the same model, whose rows are linearSplit over the N ranks
       (KeyRange.java:68-80); step = ordered pre-reduce of the 32 local pushes,
       RCCL reduce-scatter of the partials (pipelined in row slices), owner apply.

Legs reported in the same JSON line (same N, same process group):
  "config4": BASELINE config 4, Word2Vec rows 10M x 200 fp32 (8 GB model),
             W full-range pushes per GPU ([int32][200 x f32] = 804 B records);
             N=1 one store, N>1 linearSplit + pre-reduce + reduce-scatter
             (weak scaling: W pushes per GPU at every N).
  "config4_ada": config 4's AdaGrad variant (FloatMatrixStoreAdaGrad, 10M x 200:
             data, alpha, delta), W full-range pushes per GPU through the exact
             exchange path (split by owner, all-to-all, ordered owner apply; the
             reduce-scatter cannot reproduce AdaGrad's per-push updates).
  "config5": BASELINE config 5, LDA IntMatrixStore 1M x 1000 int32 (4 GB),
             32 pushes of 65 536 distinct vocabulary rows, split per shard the
             way the reference's client splits them (SparseMatrix.java:46-60),
             each shard's part applied by its owner with the negativity check
             (strong scaling: the model and the pushes are fixed, N shards).
  "sparse":  (N=1) config 3, 1e9-dim fp32 FloatArrayStore, 32 x 1e6 keys.
  "cpu_baseline": (N=1, rank 0) the oracle's restatement of
             FloatMatrixStore.updateRow on the same pushes, on this host's
             cores: one thread (the reference's one selector thread per PS)
             and all usable cores (row-partitioned).

Without a launcher (`python bench.py --gpus N`, WORLD_SIZE unset) the script
starts its N rank processes itself before any GPU call and prints rank 0's
line; under torchrun it reads RANK / LOCAL_RANK / WORLD_SIZE.

`--config 4|4-perm|4-32|4-256|4-ada|5` measures one GPU's shard of configs 4
and 5 (the per-shard kernel numbers DESIGN.md §7 quotes), N=1 only.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# HIP's default hardware queues (4 per process), as the PS JVM runs: the store and
# group paths measured the same at 4 and 8 (round 3).

METRIC = "device-resident gradient-bucket reduce GiB/s (dense fp32 + sparse scatter-add)"
ROWS, COLS, W = 16384, 1024, 32
REC = 4 + 4 * COLS
BUCKET = ROWS * REC                      # 67 174 400 B
SHARD = ROWS * COLS * 4                  # 67 108 864 B
HBM_PEAK_GBS = 8000.0                    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

C4_ROWS, C4_COLS = 10_000_000, 200       # Word2Vec rows (BASELINE config 4)
C5_ROWS, C5_COLS, C5_W, C5_NNZ = 1_000_000, 1000, 32, 65536  # LDA word-topic counts (config 5)
C5_TOPICS = 1000                         # LDA doc-topic totals (IntArrayStore, K topics)
SHUFFLE_ORDERS = 64                      # seeded push orders of the headline's arrival-order sub-line
RS_CHANNELS = 128                        # RCCL channels (CTAs) per collective


# ---------------------------------------------------------------- HBM footprint
HBM_BYTES = 288e9                        # MI355X HBM3E per GPU
WS_BYTES_PER_ROW = 64 * 4 + 4            # slot table row (kMaxW int32) + rowflag, per workspace


def hbm_check(torch, leg: str, parts: dict) -> None:
    """Fail fast (exit 3, with a message) when a leg's per-rank HBM footprint — the
    sum of `parts`, bytes — would not fit the device, before anything is allocated."""
    cap = HBM_BYTES
    try:
        cap = min(cap, float(torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory))
    except Exception:
        pass
    total = sum(parts.values())
    if total > 0.97 * cap:
        detail = ", ".join(f"{k} {v / 1e9:.1f} GB" for k, v in parts.items())
        sys.stderr.write(f"bench.py: leg {leg} needs {total / 1e9:.1f} GB of HBM per rank ({detail}); "
                         f"the device has {cap / 1e9:.1f} GB\n")
        raise SystemExit(3)


def store_bytes(rows: int, cols: int, vbytes: int, spec: bool = False, ada: bool = False) -> float:
    """A dml_store: the shard (+ its second buffer under speculation, + AdaGrad's alpha
    and delta) and the three-workspace ring."""
    arrays = 1 + (1 if spec else 0) + (2 if ada else 0)
    return arrays * rows * cols * vbytes + 3 * rows * WS_BYTES_PER_ROW


def group_bytes(world: int, rows: int, cols: int, vbytes: int) -> float:
    """ShardGroup's full-range path: two partial / receive sets and the pre-reduce context."""
    step = (rows - 1 + world) // world
    return 2 * world * step * cols * vbytes + 2 * step * cols * vbytes + 3 * rows * WS_BYTES_PER_ROW


# ---------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv) -> int:
    """Start n rank processes of this script (one per GPU) when no launcher set
    WORLD_SIZE. Nothing here touches the GPU. Rank 0's stdout (the JSON line)
    passes through; the other ranks' stdout goes to stderr. If a rank fails, the
    others are terminated (they may be blocked in a collective)."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in alive:
                    q.terminate()
        time.sleep(0.05)
    return rc


class Ctx:
    """Rank context: barrier, max over ranks, rank 0 output."""

    def __init__(self, torch, dist, world: int, rank: int, local: int):
        self.torch, self.dist, self.world, self.rank, self.local = torch, dist, world, rank, local

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.coll_device())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def coll_device(self) -> str:
        """Device of small collective tensors: the GPU under RCCL, the host under gloo."""
        return "cpu" if self.dist.get_backend() == "gloo" else "cuda"


def timed_steps(ctx: Ctx, step, finish, steps: int, warmup: int, ramp_s: float = 0.0, reset=None) -> float:
    """W untimed warmup steps (plus, if they took less than ramp_s, as many more as
    fill it: a GPU that sat idle through start-up runs ~5 % slow for the first
    milliseconds), then EXACTLY `steps` steps between barrier + synchronize pairs.
    `reset` (e.g. the kernel-timing counters) runs right before the timed region.
    Returns the max over ranks of the timed region's wall time."""
    t0 = time.perf_counter()
    for _ in range(warmup):
        step()
    finish()
    ctx.torch.cuda.synchronize()
    el = time.perf_counter() - t0
    extra = 0
    if ramp_s > el:
        per = el / max(warmup, 1)
        extra = int(min(ctx.max(math.ceil((ramp_s - el) / max(per, 1e-6))), 100_000))
    for _ in range(extra):
        step()
    finish()
    if reset is not None:
        reset()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    finish()
    ctx.barrier()
    return ctx.max(time.perf_counter() - t0)


# ---------------------------------------------------------------- host / CPU baseline
def host_info() -> dict:
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    # the GPU box gives one GPU's job a 16-CPU share (OMP_NUM_THREADS), while nproc shows the machine
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(usable, share) if share > 0 else usable
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable, "omp_num_threads": share or None,
            "threads_used_all_cores": threads}


def perm_for(b: int):
    # even pushes list rows ascending (Java HashMap<Integer> order), odd ones a seeded permutation
    return (1, 0) if b % 2 == 0 else (((2 * b + 1) * 2654435761) % ROWS | 1, (b * 7919) % ROWS)


def cpu_baseline(budget_s: float = 8.0, all_s: float = 4.0):
    """Oracle (C restatement of FloatMatrixStore.updateRow) on the same 32 x 64 MiB
    pushes: one thread until `budget_s`, then all usable cores (row-partitioned, each
    thread scanning every record in push order) until `all_s`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    bufs = [pyoracle.synth_dense_bucket(0, 1, 0, ROWS, ROWS, COLS, 1000 + b, *perm_for(b)) for b in range(W)]
    o = pyoracle.OracleStore(1, 0, 1, 0, ROWS - 1, COLS)
    o.synth_fill(7)
    algo = W * BUCKET + 2 * SHARD
    host = host_info()

    def run(threads, budget):
        reps, t0 = 0, time.perf_counter()
        while True:
            assert o.push_many(bufs, threads=threads) == 0
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget or reps >= 50:
                return reps, el

    reps, el = run(1, budget_s)
    nt = host["threads_used_all_cores"]
    reps_a, el_a = run(nt, all_s)
    return {"value": round(reps * algo / el / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"full config-2 workload (32 x 64 MiB pushes -> 16384x1024 fp32 shard) x{reps} reps, "
                      f"{el:.1f} s, oracle/dml_oracle.c single thread",
            "all_cores": {"value": round(reps_a * algo / el_a / 2**30, 3), "unit": "GiB/s", "cores": nt,
                          "sample": f"same workload x{reps_a} reps, {el_a:.1f} s, rows partitioned over {nt} threads"},
            "host": host}


def _coprime(a, n):
    while math.gcd(a, n) != 1:
        a += 1
    return a


def _sparse_perm(b, dim):
    pa = (2 * b + 3) * 999_999_937 % dim
    while pa % 2 == 0 or pa % 5 == 0:
        pa += 1
    return pa, (b * 12_345_701) % dim


# ---------------------------------------------------------------- config 2
# Where a call's pushes sit in HBM moves the reduces' DRAM efficiency by a few per cent
# (same bytes, same kernels; DESIGN.md §4.1 / §4.2, profiles/r06_ab_slab_legs.txt):
#  - config 2 (32 x 64 MiB): one allocation per push, the buffers allocated first in the
#    process, ran 330-333 us per launch against 336-338 us as slices of one slab (r06, two
#    GPU calls, 7 of 7 alternating rounds; the driver's lines: r03 / r04 330 / 334 us with
#    separate buffers, r05 339 us with the slab). Separate buffers allocated after and
#    around others drew 332-348 us (r05 placement probe, scripts/probe_placement.py);
#  - configs 4 / 4a (16 x 8 GB): slices of one slab 2-4 % faster on one box, equal on another;
#  - config 5: one allocation per push (its slab 1.7-2.2 % slower, r05 and r06).
# --push-layout slab / separate forces one layout on every leg (--separate-buffers =
# separate).
SLAB = [False]   # config 2
SLAB4 = [True]   # configs 4 / 4a


def push_buffers(torch, n: int, nbytes: int):
    """n push buffers of nbytes for the config-4 legs: slices of one receive slab (SLAB4),
    or one allocation each."""
    if SLAB4[0]:
        slab = torch.empty(n * nbytes, dtype=torch.uint8, device="cuda")
        return [slab[i * nbytes:(i + 1) * nbytes] for i in range(n)]
    return [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]


def make_buckets(L, torch, fmt, n, rows_total, value_seed: int = 1000, alloc_seed: int = 0):
    st = torch.cuda.current_stream().cuda_stream
    bufs = []
    if SLAB[0]:  # the n buckets as slices of one allocation (the receive slab)
        slab = torch.empty(n * rows_total * REC, dtype=torch.uint8, device="cuda")
        mem = [slab[i * rows_total * REC:(i + 1) * rows_total * REC] for i in range(n)]
    else:
        mem = [torch.empty(rows_total * REC, dtype=torch.uint8, device="cuda") for _ in range(n)]
    if alloc_seed:  # diagnostic: bucket b in the alloc_order[b]-th allocation (addresses not in push order)
        import random
        random.Random(alloc_seed).shuffle(mem)
    for b in range(n):
        t = mem[b]
        pa, pc = perm_for(b)
        rc = L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows_total, rows_total, COLS,
                                      value_seed + b, pa % rows_total, pc % rows_total, C.c_void_p(st))
        assert rc == 0, rc
        bufs.append(t)
    torch.cuda.synchronize()
    return bufs


def _pre_time(L, every: int, reset: bool):
    """Pre-reduce piece timing of the sharded path (dml_prereduce_timing / _kernel_time):
    returns the totals so far, then samples one call in `every` (0 = off)."""
    ms, n = C.c_double(0.0), C.c_int64(0)
    assert L.dml_prereduce_kernel_time(C.byref(ms), C.byref(n), 1 if reset else 0) == 0
    assert L.dml_prereduce_timing(every) == 0
    return ms.value, n.value


# Device-code sources: a profile's counted bytes stand for the kernels built from these
DEVICE_SOURCES = ("dml_device.h", "dml_internal.h", "dml_kernels.hip", "dml_sparse.hip", "dml_split.hip")


# the sources each profiled kernel is built from: the dense reduce kernels
# (dml_kernels.hip) and the sparse partition / leaf kernels (dml_sparse.hip)
KERNEL_SOURCES = {"dense": ("dml_device.h", "dml_internal.h", "dml_kernels.hip"),
                  "sparse": ("dml_device.h", "dml_internal.h", "dml_sparse.hip")}
TRAFFIC_GROUP = {"sparse": "sparse", "sparse_l1": "sparse", "sparse_l2": "sparse"}  # others: dense


def device_src_hash(files=DEVICE_SOURCES, read=None) -> str:
    """sha256 (16 hex digits) of device-code sources (all of them by default);
    scripts/gpu_prof.sh records it with every profile, and a stored traffic figure
    counts only while the sources of its kernel still match. `read(f)` returns a
    file's bytes (default: the working tree)."""
    import hashlib
    h = hashlib.sha256()
    for f in files:
        h.update(f.encode())
        if read is not None:
            h.update(read(f))
        else:
            with open(os.path.join(ROOT, "distml_amd", "csrc", f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def device_src_hashes(read=None) -> dict:
    """device_src_hash of every kernel group (KERNEL_SOURCES) and of all sources."""
    out = {g: device_src_hash(fs, read) for g, fs in KERNEL_SOURCES.items()}
    out["all"] = device_src_hash(DEVICE_SOURCES, read)
    return out


def _kernel_sig(name: str) -> str:
    """rocprof's kernel name without "void " and the parameter list."""
    n = name[5:] if name.startswith("void ") else name
    return n.split("(", 1)[0].strip()


def traffic_for(key: str, kernel_ran: str) -> dict:
    """roofline.traffic from profiles/pmc_traffic.json (PMC FETCH_SIZE / WRITE_SIZE per
    dispatch), only when the stored entry profiled the same kernel instantiation that
    ran here (dml_store_kernel_name) from the same device sources; otherwise
    traffic = null and traffic_stale says why."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        e = (json.load(open(p)).get("per_config") or {}).get(key)
    except Exception:
        e = None
    if not e:
        return {"traffic": None, "traffic_stale": f"no profile entry '{key}'"}
    prof = _kernel_sig(e.get("kernel", ""))
    if prof != kernel_ran:
        return {"traffic": None, "traffic_stale": f"profiled {prof or '?'}, ran {kernel_ran or '?'}"}
    group = TRAFFIC_GROUP.get(key, "dense")
    by = e.get("src_sha_by_group") or {}
    want, have = (by.get(group), device_src_hash(KERNEL_SOURCES[group])) if by.get(group) else \
        (e.get("src_sha"), device_src_hash())
    if want != have:
        return {"traffic": None, "traffic_stale": f"device sources {have} differ from the profiled {want}"}
    return {"traffic": e["hbm_bytes_per_launch"],
            "traffic_source": f"{e.get('source', '?')}; commit {e.get('commit', '?')}; {group} sources {have}"}


def prereduce_roofline(L, ctx, pieces, pre_ms, pre_n, pre_bytes, label):
    calls = pre_n / pieces
    avg_s = pre_ms / calls / 1e3
    achieved = pre_bytes / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": f"k_reduce_rows pre-reduce ({pieces} pieces per call, rank {ctx.rank}; {label})",
            "avg_kernel_us": round(avg_s * 1e6, 2), "launches": pre_n, "algorithmic_bytes_per_call": pre_bytes}


def headline(ctx: Ctx, L, args, out_line: dict):
    torch = ctx.torch
    from distml_amd import DataDesc, DataStore, KeyRange
    from distml_amd.group import ShardGroup
    from distml_amd.store import DeviceBatch
    world, rank = ctx.world, ctx.rank
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_FLOAT)
    sharded = world > 1 or args.group
    group = None
    shuffled_batches = None
    step_rows = (ROWS - 1 + world) // world
    hbm_check(torch, "config2", {"pushes": 2 * W * BUCKET,
                                 "store": store_bytes(step_rows if sharded else ROWS, COLS, 4, spec=True),
                                 "group": group_bytes(world, ROWS, COLS, 4) if sharded else 0})
    if not sharded:
        store = DataStore(fmt, KeyRange(0, ROWS - 1), COLS, device=ctx.local)
        store.synth_fill(7)
        # two bucket sets, stepped alternately: the same key order per push position
        # (a worker pushing the same key set), different gradient values every step
        bufs = (make_buckets(L, torch, fmt, W, ROWS, alloc_seed=args.alloc_seed) +
                make_buckets(L, torch, fmt, W, ROWS, value_seed=5000, alloc_seed=args.alloc_seed))
        batches = [DeviceBatch([b.data_ptr() for b in bs], [b.numel() for b in bs]) for bs in (bufs[:W], bufs[W:])]
        # the same steps with the 32 pushes in a new seeded order every step: the PS
        # selector applies pushes in arrival order (PSAgent.java:166-186)
        import random
        shuffled_batches = []
        for k in range(SHUFFLE_ORDERS):
            bs = bufs[:W] if k % 2 == 0 else bufs[W:]
            order = list(range(W))
            # diagnostics: one order every step (--shuffle-orders 1), or only the
            # ascending / only the permuted pushes shuffled among their own positions
            rnd2 = random.Random(2024 + (k % args.shuffle_orders if args.shuffle_orders else k))
            rnd2.shuffle(order)
            ev, od = [j for j in order if j % 2 == 0], [j for j in order if j % 2 == 1]
            if args.shuffle_keep_parity:  # diagnostic: ascending pushes stay at even positions
                order = [x for pair in zip(ev, od) for x in pair]
            elif args.shuffle_only == "asc":
                order = [x for pair in zip(ev, range(1, W, 2)) for x in pair]
            elif args.shuffle_only == "perm":
                order = [x for pair in zip(range(0, W, 2), od) for x in pair]
            shuffled_batches.append(DeviceBatch([bs[j].data_ptr() for j in order], [bs[j].numel() for j in order]))
        k_step = [0]
        cur = [batches]

        def step():
            # async: ack once captured; the store keeps <= 2 batches in flight and the
            # key index of batch k+1 overlaps the reduce of batch k
            bl = cur[0]
            store.pushDevice(bl[k_step[0] % len(bl)])
            k_step[0] += 1

        finish = store.flush  # every pushed batch applied and error-checked
        timed_store = store
        algo_per_rank = W * BUCKET + 2 * SHARD
    else:
        group = ShardGroup(fmt, ROWS, COLS, rank, world, device=ctx.local, pieces=args.pieces,
                           emulate_world=args.emulate_rs, emulate_channels=args.emulate_channels)
        if args.index_normal_prio:  # diagnostic: the next call's index chain at normal priority
            group.istream = torch.cuda.Stream(device=torch.device("cuda", ctx.local))
        bufs = make_buckets(L, torch, fmt, W, ROWS) + make_buckets(L, torch, fmt, W, ROWS, value_seed=5000)
        sets = [([b.data_ptr() for b in bs], [b.numel() for b in bs]) for bs in (bufs[:W], bufs[W:])]
        st = torch.cuda.current_stream().cuda_stream
        k_step = [0]

        def step():
            group.push_full_range(*sets[k_step[0] & 1], st)
            k_step[0] += 1

        finish = group.flush
        timed_store = group.store
        algo_per_rank = W * BUCKET + 2 * group.shard.size() * COLS * 4

    timing = not args.no_timing
    # one chunk in 4 carries start/stop events (>= 5 launches averaged over the default
    # 20 steps): events in every dispatch lengthen the boundary between two reduces
    # 
    timed_store.set_timing(timing and not sharded, every=4)
    t0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    finish()

    def reset():
        timed_store.kernel_time(reset=True)
        if not sharded:
            timed_store.stats(reset=True)
        else:
            group.prereduce_stats(reset=True)
        if sharded and timing:
            _pre_time(L, every=4, reset=True)

    el = timed_steps(ctx, step, finish, args.steps, 0, ramp_s=max(0.0, 0.3 - (time.perf_counter() - t0)),
                     reset=reset)
    k_ms, k_n = timed_store.kernel_time(reset=True)
    pre_ms, pre_n = _pre_time(L, every=0, reset=True) if sharded else (0.0, 0)
    shuffled = None
    if not sharded:
        counts = timed_store.stats(reset=True)
        # the arrival-order case: every step's 32 pushes in a new order (SHUFFLE_ORDERS
        # seeded orders, cycled), same store, warm
        cur[0] = shuffled_batches
        k_step[0] = 0
        el_s = timed_steps(ctx, step, finish, args.steps, min(args.warmup, 50), reset=reset)
        ks_ms, ks_n = timed_store.kernel_time(reset=True)
        cs = timed_store.stats(reset=True)
        shuffled = {"pushes": f"the same two bucket sets, each step's 32 pushes in a new seeded order "
                              f"({SHUFFLE_ORDERS} orders cycled): slot reuse keyed by the pushes' content",
                    "value": round(algo_per_rank * args.steps / el_s / 2**30, 2), "unit": "GiB/s",
                    "ms_per_step": round(el_s / args.steps * 1e3, 4)}
        if ks_n:
            a_s = algo_per_rank / (ks_ms / ks_n / 1e3) / 1e9
            shuffled.update({"avg_kernel_us": round(ks_ms / ks_n * 1e3, 2), "achieved": round(a_s, 1),
                             "frac": round(a_s / HBM_PEAK_GBS, 4)})
        shuffled["pushes_per_step"] = {k: round(cs[k] / max(cs["chunks"], 1), 2)
                                       for k in ("identity_pushes", "reused_pushes", "indexed_pushes")}
        shuffled["spec_reruns"] = cs["spec_reruns"]
        # the in-order steps once more, right after: separates the arrival order's cost
        # from the box's drift over a sustained run (the headline is measured first)
        cur[0] = batches
        k_step[0] = 0
        el_a = timed_steps(ctx, step, finish, args.steps, min(args.warmup, 50), reset=reset)
        ka_ms, ka_n = timed_store.kernel_time(reset=True)
        timed_store.stats(reset=True)
        if ka_n:
            shuffled["in_order_again"] = {
                "ms_per_step": round(el_a / args.steps * 1e3, 4), "avg_kernel_us": round(ka_ms / ka_n * 1e3, 2),
                "frac": round(algo_per_rank / (ka_ms / ka_n / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        # the same steps with the buckets generated into the 32 buffers in a seeded
        # order (which buffer holds which push is the PS's accident): DESIGN.md §4
        shuffled["buffers_shuffled"] = buffers_shuffled_line(ctx, L, args, timed_store, step, finish, cur, k_step,
                                                             fmt, algo_per_rank)
    timed_store.set_timing(False)
    value = algo_per_rank * world * args.steps / el / 2**30
    out_line.update({
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "config2: dense fp32 reduce, 32 device-resident pushes x 64 MiB "
                               "([int32 key][1024 x f32] x 16384) -> 16384x1024 fp32 model per GPU",
                   "pushes_per_gpu": W, "push_bytes": BUCKET, "model_rows": ROWS, "cols": COLS,
                   "rccl_channels": int(os.environ.get("NCCL_MAX_NCHANNELS", "0")) if sharded else None,
                   "parallelism": ("single shard" if not sharded else f"linearSplit({world}) + RCCL reduce-scatter"
                                   + (f" (DIAGNOSTIC: one rank's ring reduce-scatter footprint at {args.emulate_rs} "
                                      f"ranks emulated on {args.emulate_channels} blocks, pieces {args.pieces}, "
                                      "results not valid)" if args.emulate_rs else "")),
                   "pushes": "16 ascending + 16 permuted per step; two bucket sets stepped alternately "
                             "(same key order per push position, different values)"
                             + ("; each set's 32 pushes in one device receive slab" if SLAB[0]
                                else "; one allocation per push"),
                   "algorithmic_bytes_per_step_per_gpu": algo_per_rank},
    })
    if not sharded and k_n > 0:
        avg_s = k_ms / k_n / 1e3
        achieved = algo_per_rank / avg_s / 1e9
        pk = stream_peaks(L, torch)
        kn = timed_store.kernel_name()
        out_line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                                **traffic_for("config2", kn), "kernel": kn,
                                "avg_kernel_us": round(avg_s * 1e6, 2), "launches": k_n,
                                "measured_read_peak": round(pk["read"], 1),
                                "frac_of_measured_read": round(achieved / pk["read"], 4),
                                "measured_copy_peak": round(pk["copy"], 1)}
        out_line["pushes_per_step"] = {k: round(counts[k] / max(counts["chunks"], 1), 2)
                                                 for k in ("identity_pushes", "reused_pushes", "indexed_pushes")}
        out_line["spec_reruns"] = counts["spec_reruns"]
        out_line["shuffled"] = shuffled
    elif pre_n > 0:
        # the pre-reduce pieces (k_reduce_rows in pre-reduce mode) are the dominant
        # kernel; per call they read the W pushes and write the full-model partial
        out_line["roofline"] = prereduce_roofline(L, ctx, args.pieces, pre_ms, pre_n,
                                                  W * BUCKET + world * group.step_rows * COLS * 4, "config 2")
    if sharded:
        pst = group.prereduce_stats(reset=True)
        out_line["pushes_per_step"] = {k: round(pst.get(k, 0) / max(pst.get("chunks", 0), 1), 2)
                                       for k in ("identity_pushes", "reused_pushes", "indexed_pushes")}
        out_line["spec_reruns"] = pst.get("spec_reruns", 0)
    if group is not None:
        group.close()
    else:
        store.close()
    del bufs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def guarded_leg(ctx: Ctx, line: dict, out, key: str, fn, seconds: float):
    """A secondary leg that must not cost the line: if it raises, or has not returned
    after `seconds` (a collective that never completes), rank 0 prints the line so
    far with the leg's error and every rank exits (os._exit: no exec)."""
    import threading

    def bail(msg: str):
        if ctx.rank == 0:
            print(json.dumps(dict(line, **{key: {"error": msg}})), file=out, flush=True)
        os._exit(0)

    t = threading.Timer(seconds, bail, args=(f"did not finish within {seconds:.0f} s",))
    t.daemon = True
    t.start()
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 — reported in the line, not raised
        t.cancel()
        bail(repr(e)[:400])
    finally:
        t.cancel()


def leg_native_group(ctx: Ctx, L, args) -> dict:
    """The config-2 workload through the native shard group (dml_group_*, the RCCL
    communicator libdistml_ps creates itself; what the JNI's GpuShardGroup binds):
    the same per-rank work as the headline's sharded path — 32 full-range pushes per
    GPU, ordered pre-reduce, ncclReduceScatter of the [rank][row] slices over xGMI, the
    owner apply — run by every N > 1 line (and at N = 1 with --native-group). The
    unique id travels from rank 0 over torch.distributed."""
    torch, dist = ctx.torch, ctx.dist
    from distml_amd import DataDesc
    from distml_amd.group import NativeShardGroup
    world, rank = ctx.world, ctx.rank
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_FLOAT)
    hbm_check(torch, "native_group", {"pushes": 2 * W * BUCKET,
                                      "store": store_bytes((ROWS - 1 + world) // world, COLS, 4),
                                      "group": group_bytes(world, ROWS, COLS, 4)})
    uid = [NativeShardGroup.unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    g = NativeShardGroup(fmt, ROWS, COLS, rank, world, uid[0], device=ctx.local, pieces=args.pieces)
    g.store.synth_fill(7)
    bufs = make_buckets(L, torch, fmt, W, ROWS) + make_buckets(L, torch, fmt, W, ROWS, value_seed=5000)
    sets = [([b.data_ptr() for b in bs], [b.numel() for b in bs]) for bs in (bufs[:W], bufs[W:])]
    k_step = [0]

    def step():
        g.push_full_range(*sets[k_step[0] & 1])
        k_step[0] += 1

    timing = not args.no_timing

    def reset():
        g.prereduce_stats(reset=True)
        if timing:
            _pre_time(L, every=4, reset=True)

    el = timed_steps(ctx, step, g.flush, args.steps, args.warmup, ramp_s=0.3, reset=reset)
    pre_ms, pre_n = _pre_time(L, every=0, reset=True)
    pst = g.prereduce_stats(reset=True)
    shard_rows = g.shard.size()
    algo = W * BUCKET + 2 * shard_rows * COLS * 4
    out = {"workload": "config2 through dml_group (native RCCL communicator, the JNI binding's path)",
           "value": round(algo * world * args.steps / el / 2**30, 2), "unit": "GiB/s",
           "ms_per_step": round(el / args.steps * 1e3, 4), "n_gpus": world, "pieces": args.pieces,
           "pushes_per_step": {k: round(pst.get(k, 0) / max(pst.get("chunks", 0), 1), 2)
                               for k in ("identity_pushes", "reused_pushes", "indexed_pushes")},
           "spec_reruns": pst.get("spec_reruns", 0)}
    if pre_n > 0:
        step_rows = (ROWS - 1 + world) // world
        out["roofline"] = prereduce_roofline(L, ctx, args.pieces, pre_ms, pre_n,
                                             W * BUCKET + world * step_rows * COLS * 4, "config 2, native group")
    g.close()
    del bufs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def buffers_shuffled_line(ctx: Ctx, L, args, store, step, finish, cur, k_step, fmt, algo_per_rank) -> dict:
    """The in-order steps over two new bucket sets whose pushes were generated into
    their buffers in a seeded order (make_buckets(alloc_seed=7)): the headline's
    buffers hold the pushes in allocation order, a PS's receive buffers do not."""
    torch = ctx.torch
    from distml_amd.store import DeviceBatch
    b2 = (make_buckets(L, torch, fmt, W, ROWS, alloc_seed=7) +
          make_buckets(L, torch, fmt, W, ROWS, value_seed=5000, alloc_seed=7))
    cur[0] = [DeviceBatch([b.data_ptr() for b in bs], [b.numel() for b in bs]) for bs in (b2[:W], b2[W:])]
    k_step[0] = 0
    el = timed_steps(ctx, step, finish, args.steps, min(args.warmup, 50),
                     reset=lambda: (store.kernel_time(reset=True), store.stats(reset=True)))
    k_ms, k_n = store.kernel_time(reset=True)
    store.stats(reset=True)
    out = {"pushes": "in order, over two bucket sets generated into their 32 buffers in a seeded order",
           "value": round(algo_per_rank * args.steps / el / 2**30, 2), "unit": "GiB/s",
           "ms_per_step": round(el / args.steps * 1e3, 4)}
    if k_n:
        out.update({"avg_kernel_us": round(k_ms / k_n * 1e3, 2),
                    "frac": round(algo_per_rank / (k_ms / k_n / 1e3) / 1e9 / HBM_PEAK_GBS, 4)})
    cur[0] = []
    del b2
    torch.cuda.synchronize()
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


# ---------------------------------------------------------------- config 3 (N=1)
def sparse_leg(ctx: Ctx, L, steps: int, cpu: bool, cu_split: int = 0):
    """Config 3 (reported beside the headline): 1e9-dim fp32 FloatArrayStore shard
    (4 GB), 32 device-resident pushes x 1e6 unique keys ([int64 key][f32] = 12 B),
    ordered per-push scatter-add. Algorithmic bytes per step = 32 x 12e6 + 2 x 4 x 32e6."""
    torch = ctx.torch
    from distml_amd import DataDesc, DataStore, KeyRange
    from distml_amd.store import DeviceBatch
    dim, nnz, w = 10**9, 10**6, 32
    fmt = DataDesc(DataDesc.DATA_TYPE_ARRAY, DataDesc.KEY_TYPE_LONG, DataDesc.ELEMENT_TYPE_FLOAT)
    # the shard, the pushes, and three partition workspaces (~40 B per record of a chunk)
    hbm_check(torch, "sparse", {"shard": 4 * dim, "pushes": w * nnz * 12, "workspaces": 3 * 40 * w * nnz})
    store = DataStore(fmt, KeyRange(0, dim - 1), device=ctx.local)
    if cu_split:  # the partition's stream on part of the CUs, the leaf's on the rest
        store.set_knob(2, cu_split)
    bufs = []
    st = torch.cuda.current_stream().cuda_stream
    for b in range(w):
        t = torch.empty(nnz * 12, dtype=torch.uint8, device="cuda")
        assert L.dml_synth_sparse_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, dim, nnz, 2000 + b,
                                         *_sparse_perm(b, dim), C.c_void_p(st)) == 0
        bufs.append(t)
    torch.cuda.synchronize()
    batch = DeviceBatch([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
    # start events on every leaf launch (a ~1.2 ms kernel: the events' boundary cost is
    # under 1 %), so the roofline averages the same launches rocprof's kernel trace does
    store.set_timing(True, every=1)

    def step():
        store.pushDevice(batch)

    for _ in range(max(2, steps)):  # warmup: as many untimed steps as timed ones
        step()
    store.flush()
    store.kernel_time(reset=True)
    el = timed_steps(ctx, step, store.flush, steps, 0)
    k_ms, k_n = store.kernel_time(reset=True)
    kn = store.kernel_name()
    algo = w * nnz * 12 + 2 * 4 * w * nnz
    out = {"workload": "config3: 1e9-dim fp32 array shard, 32 pushes x 1e6 unique int64 keys, ordered scatter-add",
           "value": round(steps * algo / el / 2**30, 2), "unit": "GiB/s (algorithmic)", "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 3), "algorithmic_bytes_per_step": algo}
    if k_n:
        # the leaf apply (ordered scatter-add) is the dominant kernel; the two partition
        # passes of the next chunk run beside it on the index stream
        k_s = k_ms / k_n / 1e3
        out["roofline"] = {"bound": "hbm", "achieved": round(algo / k_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(algo / k_s / 1e9 / HBM_PEAK_GBS, 4),
                           **traffic_for("sparse", kn), "kernel": kn, "avg_kernel_us": round(k_s * 1e6, 2),
                           "launches": k_n,
                           "note": "random 4-B RMW into a 4 GB array: line-granular (64-B read / 32-B write "
                                   "sectors), so counted traffic is ~3.9x the algorithmic bytes (DESIGN.md §4)"}
        tr = out["roofline"].get("traffic")
        if tr:  # the effective (counted-bytes) rate beside the algorithmic one
            out["roofline"]["effective_GBps"] = round(tr / k_s / 1e9, 1)
        # the random-RMW floor of the same 32e6 updates on this box (dml_diag_rmw_floor):
        # sorted globally, one plain read-modify-write each, no partition — the leaf's best
        # case; measured into the shard after the timed steps (its values are not used again)
        keys = torch.cat([b.view(-1, 12)[:, :8].contiguous().view(torch.int64).view(-1) for b in bufs])
        idx = torch.sort(keys).values.to(torch.int32)
        del keys
        ones = torch.ones(idx.numel(), dtype=torch.float32, device="cuda")
        ms = C.c_float()
        best = None
        for _ in range(3):
            assert L.dml_diag_rmw_floor(C.c_void_p(store.device_ptr()), C.c_void_p(idx.data_ptr()),
                                        C.c_void_p(ones.data_ptr()), idx.numel(), C.c_void_p(st), C.byref(ms)) == 0
            best = ms.value if best is None else min(best, ms.value)
        del idx, ones
        out["roofline"]["measured_rmw_floor_us"] = round(best * 1e3, 1)
        out["roofline"]["frac_of_measured_floor"] = round(best * 1e-3 / k_s, 3)
    store.close()
    del bufs
    torch.cuda.empty_cache()
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        o = pyoracle.OracleStore(0, 1, 1, 0, dim - 1)
        n, spent = 0, 0.0
        while n < w and spent < 6.0:
            buf = pyoracle.synth_sparse_bucket(1, 1, 0, dim, nnz, 2000 + n, *_sparse_perm(n, dim))
            t1 = time.perf_counter()
            assert o.push(buf) == 0
            spent += time.perf_counter() - t1
            n += 1
        o.close()
        out["cpu_baseline"] = {"value": round(n * (nnz * 12 + 2 * 4 * nnz) / spent / 2**30, 3),
                               "unit": "GiB/s (algorithmic)", "cores": 1, "kind": "port",
                               "sample": f"first {n} of the 32 pushes into the 4 GB host array in {spent:.1f} s, "
                                         f"oracle/dml_oracle.c FloatArrayStore restatement, single thread"}
    return out


# ---------------------------------------------------------------- config 4 (model level)
def c4_fit_rows(ctx: Ctx, w: int, cols: int = C4_COLS, cap: int = C4_ROWS, share: int = 1) -> int:
    """The most config-4 rows (<= cap, whole 100 000s) whose W pushes, store (two shard
    buffers and the workspace ring) and, at N > 1, group buffers fit the free HBM and
    still leave the store the headroom it keeps before it allocates its speculative second
    buffer (1/8 of the device, dml_store.hip): without it the chunks run the key index.
    `share`: ranks sharing the device (the one-GPU gloo rehearsal)."""
    free, total = ctx.torch.cuda.mem_get_info()
    free = (0.97 * free - max(total / 8, 4 << 30)) / share
    world = ctx.world
    sharded = world > 1
    per_row = w * (4 + 4 * cols) + (2 * cols * 4 + 3 * WS_BYTES_PER_ROW) / (world if sharded else 1)
    if sharded:
        per_row += (2 * cols * 4 + 2 * cols * 4 / world) + 3 * WS_BYTES_PER_ROW
    rows = int(min(cap, free / per_row) // 100_000 * 100_000)
    return int(-ctx.max(-rows))  # every rank the same model (the smallest fit)


def leg_config4(ctx: Ctx, L, args, w: int = 0, rows: int = 0, cpu: bool = True) -> dict:
    """BASELINE config 4: Word2Vec rows 10M x 200 fp32, W full-range pushes per GPU.
    N=1: one store, the ordered batch reduce. N>1: linearSplit(N) shards, ordered
    pre-reduce of the W local pushes, RCCL reduce-scatter, owner apply (plain
    FloatMatrixStore sum, the config's metric; weak scaling: W pushes per GPU).
    `w` / `rows` override --c4-pushes / 10 M rows (SURVEY §8(d)'s W = 8 and W = 32)."""
    torch = ctx.torch
    from distml_amd import DataDesc, DataStore, KeyRange
    from distml_amd.group import ShardGroup
    from distml_amd.store import DeviceBatch
    world, rank = ctx.world, ctx.rank
    rows, cols, w = rows or C4_ROWS, C4_COLS, w or args.c4_pushes
    rec = 4 + 4 * cols
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_FLOAT)
    st = torch.cuda.current_stream().cuda_stream
    sharded = world > 1 or args.group
    S4 = (rows - 1 + world) // world
    hbm_check(torch, "config4", {"pushes": w * rows * rec, "store": store_bytes(S4 if sharded else rows, cols, 4, spec=True),
                                 "group": group_bytes(world, rows, cols, 4) if sharded else 0})
    bufs = []
    asc = args.c4_order == "asc"
    mem = push_buffers(torch, w, rows * rec)
    for b in range(w):
        t = mem[b]
        seed = 3000 + 64 * rank + b
        pa, pc = (1, 0) if asc else (_coprime(seed * 2654435761 % rows | 1, rows), b * 7919 % rows)
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows, rows, cols, seed, pa, pc,
                                        C.c_void_p(st)) == 0
        bufs.append(t)
    torch.cuda.synchronize()
    ptrs, lens = [b.data_ptr() for b in bufs], [b.numel() for b in bufs]
    group = None
    if not sharded:
        store = DataStore(fmt, KeyRange(0, rows - 1), cols, device=ctx.local)
        store.synth_fill(13)
        batch = DeviceBatch(ptrs, lens)

        def step():
            store.pushDevice(batch)

        finish = store.flush
        shard_rows = rows
        store.set_timing(True)
    else:
        group = ShardGroup(fmt, rows, cols, rank, world, device=ctx.local, pieces=args.pieces)
        group.store.synth_fill(13)

        def step():
            group.push_full_range(ptrs, lens, st)

        finish = group.flush
        shard_rows = group.shard.size()
        store = group.store
    for _ in range(args.c4_warmup):
        step()
    finish()

    def reset():
        store.kernel_time(reset=True)
        if sharded:
            _pre_time(L, every=1, reset=True)

    el = timed_steps(ctx, step, finish, args.c4_steps, 0, reset=reset)
    k_ms, k_n = store.kernel_time(reset=True)
    store.set_timing(False)
    pre_ms, pre_n = _pre_time(L, every=0, reset=True) if sharded else (0.0, 0)
    algo = w * rows * rec + 2 * shard_rows * cols * 4
    out = {"workload": f"config4: Word2Vec rows {rows}x{cols} fp32 model, {w} full-range pushes per GPU "
                       f"([int32][{cols} x f32], rows {'ascending (keys implicit = row)' if asc else 'permuted per push'})",
           "value": round(algo * world * args.c4_steps / el / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
           "pushes_per_gpu": w, "push_buffers": "one receive slab" if SLAB4[0] else "one allocation per push",
           "steps": args.c4_steps, "ms_per_step": round(el / args.c4_steps * 1e3, 3),
           "scaling": "weak", "dtype": "f32",
           "parallelism": "single shard" if not sharded else f"linearSplit({world}) + RCCL reduce-scatter",
           "algorithmic_bytes_per_step_per_gpu": algo}
    if not sharded and k_n:
        k_s = k_ms / k_n / 1e3
        kn = store.kernel_name()
        out["roofline"] = {"bound": "hbm", "achieved": round(algo / k_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(algo / k_s / 1e9 / HBM_PEAK_GBS, 4),
                           **(traffic_for("leg4", kn) if (w, rows) == (16, C4_ROWS) else
                              {"traffic": None, "traffic_stale": "the counters were taken at W = 16, 10 M rows"}),
                           "kernel": kn, "avg_kernel_us": round(k_s * 1e6, 1), "launches": k_n}
        if asc:
            # the plain stream of the same bytes over the same allocations (dml_diag_dense_floor:
            # no key checks; out of place like the speculative chunk): the live ceiling
            fl, oop = dense_floor(L, store, ptrs, lens, st)
            out["roofline"].update({"measured_stream_floor_us": round(fl * 1e3, 1),
                                    "measured_stream_floor_frac": round(algo / (fl * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                    "frac_of_measured_floor": round(fl * 1e-3 / k_s, 3),
                                    "floor_layout": "out of place" if oop else "in place"})
    elif pre_n:
        out["roofline"] = prereduce_roofline(L, ctx, args.pieces, pre_ms, pre_n,
                                             w * rows * rec + world * group.step_rows * cols * 4, "config 4")
    if group is not None:
        group.close()
    else:
        store.close()
    del bufs, ptrs, mem, t  # the slab goes with its last slice
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if world == 1 and not args.no_cpu and cpu:
        out["cpu_baseline"] = leg_cpu_baseline("4")
    return out


def leg_cpu_baseline(which: str, budget_s: float = 3.0) -> dict:
    """The oracle on one linearSplit(8) shard of the leg's workload (SURVEY §8(d):
    configs 4 and 5 time one shard on the CPU; the whole model is 8 such shards)."""
    b = shard_cpu_baseline(SHARD_CONFIGS[which], budget_s)
    b["sample"] = "one 1/8 shard of the model (" + SHARD_CONFIGS[which]["name"] + "): " + b["sample"]
    return b


# ---------------------------------------------------------------- config 4, AdaGrad (model level)
def leg_config4_ada(ctx: Ctx, L, args) -> dict:
    """Config 4's AdaGrad store (FloatMatrixStoreAdaGrad.java:239-284) at N GPUs:
    rows linearSplit(N); every rank holds W full-range ascending pushes of the 10M x
    200 model; a step = ShardGroup.push_exchange (dml_shard_split by owner, RCCL
    all-to-all, every owner applies the N x W slices in rank-major push order with
    the exact AdaGrad reduce). Weak scaling (W pushes per GPU). Algorithmic bytes
    per rank: its push bytes + the shard's data and delta read and written (alpha is
    written only where delta ends above 1)."""
    torch = ctx.torch
    from distml_amd import DataDesc
    from distml_amd.group import ShardGroup
    world, rank = ctx.world, ctx.rank
    rows, cols, w = C4_ROWS, C4_COLS, args.c4a_pushes
    rec = 4 + 4 * cols
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_FLOAT, False, True, True)
    st = torch.cuda.current_stream().cuda_stream
    S4 = (rows - 1 + world) // world
    # exchange buffers: a send and a receive set of up to all push bytes each, two in flight
    hbm_check(torch, "config4_ada", {"pushes": w * rows * rec, "store": store_bytes(S4, cols, 4, ada=True),
                                     "exchange": 0 if world == 1 else 4 * w * rows * rec})
    bufs = []
    mem = push_buffers(torch, w, rows * rec)
    for b in range(w):
        t = mem[b]
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows, rows, cols, 5000 + 64 * rank + b,
                                        1, 0, C.c_void_p(st)) == 0
        bufs.append(t)
    torch.cuda.synchronize()
    ptrs, lens = [b.data_ptr() for b in bufs], [b.numel() for b in bufs]
    group = ShardGroup(fmt, rows, cols, rank, world, device=ctx.local, exchange_only=True)
    store = group.store
    store.setAlpha(0.025, 0.0001, 1.0)
    store.synth_fill(13)

    calls = []  # host time of each call (diagnostic: the split's counts and the exchange wait there)

    moments = args.c4a_path == "moments"

    def step():
        t = time.perf_counter()
        if moments:  # Σu / Σu² pre-reduce, one reduce-scatter, owner apply (within 1e-6)
            group.push_moments(ptrs, lens)
        else:        # exact: split, all-to-all, ordered owner apply
            group.push_exchange(ptrs, lens)
        calls.append(time.perf_counter() - t)

    for _ in range(args.c4a_warmup):
        step()
    group.flush()
    store.set_timing(True)
    el = timed_steps(ctx, step, group.flush, args.c4a_steps, 0, reset=lambda: store.kernel_time(reset=True))
    k_ms, k_n = store.kernel_time(reset=True)
    store.set_timing(False)
    S = group.shard.size()
    # the reference's updateRow (FloatMatrixStoreAdaGrad.java:262-277) reads and writes
    # data and delta and writes alpha only where delta ends above 1, which these
    # gradients (|u| ~ 1e-3 from delta = 0) never reach: 4 state bytes moves per element
    algo = w * rows * rec + 4 * S * cols * 4
    path = ("two-moment path (Σu, Σu² reduce-scatter; within 1e-6)" if moments else "exact exchange path")
    out = {"workload": f"config4 AdaGrad: FloatMatrixStoreAdaGrad {rows}x{cols} fp32 (data + alpha + delta), {w} "
                       f"full-range pushes per GPU (rows ascending), {path}",
           "value": round(algo * world * args.c4a_steps / el / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
           "pushes_per_gpu": w, "push_buffers": "one receive slab" if SLAB4[0] else "one allocation per push",
           "steps": args.c4a_steps, "ms_per_step": round(el / args.c4a_steps * 1e3, 3),
           "scaling": "weak", "dtype": "f32",
           "parallelism": "single shard (local exchange)" if world == 1 else
                          f"linearSplit({world}) + dml_shard_split + RCCL all-to-all + ordered owner apply",
           "algorithmic_bytes_per_step_per_gpu": algo,
           "host_ms_per_call": [round(x * 1e3, 2) for x in calls[-args.c4a_steps:]]}
    if k_n:
        k_s = k_ms / k_n / 1e3
        # one owner launch: every rank's slices + data/delta RMW (moments: the received
        # Σu / Σu² rows instead of the slices)
        owner = (2 * S * cols * 4 if moments else world * w * S * rec) + 4 * S * cols * 4
        kn = store.kernel_name()
        tr = traffic_for("leg4a", kn) if world == 1 else {"traffic": None, "traffic_stale": "profiled at N = 1 only"}
        out["roofline"] = {"bound": "hbm", "achieved": round(owner / k_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(owner / k_s / 1e9 / HBM_PEAK_GBS, 4),
                           **tr, "kernel": kn, "rank": rank,
                           "avg_kernel_us": round(k_s * 1e6, 1), "launches": k_n}
        if world == 1 and not moments:
            # AdaGrad's data / delta stream with the same pushes, plain (dml_diag_dense_floor,
            # in place, no maxDelta / alpha bookkeeping): the live 4-read / 2-write ceiling
            fl, _ = dense_floor(L, store, ptrs, lens, torch.cuda.current_stream().cuda_stream)
            out["roofline"].update({"measured_stream_floor_us": round(fl * 1e3, 1),
                                    "measured_stream_floor_frac": round(owner / (fl * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                    "frac_of_measured_floor": round(fl * 1e-3 / k_s, 3)})
    group.close()
    del bufs, ptrs, mem, t  # the slab goes with its last slice
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


# ---------------------------------------------------------------- config 5 (model level)
def leg_config5(ctx: Ctx, L, args) -> dict:
    """BASELINE config 5: LDA word-topic counts, IntMatrixStore 1M x 1000 int32,
    32 pushes x 65 536 distinct vocabulary rows. The reference's client splits
    each push by server partition (SparseMatrix.java:46-60) and every shard
    applies its part with the negativity check (IntMatrixStore.java:164-178):
    rank r holds shard r of linearSplit(N) and its parts of the 32 pushes
    (65 536 x |shard| / 1M rows each). No data-path collective; strong scaling.
    Successive steps alternate the pushes with their negations (counts stay >= 0)."""
    torch = ctx.torch
    from distml_amd import DataDesc, DataStore, KeyRange
    from distml_amd.store import DeviceBatch
    world, rank = ctx.world, ctx.rank
    cols = C5_COLS
    shard = KeyRange(0, C5_ROWS - 1).linearSplit(world)[rank]
    S = shard.size()
    nrec = int(round(C5_NNZ * S / C5_ROWS))
    rec = 4 + 4 * cols
    fmt = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_INT)
    hbm_check(torch, "config5", {"pushes": 2 * C5_W * nrec * rec, "store": store_bytes(S, cols, 4)})
    store = DataStore(fmt, shard, cols, device=ctx.local)
    store.synth_fill(11)
    st = torch.cuda.current_stream().cuda_stream
    pos, neg = [], []
    # one allocation per push: slices of one slab ran this leg 1.7-2.2 % slower in
    # r05 and r06 (3 of 3 rounds each, profiles/r06_ab_slab_legs.txt)
    for b in range(C5_W):
        t = torch.empty(nrec * rec, dtype=torch.uint8, device="cuda")
        seed = 4000 + b
        pa = _coprime((seed * 2654435761 + rank) % S | 1, S)
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), shard.firstKey, S, nrec, cols, seed,
                                        pa, (b * 331 + rank) % S, C.c_void_p(st)) == 0
        pos.append(t)
        n = t.clone().view(torch.int32).view(nrec, 1 + cols)
        n[:, 1:] = -n[:, 1:]
        neg.append(n.view(torch.uint8).view(-1))
    torch.cuda.synchronize()
    sets = [DeviceBatch([b.data_ptr() for b in s], [b.numel() for b in s]) for s in (pos, neg)]
    # the doc-topic totals (LightLDA.scala:224-239: dtm.push(dt) beside wtm.push(wt)): an
    # IntArrayStore of the K = 1000 topics (IntArrayWithIntKey, [int32 key][int32] records),
    # linearSplit over the ranks like the word-topic rows; every worker's push lists all
    # its topics (a HashMap<Int> of small keys: ascending), applied with the check after
    # every add (IntArrayStore.java:97-113); alternating with the negations as above
    afmt = DataDesc(DataDesc.DATA_TYPE_ARRAY, DataDesc.KEY_TYPE_INT, DataDesc.ELEMENT_TYPE_INT)
    ash = KeyRange(0, C5_TOPICS - 1).linearSplit(world)[rank]
    A = ash.size()
    astore = DataStore(afmt, ash, device=ctx.local)
    astore.synth_fill(12)
    apos, aneg = [], []
    for b in range(C5_W):
        t = torch.empty(A * 8, dtype=torch.uint8, device="cuda")
        assert L.dml_synth_sparse_bucket(t.data_ptr(), C.byref(afmt.to_c()), ash.firstKey, A, A, 4100 + b, 1, 0,
                                         C.c_void_p(st)) == 0
        apos.append(t)
        n = t.clone().view(torch.int32).view(A, 2)
        n[:, 1] = -n[:, 1]
        aneg.append(n.view(torch.uint8).view(-1))
    torch.cuda.synchronize()
    asets = [DeviceBatch([b.data_ptr() for b in s], [b.numel() for b in s]) for s in (apos, aneg)]
    k = [0]

    def step():
        store.pushDevice(sets[k[0] & 1])
        astore.pushDevice(asets[k[0] & 1])
        k[0] += 1

    def finish():
        store.flush()
        astore.flush()

    store.set_timing(True)
    for _ in range(args.c5_warmup):
        step()
    finish()
    store.kernel_time(reset=True)
    steps = args.c5_steps + (args.c5_steps & 1)  # even: the counts return to their start
    el = timed_steps(ctx, step, finish, steps, 0)
    k_ms, k_n = store.kernel_time(reset=True)
    store.set_timing(False)
    assert store.error_state()[0] == 0, store.error_state()
    assert astore.error_state()[0] == 0, astore.error_state()
    astore.close()
    touched = int(round(S * (1 - (1 - nrec / S) ** C5_W)))
    # word-topic rows + doc-topic totals (each push byte once, the touched entries read and written once)
    algo_rows = C5_W * nrec * rec + 2 * 4 * cols * touched
    algo = algo_rows + C5_W * A * 8 + 2 * 4 * A
    algo_all = algo
    if world > 1:
        t = torch.tensor([float(algo)], dtype=torch.float64, device=ctx.coll_device())
        ctx.dist.all_reduce(t)
        algo_all = float(t.item())
    out = {"workload": f"config5: LDA IntMatrixStore {C5_ROWS}x{cols} int32 (negativity check), {C5_W} pushes x "
                       f"{C5_NNZ} distinct rows split per shard, plus the IntArrayStore doc-topic totals ({C5_TOPICS} "
                       f"topics, {C5_W} pushes of every topic); this rank: shard of {S} rows, {nrec} records per push, "
                       f"{A} topics",
           "value": round(algo_all * steps / el / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
           "pushes": C5_W, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3), "scaling": "strong",
           "dtype": "i32", "parallelism": "single shard" if world == 1 else f"linearSplit({world}), client-split pushes",
           "algorithmic_bytes_per_step_per_gpu": algo, "algorithmic_bytes_per_step": int(algo_all)}
    if k_n:
        # the word-topic reduce is the dominant kernel (the doc-topic totals' partition and
        # leaf, 256 KB per step, run beside it on the array store's streams)
        k_s = k_ms / k_n / 1e3
        kn = store.kernel_name()
        tr = traffic_for("leg5", kn) if world == 1 else {"traffic": None, "traffic_stale": "profiled at N = 1 only"}
        out["roofline"] = {"bound": "hbm", "achieved": round(algo_rows / k_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(algo_rows / k_s / 1e9 / HBM_PEAK_GBS, 4),
                           **tr, "kernel": kn, "rank": rank, "algorithmic_bytes_per_launch": algo_rows,
                           "avg_kernel_us": round(k_s * 1e6, 1), "launches": k_n}
        # the same records gathered by row into the touched rows, plain (dml_diag_gather_floor:
        # no key index, slot table or negativity check), timed after the steps into the
        # store's shard (left as it was: the pushes and their negations, applied in turn)
        fl = gather_floor(L, torch, store, pos + neg, S, cols, shard.firstKey, rec, st)
        out["roofline"]["measured_gather_floor_us"] = round(fl * 1e3, 1)
        out["roofline"]["frac_of_measured_floor"] = round(fl * 1e-3 / k_s, 3)
    store.close()
    del pos, neg, sets
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = leg_cpu_baseline("5")
    return out


def dense_floor(L, store, ptrs, lens, st, reps: int = 3):
    """Best of `reps` dml_diag_dense_floor runs (ms) over the leg's own shard and pushes
    (the same allocations), and whether it wrote out of place (k_flat_ident's layout)."""
    n = len(ptrs)
    P, Ln = (C.c_void_p * n)(*ptrs), (C.c_int64 * n)(*lens)
    best, ms, oop = None, C.c_float(), C.c_int32()
    for _ in range(reps):
        assert L.dml_diag_dense_floor(C.c_void_p(store._h), P, Ln, n, C.c_void_p(st), C.byref(ms), C.byref(oop)) == 0
        best = ms.value if best is None else min(best, ms.value)
    return best, bool(oop.value)


def gather_floor(L, torch, store, bufs, rows, cols, first, rec, st, reps: int = 3) -> float:
    """Best of `reps` dml_diag_gather_floor runs (ms) over the records of `bufs`: the
    first half ([:W]) then the second ([W:]) in turn, so the shard ends where it began.
    Row lists are built on the device: every record's row, stable-sorted by row, with
    the records of one row in push order."""
    half = len(bufs) // 2
    lists = []
    for part in (bufs[:half], bufs[half:]):
        rows_l, addr_l = [], []
        for b in part:
            r = b.view(-1, rec)[:, :4].contiguous().view(torch.int32).view(-1).to(torch.int64) - first
            rows_l.append(r)
            addr_l.append(b.data_ptr() + 4 + torch.arange(r.numel(), device="cuda", dtype=torch.int64) * rec)
        r = torch.cat(rows_l)
        a = torch.cat(addr_l)
        o = torch.sort(r, stable=True).indices
        r, a = r[o], a[o]
        cnt = torch.bincount(r, minlength=rows)
        trow = torch.nonzero(cnt).view(-1).to(torch.int32)
        tptr = torch.zeros(trow.numel() + 1, dtype=torch.int32, device="cuda")
        tptr[1:] = torch.cumsum(cnt[cnt > 0], 0).to(torch.int32)
        lists.append((trow, tptr, a.contiguous()))
    torch.cuda.synchronize()
    best, ms = None, C.c_float()
    for i in range(2 * reps):
        trow, tptr, a = lists[i & 1]
        assert L.dml_diag_gather_floor(C.c_void_p(store.device_ptr()), cols, C.c_void_p(trow.data_ptr()),
                                       C.c_void_p(tptr.data_ptr()), C.c_void_p(a.data_ptr()), trow.numel(),
                                       C.c_void_p(st), C.byref(ms)) == 0
        best = ms.value if best is None else min(best, ms.value)
    del lists
    return best


# ---------------------------------------------------------------- configs 4 and 5, one shard
# One GPU's shard of BASELINE.json configs 4 and 5 (8-GPU configs):
# the rows linearSplit(8) gives one rank, device-resident pushes of the named
# shapes, the store's ordered batch reduce. `python bench.py --config 5|4`.
SHARD_CONFIGS = {
    "5": dict(name="config5: LDA IntMatrixStore shard 125000x1000 int32 (negativity check), "
                   "32 pushes x 8192 distinct rows ([int32][1000 x int32])",
              rows=125_000, cols=1000, W=32, nrec=8192, vt=0, ada=None, seed0=4000, mult=331, init=11, steps=20),
    # config 4's metric is the plain sum (FloatMatrixStore), W = 8 and 32; AdaGrad is its variant.
    # full-range gradients, keys implicit = row, i.e. every push lists the
    # rows in ascending order (also Java HashMap<Integer>'s iteration order of a full key
    # set); "4-perm" permutes the rows of every push (seeded), the harder layout.
    "4": dict(name="config4: Word2Vec rows, FloatMatrixStore shard 1250000x200 fp32, 8 full-range pushes "
                   "([int32][200 x f32], rows ascending)",
              rows=1_250_000, cols=200, W=8, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919, init=13,
              steps=10, asc=True),
    "4-perm": dict(name="config4 with the rows of every push permuted (seeded): FloatMatrixStore shard "
                        "1250000x200 fp32, 8 full-range pushes",
                   rows=1_250_000, cols=200, W=8, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919, init=13,
                   steps=10),
    "4-32": dict(name="config4 (W=32): Word2Vec rows, FloatMatrixStore shard 1250000x200 fp32, 32 full-range pushes "
                      "(rows ascending)",
                 rows=1_250_000, cols=200, W=32, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919, init=13,
                 steps=5, asc=True),
    "4-256": dict(name="config4 shape probe: FloatMatrixStore shard 1250000x256 fp32 (whole 1-KiB rows), 8 full-range "
                       "pushes", rows=1_250_000, cols=256, W=8, nrec=1_250_000, vt=1, ada=None, seed0=3000, mult=7919,
                  init=13, steps=10),
    "4-ada": dict(name="config4 AdaGrad variant: FloatMatrixStoreAdaGrad shard 1250000x200 fp32 (data + alpha + "
                       "delta), 8 full-range pushes",
                  rows=1_250_000, cols=200, W=8, nrec=1_250_000, vt=1, ada=(0.025, 0.0001, 1.0), seed0=3000,
                  mult=7919, init=13, steps=5),
}


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
            "kind": "port", "sample": f"{nb} pushes of the same shapes in {el:.1f} s, oracle/dml_oracle.c",
            "host": host_info()}


def run_shard_config(which: str, cpu_s: float, no_cpu: bool) -> dict:
    import torch
    from distml_amd import DataDesc, DataStore, KeyRange, _lib
    c = SHARD_CONFIGS[which]
    L = _lib.load()
    rows, cols, W_, nrec = c["rows"], c["cols"], c["W"], c["nrec"]
    fmt = DataDesc(1, 0, c["vt"], False, True, c["ada"] is not None)
    hbm_check(torch, "config " + which, {"pushes": (2 if c["vt"] == 0 else 1) * W_ * nrec * (4 + 4 * cols),
                                         "store": store_bytes(rows, cols, 4, spec=c["vt"] == 1 and not c["ada"],
                                                              ada=c["ada"] is not None)})
    store = DataStore(fmt, KeyRange(0, rows - 1), cols)
    if c["ada"]:
        store.setAlpha(*c["ada"])
    store.synth_fill(c["init"])
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
    touched = rows if nrec >= rows else int(round(rows * (1 - (1 - nrec / rows) ** W_)))
    # AdaGrad: data and delta read and written (alpha written only where delta ends above 1: never here)
    algo = W_ * nrec * (4 + 4 * cols) + 2 * (2 if c["ada"] else 1) * 4 * cols * touched
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
    kn = store.kernel_name()
    assert store.error_state()[0] == 0, store.error_state()
    store.close()
    del bufs, sets
    torch.cuda.empty_cache()
    k_s = k_ms / max(k_n, 1) / 1e3
    line = {"metric": "device-resident push reduce GiB/s (one GPU's shard)", "value": round(steps * algo / el / 2**30, 1),
            "unit": "GiB/s", "n_gpus": 1, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
            "higher_is_better": True, "dtype": "i32" if c["vt"] == 0 else "f32", "data": "synthetic",
            "config": {"workload": c["name"], "rows": rows, "cols": cols, "pushes": W_, "records_per_push": nrec,
                       "algorithmic_bytes_per_step": algo},
            "roofline": {"bound": "hbm", "achieved": round(algo / k_s / 1e9, 1) if k_n else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / k_s / 1e9 / HBM_PEAK_GBS, 4) if k_n else None,
                         "kernel_us_avg": round(k_s * 1e6, 1), "kernel": kn,
                         **traffic_for("cfg" + which.replace("-", ""), kn)}}
    if not no_cpu:
        line["cpu_baseline"] = shard_cpu_baseline(c, cpu_s)
    return line


# ---------------------------------------------------------------- main
def launcher_check(args, out):
    """CPU-only rehearsal of the multi-rank plumbing (tests/test_bench_launcher.py):
    the same env / rendezvous / max-over-ranks / rank-0 line, over gloo, no GPU."""
    import torch
    import torch.distributed as dist
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t0 = time.perf_counter()
    time.sleep(0.02 * (rank + 1))
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "launcher-check", "value": float(t.item()), "n_gpus": world,
                          "ranks_seen": world, "local_rank": int(os.environ["LOCAL_RANK"])}), file=out, flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~0.2 s of warmup and ~0.4 s timed at N=1 by default
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    ap.add_argument("--no-timing", action="store_true", help="no kernel timing events in the timed region")
    ap.add_argument("--sparse-steps", type=int, default=20, help="config-3 sparse leg steps (0 = skip; N=1 only)")
    ap.add_argument("--pieces", type=int, default=1, help="pre-reduce row slices per call (sharded path)")
    ap.add_argument("--sparse-cu-split", type=int, default=0,
                    help="config 3: CUs of the partition's stream (| pattern << 16; 0 = every CU for both)")
    ap.add_argument("--shuffle-keep-parity", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--shuffle-orders", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--alloc-seed", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--push-layout", choices=["auto", "slab", "separate"], default="auto",
                    help="push buffers: auto = config 2 and 5 one allocation per push, configs 4 / 4a one slab "
                         "(diagnostic override for every leg)")
    ap.add_argument("--separate-buffers", action="store_true", help="= --push-layout separate")
    ap.add_argument("--shuffle-only", choices=["", "asc", "perm"], default="", help=argparse.SUPPRESS)
    ap.add_argument("--emulate-rs", type=int, default=0,
                    help="diagnostic with --group at N = 1: the owner-side HBM footprint of an N-rank "
                         "ring reduce-scatter + 1/N apply (results not valid)")
    ap.add_argument("--emulate-channels", type=int, default=RS_CHANNELS,
                    help="--emulate-rs: blocks of the ring reduce-scatter footprint (RCCL: one per channel)")
    ap.add_argument("--index-normal-prio", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--native-group", action="store_true",
                    help="also run the config-2 workload through dml_group at N = 1 (always at N > 1)")
    ap.add_argument("--group", action="store_true",
                    help="use the sharded pre-reduce/reduce-scatter path even at N=1 (path check)")
    ap.add_argument("--legs", default="4,4w,5,4a",
                    help="model-level config legs in the line (4, 4w = config 4 at W 8 and 32, 5, 4a; '' = none)")
    ap.add_argument("--c4-pushes", type=int, default=16, help="config-4 full-range pushes per GPU (8.04 GB each)")
    ap.add_argument("--c4-order", choices=["asc", "perm"], default="asc",
                    help="config-4 row order per push: ascending (SURVEY §8d, keys implicit = row) or permuted")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--c4-warmup", type=int, default=2)
    ap.add_argument("--c4a-pushes", type=int, default=2, help="config-4 AdaGrad full-range pushes per GPU")
    ap.add_argument("--c4a-steps", type=int, default=3)
    ap.add_argument("--c4a-path", choices=["exchange", "moments"], default="exchange",
                    help="config-4 AdaGrad leg: the exact exchange path, or the two-moment reduce-scatter")
    ap.add_argument("--c4a-warmup", type=int, default=3, help="(the exchange buffer pool fills in the first calls)")
    ap.add_argument("--c5-steps", type=int, default=20)
    ap.add_argument("--c5-warmup", type=int, default=4)
    ap.add_argument("--config", choices=["2", "4", "4-perm", "4-32", "4-256", "4-ada", "5"], default="2",
                    help="2 = the headline line (default); 4, 4-32, 4-ada, 5 = one GPU's shard of those configs")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline budget for --config 4/5")
    ap.add_argument("--launcher-check", action="store_true", help=argparse.SUPPRESS)
    # rehearsal of the N-rank legs on a one-GPU box: every rank on cuda:0, gloo collectives
    # (RCCL refuses two ranks on one device); numbers from it are not measurements
    ap.add_argument("--rehearse-gloo", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    layout = "separate" if args.separate_buffers else args.push_layout
    if layout != "auto":
        SLAB[0] = SLAB4[0] = layout == "slab"
    # RCCL's channel count for the torch binding's reduce-scatter, pinned before any GPU
    # call (RCCL reads it at communicator creation; the native group pins the same count
    # through ncclCommInitRankConfig): the one-GPU ring emulation favours
    # 128 blocks at N = 4 and 8 over RCCL's own choice
    for k in ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS"):
        os.environ.setdefault(k, str(RS_CHANNELS))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    # stdout carries exactly the one JSON line: RCCL and other native libraries print
    # banners to fd 1 (e.g. "RCCL version : ..."), so fd 1 goes to stderr for the run
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.launcher_check:
        launcher_check(args, out)
        return
    if args.config != "2":
        assert args.gpus == 1, "--config 4/5 measure one GPU's shard; the N-GPU legs run in the default line"
        print(json.dumps(run_shard_config(args.config, args.cpu_seconds, args.no_cpu)), file=out, flush=True)
        return

    import torch
    import torch.distributed as dist
    from distml_amd import _lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    if args.rehearse_gloo:
        local = 0
    torch.cuda.set_device(local)
    if world > 1 and args.rehearse_gloo:
        dist.init_process_group("gloo")
    elif world > 1 or args.group:
        # RCCL's collectives run on a high-priority stream: when a reduce-scatter and
        # the next call's pre-reduce compete for CUs, the collective's blocks go first
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local),
                                    pg_options=opts)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), pg_options=opts)
    L = _lib.load()
    ctx = Ctx(torch, dist, world, rank, local)

    line: dict = {}
    headline(ctx, L, args, line)
    legs = [x for x in args.legs.split(",") if x]
    if "4" in legs:
        line["config4"] = leg_config4(ctx, L, args)
    if "4w" in legs:
        # config 4 at W = 8 (one push per GPU of the 8-GPU job) and W = 32 (at
        # the most rows whose 32 pushes fit beside the store: 32 x 8.04 GB exceed 288 GB at 10 M)
        share = world if args.rehearse_gloo else 1  # rehearsal: every rank on one GPU
        line["config4_w8"] = leg_config4(ctx, L, args, w=8, rows=c4_fit_rows(ctx, 8, share=share), cpu=False)
        line["config4_w32"] = leg_config4(ctx, L, args, w=32, rows=c4_fit_rows(ctx, 32, share=share), cpu=False)
    if "5" in legs:
        line["config5"] = leg_config5(ctx, L, args)
    if "4a" in legs:
        line["config4_ada"] = leg_config4_ada(ctx, L, args)
    if (world > 1 and not args.rehearse_gloo) or args.native_group:
        line["native_group"] = guarded_leg(ctx, line, out, "native_group", lambda: leg_native_group(ctx, L, args),
                                           seconds=180.0)
    if world == 1 and not args.group and args.sparse_steps > 0:
        line["sparse"] = sparse_leg(ctx, L, args.sparse_steps, cpu=not args.no_cpu, cu_split=args.sparse_cu_split)
    if rank == 0 and world == 1 and not args.no_cpu and not args.group:
        line["cpu_baseline"] = cpu_baseline()
    if args.rehearse_gloo and world > 1:
        # diagnostic only: the collectives ran over gloo through host memory with every
        # rank on one GPU, so the timing says nothing about xGMI / RCCL
        line["rehearsal"] = f"gloo collectives, {world} ranks sharing cuda:0 (schedule check, not a measurement)"
    if rank == 0:
        print(json.dumps(line), file=out, flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
