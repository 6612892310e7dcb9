"""Per-GPU measurements of BASELINE.json configs 4 and 5 on one
MI355X: the shard one GPU owns under linearSplit(8), device-resident pushes of
the named shapes, the store's ordered batch reduce (the same C-ABI path as the
bench's config 2), algorithmic GiB/s by the §8d byte count, the reduce kernel's
average time from its in-packet HIP events, and the CPU oracle (1 thread) on a
bounded sample of the same pushes.

  config 5 (LDA):      IntMatrixStore shard 125 000 x 1 000 int32 (negativity
                       check on), 32 pushes x 8 192 distinct rows ([int32][1000 x int32]).
  config 4 (Word2Vec): FloatMatrixStoreAdaGrad shard 1 250 000 x 200 fp32
                       (data + alpha + delta), 8 full-range pushes ([int32][200 x f32]).

Prints one JSON line per config. Synthetic data."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pyoracle  # noqa: E402
from distml_amd import DataDesc, DataStore, KeyRange, _lib  # noqa: E402


def synth(L, fmt, rows, nrec, cols, seeds, perms):
    st = torch.cuda.current_stream().cuda_stream
    rec = 4 + 4 * cols
    out = []
    for sd, (pa, pc) in zip(seeds, perms):
        t = torch.empty(nrec * rec, dtype=torch.uint8, device="cuda")
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows, nrec, cols, sd, pa, pc,
                                        C.c_void_p(st)) == 0
        out.append(t)
    torch.cuda.synchronize()
    return out


def coprime(a, n):
    while np.gcd(a, n) != 1:
        a += 1
    return a


def run(name, fmt, rows, cols, nrec, W, seeds, perms, init_seed, steps, cpu_budget_s, ada=None):
    L = _lib.load()
    store = DataStore(fmt, KeyRange(0, rows - 1), cols)
    if ada:
        store.setAlpha(*ada)
    store.rand(init_seed)
    bufs = synth(L, fmt, rows, nrec, cols, seeds, perms)
    rec = 4 + 4 * cols
    sets = [([b.data_ptr() for b in bufs], [b.numel() for b in bufs])]
    if fmt.valueType == 0:
        # int32 counts: alternate the pushes with their negation so repeated steps do
        # not drift the counts below zero (the negativity check would stop the store)
        neg = []
        for b in bufs:
            t = b.clone().view(torch.int32).view(nrec, 1 + cols)
            t[:, 1:] = -t[:, 1:]
            neg.append(t.view(torch.uint8).view(-1))
        bufs = bufs + neg
        sets.append(([b.data_ptr() for b in neg], [b.numel() for b in neg]))
    torch.cuda.synchronize()
    # every push byte once + the touched shard rows read and written once
    # (AdaGrad: + alpha and delta read and written)
    touched = rows if nrec >= rows else int(round(rows * (1 - (1 - nrec / rows) ** W)))
    arrays = 3 if ada else 1
    algo = W * nrec * rec + 2 * arrays * 4 * cols * touched
    for i in range(4):
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
    del bufs
    store.close()
    torch.cuda.empty_cache()
    # CPU oracle on a bounded sample: the first pushes of the same workload
    host = [pyoracle.synth_dense_bucket(0, fmt.valueType, 0, rows, nrec, cols, sd, pa, pc)
            for sd, (pa, pc) in zip(seeds[:4], perms[:4])]
    if fmt.valueType == 0:  # alternate with the negated pushes, as on the GPU
        negs = []
        for h in host:
            t = h.view(np.int32).reshape(nrec, 1 + cols).copy()
            t[:, 1:] = -t[:, 1:]
            negs.append(t.view(np.uint8).reshape(-1))
        host = [x for pair in zip(host, negs) for x in pair]
    o = pyoracle.OracleStore(1, 0, fmt.valueType, 0, rows - 1, cols, ada_grad=1 if ada else 0)
    if ada:
        o.set_alpha(*ada)
    o.synth_fill(init_seed)
    nb, c0 = 0, time.perf_counter()
    while time.perf_counter() - c0 < cpu_budget_s:
        assert o.push(host[nb % len(host)]) == 0
        nb += 1
    cel = time.perf_counter() - c0
    cpu_bytes = nb * nrec * rec  # push bytes applied (the shard traffic of a push is inside)
    return {"config": name, "rows": rows, "cols": cols, "pushes": W, "records_per_push": nrec,
            "algorithmic_bytes_per_step": algo, "ms_per_step": round(el / steps * 1e3, 3),
            "value_GiBps": round(steps * algo / el / 2**30, 1),
            "reduce_kernel_us_avg": round(k_ms / max(k_n, 1) * 1e3, 1),
            "kernel_TBps": round(algo / (k_ms / max(k_n, 1) / 1e3) / 1e12, 3) if k_n else None,
            "cpu_baseline": {"GiBps_of_push_bytes": round(cpu_bytes / cel / 2**30, 3), "cores": 1, "kind": "port",
                             "sample": f"{nb} pushes of the same shapes in {cel:.1f} s"}}


def main():
    which = sys.argv[1:] or ["5", "4"]
    if "5" in which:
        rows, cols, W, nrec = 125_000, 1000, 32, 8192
        perms = [(coprime((4000 + b) * 2654435761 % rows | 1, rows), b * 331 % rows) for b in range(W)]
        print(json.dumps(run("config5 LDA IntMatrixStore shard 125000x1000 int32, 32 pushes x 8192 rows",
                             DataDesc(1, 0, 0), rows, cols, nrec, W, [4000 + b for b in range(W)], perms, 11,
                             steps=20, cpu_budget_s=float(os.environ.get("CFG_CPU_S", "8.0")))), flush=True)
    if "4" in which:
        rows, cols, W = 1_250_000, 200, 8
        perms = [(coprime((3000 + b) * 2654435761 % rows | 1, rows), b * 7919 % rows) for b in range(W)]
        print(json.dumps(run("config4 Word2Vec FloatMatrixStoreAdaGrad shard 1250000x200 fp32, 8 full-range pushes",
                             DataDesc(1, 0, 1, False, True, True), rows, cols, rows, W,
                             [3000 + b for b in range(W)], perms, 13, steps=5, cpu_budget_s=float(os.environ.get("CFG_CPU_S", "8.0")),
                             ada=(0.025, 0.0001, 1.0))), flush=True)


if __name__ == "__main__":
    main()
