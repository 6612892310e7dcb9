"""Config-1 harness (BASELINE.json configs[0]): the MNIST
softmax-regression sample with 2 worker processes and 1 parameter server over
loopback TCP, speaking the reference framing (distml_amd.psnet).

  data     synthetic MNIST-shaped text lines, "784 pixel ints 0..255 then the
           label" (MNISTReader.java:53-62), seed 1; the real set needs wget
           (data/mnist_prepare.sh:2-3). Parsed like Mnist.scala:113-127 (only
           non-zero pixels become features; one-hot label).
  model    MLRModel: DoubleMatrix(784, 10) "weights" (MLR.scala:19-26) — MATRIX,
           LONG keys, DOUBLE values, dense columns (DoubleMatrix.java:13).
  worker   MLR.train's per-partition loop (MLR.scala:51-133): per batch, fetch the
           batch's feature keys (a KeyList), SGD on a copy with softmax, push
           w - w_old for every fetched key.
  server   one shard KeyRange(0, 783) behind PSServer: a DataStore (GPU) or any
           store with the same two calls (the CPU oracle in the CPU tests).

Result check: the server's final shard must equal a CPU-oracle replay of the
pushes it received, in its arrival order (the order that defines the result).
The workers' own arithmetic is the sample's, not the product: it only feeds
pushes through the path.
"""
from __future__ import annotations

import hashlib
import math
import struct
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .datadesc import DataDesc, KeyList, KeyRange
from .psnet import PSClient

INPUT_DIM, OUTPUT_DIM = 784, 10
WEIGHTS = "weights"
MLR_FORMAT = DataDesc(DataDesc.DATA_TYPE_MATRIX, DataDesc.KEY_TYPE_LONG, DataDesc.ELEMENT_TYPE_DOUBLE)


def mnist_lines(n: int = 1000, seed: int = 1) -> List[str]:
    """Synthetic MNIST-shaped lines: ~19 % of the pixels non-zero (1..255) in a
    label-dependent band, the label 0..9 last (MNISTReader.java:53-62)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        label = int(rng.integers(0, 10))
        px = np.zeros(INPUT_DIM, np.int64)
        lo = 28 * (2 + 2 * label)
        idx = rng.choice(np.arange(lo, min(lo + 300, INPUT_DIM)), size=150, replace=False)
        px[idx] = rng.integers(1, 256, size=150)
        out.append(" ".join(str(int(v)) for v in px) + " " + str(label))
    return out


def parse_line(line: str) -> Tuple[Dict[int, float], np.ndarray]:
    """Mnist.scala:113-126: features i with a non-zero value, one-hot label."""
    items = line.split(" ")
    data = {}
    for i in range(len(items) - 1):
        v = float(items[i])
        if v != 0.0:
            data[i] = v
    label = np.zeros(OUTPUT_DIM)
    label[int(items[-1])] = 1.0
    return data, label


def encode_rows(rows: Dict[int, np.ndarray]) -> bytes:
    """SparseMatrix.writeMap dense-column layout (SparseMatrix.java:96-125):
    [LE int64 key][10 x LE float64] per row."""
    return b"".join(struct.pack("<q", k) + np.asarray(v, "<f8").tobytes() for k, v in rows.items())


def decode_rows(buf: bytes) -> Dict[int, np.ndarray]:
    """SparseMatrix.readMap (SparseMatrix.java:62-94), dense columns."""
    rec = 8 + 8 * OUTPUT_DIM
    out = {}
    for o in range(0, len(buf), rec):
        k = struct.unpack_from("<q", buf, o)[0]
        out[k] = np.frombuffer(buf, "<f8", OUTPUT_DIM, o + 8).copy()
    return out


def _softmax(x: np.ndarray) -> None:
    """MLR.softmax (MLR.scala:30-40), in place, sequential sums."""
    mx = max(x)
    s = 0.0
    for i in range(len(x)):
        x[i] = math.exp(x[i] - mx)
        s += x[i]
    for i in range(len(x)):
        x[i] /= s


def train_partition(address, lines: Sequence[str], batch_size: int = 100, iterations: int = 1,
                    lr: float = 0.1) -> Tuple[float, List[str]]:
    """One worker: MLR.train's partition loop (MLR.scala:51-133), `iterations` passes.
    Returns (cost of the last batch, sha256 of every push sent, in order)."""
    samples = [parse_line(l) for l in lines]
    cli = PSClient(address)
    cost, pushes = 0.0, []
    try:
        for _ in range(iterations):
            for b0 in range(0, len(samples), batch_size):
                batch = samples[b0:b0 + batch_size]
                keys = KeyList(k for x, _ in batch for k in x)
                w = decode_rows(cli.fetch(WEIGHTS, MLR_FORMAT, keys))
                w_old = {k: v.copy() for k, v in w.items()}
                cost = 0.0
                for x, label in batch:
                    p = np.zeros(OUTPUT_DIM)
                    for i in range(OUTPUT_DIM):
                        for k, xv in x.items():
                            p[i] += w[k][i] * xv
                    _softmax(p)
                    for i in range(OUTPUT_DIM):
                        dy = label[i] - p[i]
                        for k, xv in x.items():
                            w[k][i] += lr * dy * xv
                        if label[i] > 0.0:
                            cost += label[i] * math.log(p[i]) if p[i] > 0.0 else -math.inf
                cost /= len(batch)
                data = encode_rows({k: w[k] - w_old[k] for k in w})
                if not cli.push(WEIGHTS, MLR_FORMAT, data):
                    raise RuntimeError("push refused")
                pushes.append(hashlib.sha256(data).hexdigest())
    finally:
        cli.close()
    return cost, pushes


def worker_main(address, lines, batch_size, iterations, q) -> None:
    """multiprocessing entry point (a Spark task of MLR.train)."""
    try:
        q.put(("ok",) + train_partition(tuple(address), lines, batch_size, iterations))
    except BaseException as e:  # report, then fail the process
        q.put(("error", repr(e), []))
        raise


def run(stores_for_server, n_lines: int = 1000, workers: int = 2, batch_size: int = 100,
        iterations: int = 1, timeout: float = 300.0):
    """Start one PSServer over `stores_for_server` ({name: (store, fmt)}), run
    `workers` worker processes on contiguous partitions of the synthetic lines,
    return (server, [(status, cost, push digests)])."""
    import multiprocessing as mp

    from .psnet import PSServer

    lines = mnist_lines(n_lines)
    server = PSServer(stores_for_server).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    per = (len(lines) + workers - 1) // workers
    procs = [ctx.Process(target=worker_main,
                         args=(server.address, lines[i * per:(i + 1) * per], batch_size, iterations, q))
             for i in range(workers)]
    results = []
    try:
        for p in procs:
            p.start()
        for _ in procs:
            results.append(q.get(timeout=timeout))
        for p in procs:
            p.join(timeout=timeout)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join()
        server.stop()
    return server, results


def shard_range() -> KeyRange:
    return KeyRange(0, INPUT_DIM - 1)
