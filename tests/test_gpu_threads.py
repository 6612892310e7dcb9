"""GPU: one store called from several host threads at once, as the reference does.

The reference calls a store from three threads: the PSAgent
selector thread pushes under `synchronized(store)` (PSAgent.java:278-280), the same
thread fetches without the lock (PSAgent.java:265), and PSActor / PSSync call
rand/zero/set, writeAll and syncTo from their own threads (PSActor.java:171-201,
PSSync.java:131). The library serializes every call on the store's mutex
(include/distml_ps.h, threading contract); these tests drive pushes, fetches and
checkpoints from concurrent threads and compare the final shard with the oracle.

- int32 counts: additions commute, so the final shard is the same for every
  interleaving of the threads' pushes; every checkpoint taken meanwhile lies
  between the initial and the final shard element-wise (all deltas >= 0).
- fp32: each thread owns a disjoint row set and pushes in its own order, so the
  final shard is exact whatever the interleaving.
"""
import threading

import numpy as np
import pytest

import kat

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run_threads(fns):
    errs = []

    def wrap(fn):
        try:
            fn()
        except BaseException as e:  # surfaced in the main thread below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a caller thread did not finish"
    if errs:
        raise errs[0]


@pytest.mark.parametrize("async_push", [False, True], ids=["sync", "async"])
def test_int32_pushes_fetches_checkpoints_from_threads(oracle, async_push):
    from distml_amd import DataDesc, DataStore, KeyRange, encode_matrix_push
    rows, cols, T, P, n = 4096, 64, 4, 8, 512
    fmt = DataDesc(1, 0, 0)
    s = DataStore(fmt, KeyRange(0, rows - 1), cols, async_push=async_push)
    o = oracle.OracleStore(fmt.dataType, fmt.keyType, fmt.valueType, 0, rows - 1, cols, int(fmt.denseColumn),
                           int(fmt.adaGrad), 0)
    s.synth_fill(5)
    o.synth_fill(5)
    init = s.values().copy()
    rng = np.random.default_rng(77)
    pushes = [[encode_matrix_push(rng.permutation(rows)[:n], rng.integers(0, 4, (n, cols)), 0, 0)
               for _ in range(P)] for _ in range(T)]
    dumps, fetched = [], []

    def pusher(t):
        def run():
            for p in pushes[t]:
                s.handlePush(fmt, p)
        return run

    def fetcher():
        # handleFetch runs unlocked in the reference (PSAgent.java:265)
        for i in range(20):
            lo = (i * 193) % rows
            fetched.append(len(s.handleFetch(fmt, KeyRange(lo, min(lo + 255, rows - 1)))))

    def checkpointer():
        for _ in range(5):
            be = np.frombuffer(s.writeAll(), dtype=">i4").astype(np.int32).reshape(rows, cols)
            dumps.append(be)

    _run_threads([pusher(t) for t in range(T)] + [fetcher, checkpointer])
    s.flush()
    for t in range(T):
        for p in pushes[t]:
            assert o.push(p) == 0
    final = s.values()
    assert kat.bits_equal(final, o.data)
    assert len(fetched) == 20 and all(f > 0 for f in fetched)
    for d in dumps:  # every checkpoint is a state between the initial and the final shard
        assert (d >= init).all() and (d <= final).all()


def test_fp32_disjoint_rows_from_threads(oracle):
    from distml_amd import DataDesc, DataStore, KeyRange, encode_matrix_push
    rows, cols, T, P = 8192, 200, 4, 6
    fmt = DataDesc(1, 0, 1)
    s = DataStore(fmt, KeyRange(0, rows - 1), cols)
    o = oracle.OracleStore(fmt.dataType, fmt.keyType, fmt.valueType, 0, rows - 1, cols, int(fmt.denseColumn),
                           int(fmt.adaGrad), 0)
    s.synth_fill(9)
    o.synth_fill(9)
    rng = np.random.default_rng(78)
    own = np.array_split(rng.permutation(rows), T)  # thread t owns rows own[t]
    pushes = []
    for t in range(T):
        ps = []
        for _ in range(P):
            r = rng.permutation(own[t])[: len(own[t]) * 3 // 4]
            ps.append(encode_matrix_push(r, rng.standard_normal((len(r), cols)).astype(np.float32), 0, 1))
        pushes.append(ps)

    def pusher(t):
        def run():
            for i in range(0, P, 2):  # single pushes and two-push batches, like a PS's ingest
                if i % 4 == 0:
                    s.handlePush(fmt, pushes[t][i])
                    s.handlePush(fmt, pushes[t][i + 1])
                else:
                    s.handlePushBatch(fmt, pushes[t][i:i + 2])
        return run

    _run_threads([pusher(t) for t in range(T)])
    s.flush()
    for t in range(T):  # disjoint rows: the threads' interleaving does not change the sums
        for p in pushes[t]:
            assert o.push(p) == 0
    assert kat.bits_equal(s.values(), o.data)
