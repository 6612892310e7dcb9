"""GPU parity: libdistml_ps (HIP, gfx950) against the CPU oracle, bit for bit.

Every comparison is exact (bytes equal): fp32/fp64 adds happen in push order
with one IEEE rounding each, int32 wraps; tolerance 0. Runs through the C-ABI
(via the distml_amd mirror) on cuda:0.
"""
import ctypes as C
import io

import numpy as np
import pytest

import kat

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()


def mk_store(case_or_desc, first=None, last=None, cols=1, ref_stride=False, async_push=False):
    from distml_amd import DataDesc, DataStore, KeyRange
    if isinstance(case_or_desc, dict):
        c = case_or_desc
        d = c["desc"]
        fmt = DataDesc(d["data_type"], d["key_type"], d["value_type"], False, bool(d["dense_column"]),
                       bool(d["ada_grad"]))
        return DataStore(fmt, KeyRange(c["first"], c["last"]), c["cols"],
                         float_array_ref_stride=bool(c["float_array_ref_stride"]), async_push=async_push), fmt
    fmt = case_or_desc
    return DataStore(fmt, KeyRange(first, last), cols, float_array_ref_stride=ref_stride,
                     async_push=async_push), fmt


def oracle_store(oracle, fmt, first, last, cols=1, ref_stride=False):
    return oracle.OracleStore(fmt.dataType, fmt.keyType, fmt.valueType, first, last, cols,
                              int(fmt.denseColumn), int(fmt.adaGrad), int(ref_stride))


# --------------------------------------------------------------------------- KATs
@pytest.mark.parametrize("mode", ["sequential", "batch"])
@pytest.mark.parametrize("case", kat.cases(), ids=lambda c: c["name"])
def test_kat_on_gpu(case, mode):
    from distml_amd import DistMLException
    s, fmt = mk_store(case)
    s.load_values(kat.init_array(case))
    if case["ada"]:
        s.setAlpha(*case["ada"])
    exp = case["expected"]
    err = None
    try:
        if mode == "sequential":
            for p in kat.pushes(case):
                s.handlePush(fmt, p)
        else:
            s.handlePushBatch(fmt, kat.pushes(case))
    except DistMLException as e:
        err = e
    if exp["status"]:
        assert err is not None and (err.code, err.key, err.col) == (exp["status"], exp["key"], exp["col"])
    else:
        assert err is None
    assert kat.bits_equal(s.values(), kat.expected_array(case))
    if case["ada"]:
        a, d = s.adagrad_state()
        assert kat.bits_equal(a, kat.expected_array(case, "alpha_hex", "<f4"))
        assert kat.bits_equal(d, kat.expected_array(case, "delta_hex", "<f4"))
        v, r, c = s.maxDelta()
        assert [v, r, c] == exp["max_delta"]
    s.close()


# ----------------------------------------------------------------- random parity
def rand_matrix_pushes(rng, first, rows, cols, key_type, value_type, n, row_frac=1.0, dup=False):
    from distml_amd import encode_matrix_push
    out = []
    for b in range(n):
        k = max(1, int(rows * row_frac))
        r = rng.choice(rows, size=k, replace=False)
        if dup:
            r = np.concatenate([r, rng.choice(r, size=max(1, k // 3))])
            rng.shuffle(r)
        if value_type == 0:
            v = rng.integers(-2, 3, size=(len(r), cols)).astype(np.int32)
        elif value_type == 1:
            v = (rng.standard_normal((len(r), cols)) * 1e-3).astype(np.float32)
        else:
            v = rng.standard_normal((len(r), cols)) * 1e-3
        out.append(encode_matrix_push(first + r, v, key_type, value_type))
    return out


@pytest.mark.parametrize("value_type,key_type,cols,nb,frac,dup", [
    (1, 0, 1024, 3, 1.0, False), (1, 0, 200, 9, 0.5, False), (1, 1, 37, 70, 0.3, False),
    (1, 0, 5, 4, 1.0, True), (3, 0, 10, 6, 0.7, False), (3, 1, 33, 3, 1.0, True),
    (0, 0, 1000, 5, 0.2, False), (0, 0, 7, 66, 0.5, False), (0, 1, 16, 3, 1.0, True),
    # rows wider than one wave's 4 chunks (two waves per row: neither hands the slot rows back)
    (1, 0, 1280, 4, 0.6, False), (1, 0, 2048, 3, 0.8, True), (3, 1, 640, 5, 0.5, False),
    (0, 0, 1500, 4, 0.5, False), (1, 0, 700, 4, 0.6, False),
])
@pytest.mark.parametrize("api", ["batch", "device", "device_calls"])
def test_matrix_random_parity(oracle, value_type, key_type, cols, nb, frac, dup, api):
    """Random pushes (key subsets, permuted, optionally repeated rows) for every value
    type and many widths, bit-exact. `device_calls`: one device call per push, six
    calls in flight over the three workspaces (slot tables handed back or memset)."""
    from distml_amd import DataDesc
    rng = np.random.default_rng(cols * 1000 + nb)
    first, rows = 1000, 300
    fmt = DataDesc(1, key_type, value_type)
    s, _ = mk_store(fmt, first, first + rows - 1, cols)
    o = oracle_store(oracle, fmt, first, first + rows - 1, cols)
    if value_type == 0:
        init = rng.integers(100, 200, size=(rows, cols)).astype(np.int32)
    else:
        init = rng.standard_normal((rows, cols)).astype(s.dtype)
    s.load_values(init)
    o.data[:] = init
    pushes = rand_matrix_pushes(rng, first, rows, cols, key_type, value_type, nb, frac, dup)
    for p in pushes:
        assert o.push(p) == 0
    if api == "batch":
        s.handlePushBatch(fmt, pushes)
    else:
        bufs = [torch.frombuffer(bytearray(p), dtype=torch.uint8).cuda() for p in pushes]
        torch.cuda.synchronize()
        if api == "device":
            s.pushDevice([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
        else:
            for b in bufs:
                s.pushDevice([b.data_ptr()], [b.numel()])
        s.flush()
    assert kat.bits_equal(s.values(), o.data)
    s.close()


@pytest.mark.parametrize("value_type,key_type,ref_stride", [(1, 1, False), (1, 1, True), (1, 0, False),
                                                             (0, 0, False), (3, 0, False), (3, 1, False)])
def test_array_random_parity(oracle, value_type, key_type, ref_stride):
    from distml_amd import DataDesc, encode_array_push
    rng = np.random.default_rng(value_type * 10 + key_type)
    first, rows = 5, 100_000
    fmt = DataDesc(0, key_type, value_type)
    s, _ = mk_store(fmt, first, first + rows - 1, ref_stride=ref_stride)
    o = oracle_store(oracle, fmt, first, first + rows - 1, ref_stride=ref_stride)
    init = (rng.integers(50, 60, size=(rows, 1)).astype(np.int32) if value_type == 0
            else rng.standard_normal((rows, 1)).astype(s.dtype))
    s.load_values(init)
    o.data[:] = init
    vs = 8 if (ref_stride and value_type == 1) else None
    pushes = []
    for b in range(12):
        k = rng.choice(rows, size=20_000, replace=False)
        v = (rng.integers(-2, 3, size=len(k)) if value_type == 0 else rng.standard_normal(len(k)) * 1e-3)
        pushes.append(encode_array_push(first + k, v, key_type, value_type, value_stride=vs))
    for p in pushes:
        assert o.push(p) == 0
    s.handlePushBatch(fmt, pushes)
    assert kat.bits_equal(s.values(), o.data)


@pytest.mark.parametrize("value_type,api", [(1, "batch"), (3, "batch"), (1, "sequential")])
def test_array_repeated_keys_in_push_exact(oracle, value_type, api):
    """A push that lists a key several times (never produced by SparseArray.writeMap, but
    legal bytes): the reference adds the repeats in record order. The ordered sparse path
    sorts (row, sequence) per leaf, so the result is bit-exact; per-push float atomics
    would not fix the order of the repeats."""
    from distml_amd import DataDesc, encode_array_push
    rng = np.random.default_rng(40 + value_type)
    first, rows = 0, 50_000
    fmt = DataDesc(0, 1, value_type)
    s, _ = mk_store(fmt, first, first + rows - 1)
    o = oracle_store(oracle, fmt, first, first + rows - 1)
    init = rng.standard_normal((rows, 1)).astype(s.dtype)
    s.load_values(init)
    o.data[:] = init
    pushes = []
    for b in range(6):
        k = rng.integers(0, 3_000, size=30_000)  # ~10 repeats of every key inside one push
        v = rng.standard_normal(len(k)) * np.float64(2.0) ** rng.integers(-30, 10, size=len(k))
        pushes.append(encode_array_push(first + k, v, 1, value_type))
    for p in pushes:
        assert o.push(p) == 0
    if api == "batch":
        s.handlePushBatch(fmt, pushes)
    else:
        for p in pushes:
            s.handlePush(fmt, p)
    assert kat.bits_equal(s.values(), o.data)
    s.close()


@pytest.mark.parametrize("value_type", [1, 3])
def test_array_skewed_leaf_replay_exact(oracle, value_type):
    """One key range holds far more records than a leaf sorts in LDS (2048): the leaf
    kernel flags it and the host replays it from a full device sort, exactly."""
    from distml_amd import DataDesc, encode_array_push
    rng = np.random.default_rng(7 + value_type)
    first, rows = 10, 1_000_000
    fmt = DataDesc(0, 0, value_type)
    s, _ = mk_store(fmt, first, first + rows - 1)
    o = oracle_store(oracle, fmt, first, first + rows - 1)
    init = rng.standard_normal((rows, 1)).astype(s.dtype)
    s.load_values(init)
    o.data[:] = init
    pushes = []
    for b in range(4):
        hot = rng.integers(0, 64, size=6_000)            # 6000 records on 64 keys: one oversized leaf
        cold = rng.choice(rows, size=20_000, replace=False)
        k = rng.permutation(np.concatenate([hot, cold]))
        v = rng.standard_normal(len(k)) * 1e-2
        pushes.append(encode_array_push(first + k, v, 0, value_type))
    for p in pushes:
        assert o.push(p) == 0
    s.handlePushBatch(fmt, pushes)
    assert kat.bits_equal(s.values(), o.data)
    # and a following batch after the replay (pipeline state intact)
    more = [encode_array_push(first + rng.choice(rows, 5_000, replace=False), rng.standard_normal(5_000), 0,
                              value_type) for _ in range(3)]
    for p in more:
        assert o.push(p) == 0
    s.handlePushBatch(fmt, more)
    assert kat.bits_equal(s.values(), o.data)
    s.close()


# ----------------------------------------------------------------- error semantics
@pytest.mark.parametrize("kind", ["key", "trunc", "neg"])
def test_batch_error_state_matches_sequential(oracle, kind):
    from distml_amd import DataDesc, DistMLException, encode_matrix_push
    rng = np.random.default_rng(7)
    first, rows, cols = 0, 64, 48
    vt = 0 if kind == "neg" else 1
    fmt = DataDesc(1, 0, vt)
    pushes = rand_matrix_pushes(rng, first, rows, cols, 0, vt, 6, 0.8)
    if kind == "key":
        cut = 5 * (4 + 4 * cols)
        pushes[3] = pushes[3][:cut] + encode_matrix_push([rows + 3], np.ones((1, cols)), 0, vt) + pushes[3][cut:]
    elif kind == "trunc":
        pushes[2] = pushes[2][:-(4 * cols // 2 + 2)]
    else:
        bad = np.zeros((1, cols), np.int32)
        bad[0, 17] = -1000
        pushes[2] = pushes[2] + encode_matrix_push([9], bad, 0, 0) + encode_matrix_push([10], bad, 0, 0)
    o = oracle_store(oracle, fmt, first, rows - 1, cols)
    init = (rng.integers(5, 9, size=(rows, cols)).astype(np.int32) if vt == 0
            else rng.standard_normal((rows, cols)).astype(np.float32))
    o.data[:] = init
    rc = 0
    for p in pushes:
        rc = o.push(p)
        if rc:
            break
    assert rc != 0
    for api in ("sequential", "batch"):
        s, _ = mk_store(fmt, first, rows - 1, cols)
        s.load_values(init)
        with pytest.raises(DistMLException) as ei:
            if api == "batch":
                s.handlePushBatch(fmt, pushes)
            else:
                for p in pushes:
                    s.handlePush(fmt, p)
        assert (ei.value.code, ei.value.key, ei.value.col) == o.error()
        assert kat.bits_equal(s.values(), o.data)
        # the failed store refuses further pushes (the reference's PS loop has ended)
        with pytest.raises(DistMLException):
            s.handlePush(fmt, pushes[0])
        s.close()


@pytest.mark.parametrize("cols", [48, 37, 1000, 1024, 2048, 3])
def test_int32_negative_widths_exact(oracle, cols):
    """IntMatrixStore's negativity check (IntMatrixStore.java:172-176) at every
    k_reduce_rows shape: whole-vector rows (48, 1000: the config-5 width, 1024: whole
    4-KiB rows, 2048: two waves per row), a ragged width (37) and rows narrower than one
    vector (3). The reduce ORs the counters after each add and replays a wave's adds from
    the shard only when one went negative (neg_first): the error, its (key, col) and the
    rolled-back store must equal the oracle's, for a negative reached mid-batch by a later
    push of a row two pushes list, and a second one further on."""
    from distml_amd import DataDesc, DistMLException, encode_matrix_push
    rng = np.random.default_rng(cols)
    first, rows = 0, 96
    fmt = DataDesc(1, 0, 0)
    pushes = rand_matrix_pushes(rng, first, rows, cols, 0, 0, 6, 0.7)
    c = cols // 2
    dip = np.zeros((1, cols), np.int32)
    dip[0, c] = -7                      # row 9 is 5..8: negative after this add ...
    lift = np.zeros((1, cols), np.int32)
    lift[0, c] = 100                    # ... and positive again after the next push's
    pushes[2] = pushes[2] + encode_matrix_push([9], dip, 0, 0)
    pushes[3] = encode_matrix_push([9], lift, 0, 0) + pushes[3]
    late = np.zeros((1, cols), np.int32)
    late[0, cols - 1] = -1000
    pushes[4] = pushes[4] + encode_matrix_push([40], late, 0, 0)
    init = rng.integers(5, 9, size=(rows, cols)).astype(np.int32)
    o = oracle_store(oracle, fmt, first, rows - 1, cols)
    o.data[:] = init
    rc = 0
    for p in pushes:
        rc = o.push(p)
        if rc:
            break
    assert rc != 0
    s, _ = mk_store(fmt, first, rows - 1, cols)
    s.load_values(init)
    with pytest.raises(DistMLException) as ei:
        s.handlePushBatch(fmt, pushes)
    assert (ei.value.code, ei.value.key, ei.value.col) == o.error()
    assert kat.bits_equal(s.values(), o.data)
    s.close()


@pytest.mark.parametrize("middle", ["normal", "dup", "key", "neg"])
def test_pipelined_batches(oracle, middle):
    """Several device batches in flight (no flush between them): a repeated row in
    the middle batch is replayed and the next batch relaunched; an error stops the
    store there (later batches never applied), surfacing at a later call."""
    from distml_amd import DataDesc, DistMLException, encode_matrix_push
    rng = np.random.default_rng({"normal": 1, "dup": 2, "key": 3, "neg": 4}[middle])
    rows, cols = 257, 40
    vt = 0 if middle == "neg" else 1
    fmt = DataDesc(1, 0, vt)
    batches = [rand_matrix_pushes(rng, 0, rows, cols, 0, vt, 5, 0.7) for _ in range(5)]
    if middle == "dup":
        batches[2] = rand_matrix_pushes(rng, 0, rows, cols, 0, vt, 5, 0.7, dup=True)
    elif middle == "key":
        batches[2][1] = batches[2][1] + encode_matrix_push([rows + 5], np.ones((1, cols), np.float32), 0, 1)
    elif middle == "neg":
        bad = np.zeros((1, cols), np.int32)
        bad[0, 3] = -10_000
        batches[2][3] = batches[2][3] + encode_matrix_push([7], bad, 0, 0)
    init = (rng.integers(10, 20, size=(rows, cols)).astype(np.int32) if vt == 0
            else rng.standard_normal((rows, cols)).astype(np.float32))
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    o.data[:] = init
    rc = 0
    for bt in batches:
        for p in bt:
            rc = o.push(p)
            if rc:
                break
        if rc:
            break
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    s.load_values(init)
    dev = [[torch.frombuffer(bytearray(p), dtype=torch.uint8).cuda() for p in bt] for bt in batches]
    torch.cuda.synchronize()
    err = None
    try:
        for bt in dev:
            s.pushDevice([b.data_ptr() for b in bt], [b.numel() for b in bt])
        s.flush()
    except DistMLException as e:
        err = e
    if rc:
        assert err is not None and (err.code, err.key, err.col) == o.error()
    else:
        assert err is None
    assert kat.bits_equal(s.values(), o.data)
    s.close()


def test_async_push_defers_error_to_flush(oracle):
    from distml_amd import DataDesc, IllegalStateException, encode_matrix_push
    fmt = DataDesc(1, 0, 0)
    s, _ = mk_store(fmt, 0, 3, 2, async_push=True)
    s.handlePush(fmt, encode_matrix_push([1], [[-1, 0]], 0, 0))  # returns before the check
    with pytest.raises(IllegalStateException):
        s.flush()
    assert s.values()[1, 0] == -1


# ----------------------------------------------------------------- fetch / checkpoint
def test_fetch_layouts_match_oracle(oracle):
    from distml_amd import DataDesc, KeyList, KeyRange
    rng = np.random.default_rng(3)
    for dt, kt, vt, cols, ada in [(1, 0, 1, 17, False), (1, 1, 0, 5, False), (1, 0, 3, 3, False),
                                  (1, 0, 1, 4, True), (0, 1, 1, 1, False), (0, 0, 0, 1, False), (0, 0, 3, 1, False)]:
        fmt = DataDesc(dt, kt, vt, False, True, ada)
        s, _ = mk_store(fmt, 40, 139, cols)
        o = oracle_store(oracle, fmt, 40, 139, cols)
        init = (rng.integers(0, 100, size=(100, cols)).astype(np.int32) if vt == 0
                else rng.standard_normal((100, cols)).astype(s.dtype))
        s.load_values(init)
        o.data[:] = init
        if ada:
            s.setAlpha(0.5, 0.01, 1.5)
            o.set_alpha(0.5, 0.01, 1.5)
        keys = [139, 40, 77, 78, 100]
        assert s.handleFetch(fmt, KeyList(keys + [5, 500])) == o.fetch(keys)
        assert s.handleFetch(fmt, KeyRange(130, 200)) == o.fetch(list(range(130, 140)))
        s.close()


def test_write_all_read_all_round_trip(oracle):
    from distml_amd import DataDesc
    rng = np.random.default_rng(5)
    for vt in (0, 1, 3):
        fmt = DataDesc(1, 0, vt)
        s, _ = mk_store(fmt, 0, 999, 13)
        o = oracle_store(oracle, fmt, 0, 999, 13)
        init = (rng.integers(-50, 50, size=(1000, 13)).astype(np.int32) if vt == 0
                else rng.standard_normal((1000, 13)).astype(s.dtype))
        s.load_values(init)
        o.data[:] = init
        blob = s.writeAll()
        assert blob == o.write_all()
        s.fill(0.0)
        assert not s.values().any()
        s.readAll(io.BytesIO(blob))
        assert kat.bits_equal(s.values(), init)
        buf = io.BytesIO()
        s.syncTo(buf, 10, 20)
        assert buf.getvalue() == blob[10 * 13 * s.values().itemsize: 21 * 13 * s.values().itemsize]
        s.close()


def test_large_fetch_checkpoint_bounce_and_pinned():
    """80 MiB shard: fetch / writeAll / readAll / syncTo / syncFrom through the
    pinned bounce ring (pageable buffers, 16 MiB chunks, last one partial) and
    straight DMA (pinned_empty buffers); expected bytes built with numpy."""
    from distml_amd import DataDesc, KeyRange, pinned_empty
    rows, cols = 20_003, 1024
    fmt = DataDesc(1, 0, 1)
    s, _ = mk_store(fmt, 1000, 1000 + rows - 1, cols)
    vals = np.random.default_rng(11).standard_normal((rows, cols)).astype(np.float32)
    s.load_values(vals)
    rec = np.empty((rows, 4 + 4 * cols), np.uint8)
    rec[:, :4] = np.arange(1000, 1000 + rows, dtype="<i4").view(np.uint8).reshape(rows, 4)
    rec[:, 4:] = vals.astype("<f4").view(np.uint8).reshape(rows, 4 * cols)
    want = rec.tobytes()
    assert s.handleFetch(fmt, KeyRange(0, 10**9)) == want
    pin = pinned_empty(len(want))
    assert s.handleFetchInto(fmt, KeyRange(1000, 1000 + rows - 1), pin) == len(want)
    assert pin.tobytes() == want
    be = vals.astype(">f4").tobytes()
    assert s.writeAll() == be
    s.fill(0.0)
    s.readAll(io.BytesIO(be))
    assert kat.bits_equal(s.values(), vals)
    # pinned source for readAll-equivalent syncFrom of every row
    s.fill(0.0)
    pin_be = pinned_empty(len(be))
    pin_be[:] = np.frombuffer(be, np.uint8)
    s.syncFrom(pin_be, 0, rows - 1)
    assert kat.bits_equal(s.values(), vals)
    buf = io.BytesIO()
    s.syncTo(buf, 7, 12_345)
    assert buf.getvalue() == vals[7:12_346].astype(">f4").tobytes()
    s.close()


def test_sync_and_read_all_error_semantics():
    """syncTo/syncFrom/readAll on bad rows or short streams: the reference moves the
    rows / elements before the failure, then throws (AIOOBE / EOFException)."""
    from distml_amd import DataDesc, DistMLException
    fmt = DataDesc(1, 0, 0)
    s, _ = mk_store(fmt, 0, 9, 3)
    vals = np.arange(30, dtype=np.int32).reshape(10, 3)
    s.load_values(vals)
    buf = io.BytesIO()
    with pytest.raises(DistMLException):
        s.syncTo(buf, 8, 11)  # rows 8, 9 written, then row 10 is out of the shard
    assert buf.getvalue() == vals[8:10].astype(">i4").tobytes()
    buf = io.BytesIO()
    with pytest.raises(DistMLException):
        s.syncTo(buf, -1, 3)  # throws before writing
    assert buf.getvalue() == b""
    s.syncTo(buf, 5, 4)  # empty range: no bytes, no error
    assert buf.getvalue() == b""
    # short stream: 4 whole elements + 2 stray bytes -> rows 2..3 get 4 elements, then EOF
    with pytest.raises(DistMLException):
        s.syncFrom(io.BytesIO(np.array([-1, -2, -3, -4], ">i4").tobytes() + b"\x00\x01"), 2, 3)
    got = s.values()
    assert got[2].tolist() == [-1, -2, -3] and got[3].tolist() == [-4, 10, 11]
    assert np.array_equal(got[4:], vals[4:]) and np.array_equal(got[:2], vals[:2])
    prev = s.values().ravel()
    with pytest.raises(DistMLException):
        s.readAll(io.BytesIO(np.full(5, 7, ">i4").tobytes()))
    got = s.values().ravel()
    assert (got[:5] == 7).all() and np.array_equal(got[5:], prev[5:])
    s.close()


# ------------------------------------------------------- full-size configs (BASELINE.json)
def synth_device_buckets(L, desc, first, shard_rows, nrec, cols, seeds, perms):
    from distml_amd.datadesc import DataDesc
    K = 4 if desc.key_type == 0 else 8
    V = 8 if desc.value_type == 3 else 4
    n = nrec * (K + V * cols)
    bufs = []
    st = torch.cuda.current_stream().cuda_stream
    for sd, (pa, pc) in zip(seeds, perms):
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(desc), first, shard_rows, nrec, cols, sd, pa, pc,
                                        C.c_void_p(st)) == 0
        bufs.append(t)
    torch.cuda.synchronize()
    return bufs


def test_synth_kernel_matches_oracle_generator(oracle):
    from distml_amd import _lib
    from distml_amd.datadesc import DataDesc
    L = _lib.load()
    for kt, vt, cols in [(0, 1, 1024), (1, 3, 7), (0, 0, 1000)]:
        d = DataDesc(1, kt, vt).to_c()
        b = synth_device_buckets(L, d, 3, 509, 509, cols, [11], [(7, 5)])[0]
        want = oracle.synth_dense_bucket(kt, vt, 3, 509, 509, cols, 11, 7, 5)
        assert b.cpu().numpy().tobytes() == want.tobytes()
    d = DataDesc(0, 1, 1).to_c()
    t = torch.empty(1000 * 12, dtype=torch.uint8, device="cuda")
    assert L.dml_synth_sparse_bucket(t.data_ptr(), C.byref(d), 0, 10**9, 1000, 9, 123457, 99, C.c_void_p(0)) == 0
    torch.cuda.synchronize()
    assert t.cpu().numpy().tobytes() == oracle.synth_sparse_bucket(1, 1, 0, 10**9, 1000, 9, 123457, 99).tobytes()


def test_gather_floor_diag_is_the_plain_row_sum():
    """dml_diag_gather_floor (config 5's measured ceiling, bench.gather_floor) does the
    reduce's work: every record added to its row, each touched row read and written
    once — int32 wrapping sums equal numpy's on 6 pushes of 200 distinct rows of 500."""
    import bench
    from distml_amd import DataDesc, _lib
    L = _lib.load()
    rows, cols, nrec = 500, 100, 200
    fmt = DataDesc(1, 0, 0)
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    s.synth_fill(11)
    want = s.values().astype(np.int64)
    bufs = synth_device_buckets(L, fmt.to_c(), 0, rows, nrec, cols, [70 + b for b in range(6)],
                                [(a, 13 * b) for b, a in enumerate((7, 9, 11, 13, 17, 19))])
    for b in bufs:
        rec = b.cpu().numpy().view("<i4").reshape(nrec, 1 + cols)
        np.add.at(want, rec[:, 0], rec[:, 1:].astype(np.int64))
    ms = bench.gather_floor(L, torch, s, bufs, rows, cols, 0, 4 + 4 * cols, 0, reps=1)
    assert ms > 0
    assert np.array_equal(s.values(), want.astype(np.uint32).view(np.int32).reshape(rows, cols))
    s.close()


@pytest.mark.parametrize("ada", [False, True])
def test_dense_floor_diag_is_the_plain_stream(oracle, ada):
    """dml_diag_dense_floor (the config-4 legs' live ceiling, bench.dense_floor) moves the
    reduce's bytes with the reduce's arithmetic: on a store without a second buffer it
    writes in place exactly the oracle's sums (AdaGrad: and delta), for 5 ascending
    full-range pushes of 300 x 200 f32."""
    import bench
    from distml_amd import DataDesc, _lib
    L = _lib.load()
    rows, cols, W = 300, 200, 5
    fmt = DataDesc(1, 0, 1, False, True, ada)
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    s.synth_fill(13)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    o.synth_fill(13)
    if ada:
        s.setAlpha(0.025, 0.0001, 1.0)
        o.set_alpha(0.025, 0.0001, 1.0)
    bufs = synth_device_buckets(L, fmt.to_c(), 0, rows, rows, cols, [90 + b for b in range(W)], [(1, 0)] * W)
    for b in bufs:
        assert o.push(b.cpu().numpy().tobytes()) == 0
    ms, oop = bench.dense_floor(L, s, [b.data_ptr() for b in bufs], [b.numel() for b in bufs], 0, reps=1)
    assert ms > 0 and not oop
    assert kat.bits_equal(s.values(), o.data)
    if ada:
        assert kat.bits_equal(s.adagrad_state()[1], o.delta)
    s.close()


def config2_perm(b, rows=16384):
    # ascending row order (Java HashMap<Integer> order) for even pushes, a seeded permutation for odd
    return (1, 0) if b % 2 == 0 else ((2 * b + 1) * 2654435761 % rows | 1, (b * 7919) % rows)


def test_config2_dense_fp32_full_size_bit_exact(oracle):
    """Config 2: 32 pushes x 64 MiB ([int32 key][1024 x f32] x 16384) -> one 64 MiB shard."""
    from distml_amd import DataDesc
    rows, cols, W = 16384, 1024, 32
    fmt = DataDesc(1, 0, 1)
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    s.synth_fill(7)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    o.synth_fill(7)
    assert kat.bits_equal(s.values(), o.data)
    from distml_amd import _lib
    L = _lib.load()
    perms = [config2_perm(b) for b in range(W)]
    bufs = synth_device_buckets(L, fmt.to_c(), 0, rows, rows, cols, [1000 + b for b in range(W)], perms)
    s.pushDevice([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
    s.flush()
    host = [oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 1000 + b, *perms[b]) for b in range(W)]
    assert o.push_many(host, threads=8) == 0
    assert kat.bits_equal(s.values(), o.data)


@pytest.mark.parametrize("order", ["position", "shuffled"])
def test_config2_headline_steady_state_bit_exact(oracle, order):
    """Exactly what bench.py's N=1 headline times, at full size: a 16 384 x 1 024 fp32
    shard, two 32-push sets (16 ascending + 16 permuted, the bench's perm_for, value
    seeds 1000+b and 5000+b) pushed alternately, six pushDevice calls without a flush.
    Chunks 3..5 find their workspace's kept slot table (chunk j-3's), so their 16
    permuted pushes reuse kept columns instead of the key index — asserted through
    dml_store_stats — and the shard is bytes-equal to the oracle fed the same 192
    pushes in order (FloatMatrixStore.java:200-222). `shuffled`: every call applies
    its 32 pushes in a new seeded order (the selector's arrival order,
    PSAgent.java:166-186); the content-keyed reuse still engages."""
    from distml_amd import DataDesc, _lib
    rows, cols, W, calls = 16384, 1024, 32, 6
    fmt = DataDesc(1, 0, 1)
    L = _lib.load()
    s, _ = mk_store(fmt, 0, rows - 1, cols, async_push=True)
    s.synth_fill(7)
    perms = [config2_perm(b) for b in range(W)]
    sets = [synth_device_buckets(L, fmt.to_c(), 0, rows, rows, cols, [seed0 + b for b in range(W)], perms)
            for seed0 in (1000, 5000)]
    rng = np.random.default_rng(2024)
    orders = [rng.permutation(W) if order == "shuffled" else np.arange(W) for _ in range(calls)]
    s.stats(reset=True)
    for c in range(calls):
        bs = [sets[c & 1][j] for j in orders[c]]
        s.pushDevice([b.data_ptr() for b in bs], [b.numel() for b in bs])
    s.flush()
    st = s.stats()
    assert st["chunks"] == calls and st["spec_chunks"] == calls and st["spec_reruns"] == 0, st
    assert st["identity_pushes"] == 16 * calls, st
    assert st["reused_pushes"] == 16 * (calls - 3) and st["indexed_pushes"] == 16 * 3, st
    got = s.values()
    s.close()
    del sets
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    o.synth_fill(7)
    host = [[oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, seed0 + b, *perms[b]) for b in range(W)]
            for seed0 in (1000, 5000)]
    assert o.push_many([host[c & 1][j] for c in range(calls) for j in orders[c]], threads=16) == 0
    assert kat.bits_equal(got, o.data)


def test_config5_model_leg_bit_exact(oracle):
    """bench.py's config-5 leg at N = 1, full size: the 1 000 000 x 1 000 int32
    IntMatrixStore (4 GB) and its 32 pushes of 65 536 distinct rows (the leg's seeds
    and permutations), then the 32 negated pushes (the leg's second step); bit-exact
    against the oracle with the negativity check after each add
    (IntMatrixStore.java:164-178), no error."""
    from distml_amd import DataDesc, _lib
    import math
    rows, cols, W, nrec = 1_000_000, 1000, 32, 65536
    fmt = DataDesc(1, 0, 0)
    L = _lib.load()

    def coprime(a, n):
        while math.gcd(a, n) != 1:
            a += 1
        return a

    perms = [(coprime(((4000 + b) * 2654435761) % rows | 1, rows), (b * 331) % rows) for b in range(W)]
    s, _ = mk_store(fmt, 0, rows - 1, cols, async_push=True)
    s.synth_fill(11)
    pos = synth_device_buckets(L, fmt.to_c(), 0, rows, nrec, cols, [4000 + b for b in range(W)], perms)
    neg = []
    for t in pos:
        n = t.clone().view(torch.int32).view(nrec, 1 + cols)
        n[:, 1:] = -n[:, 1:]
        neg.append(n.view(torch.uint8).view(-1))
    torch.cuda.synchronize()
    s.pushDevice([b.data_ptr() for b in pos], [b.numel() for b in pos])
    s.pushDevice([b.data_ptr() for b in neg[:16]], [b.numel() for b in neg[:16]])
    s.flush()
    assert s.error_state()[0] == 0
    got = s.values()
    s.close()
    del pos, neg
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    o.synth_fill(11)
    host = [oracle.synth_dense_bucket(0, 0, 0, rows, nrec, cols, 4000 + b, *perms[b]) for b in range(W)]
    negh = []
    for h in host[:16]:
        t = h.view(np.int32).reshape(nrec, 1 + cols).copy()
        t[:, 1:] = -t[:, 1:]
        negh.append(t.view(np.uint8).reshape(-1))
    assert o.push_many(host + negh, threads=16) == 0
    assert kat.bits_equal(got, o.data)


def test_config3_sparse_fp32_full_size_bit_exact(oracle):
    """Config 3: 1e9-dim fp32 array shard, 32 pushes x 1e6 unique keys (12-byte records)."""
    from distml_amd import DataDesc, _lib
    dim, nnz, W = 10**9, 10**6, 32
    fmt = DataDesc(0, 1, 1)
    s, _ = mk_store(fmt, 0, dim - 1)
    L = _lib.load()
    d = fmt.to_c()
    bufs, host = [], []
    for b in range(W):
        pa, pc = (2 * b + 3) * 999_999_937 % dim, (b * 12_345_701) % dim
        while pa % 2 == 0 or pa % 5 == 0:
            pa += 1
        t = torch.empty(nnz * 12, dtype=torch.uint8, device="cuda")
        assert L.dml_synth_sparse_bucket(t.data_ptr(), C.byref(d), 0, dim, nnz, 2000 + b, pa, pc, C.c_void_p(0)) == 0
        bufs.append(t)
        host.append((pa, pc))
    torch.cuda.synchronize()
    s.pushDevice([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
    s.flush()
    o = oracle_store(oracle, fmt, 0, dim - 1)
    for b, (pa, pc) in enumerate(host):
        assert o.push(oracle.synth_sparse_bucket(1, 1, 0, dim, nnz, 2000 + b, pa, pc).tobytes()) == 0
    assert kat.bits_equal(s.values(), o.data)


def test_config5_lda_int32_shard_bit_exact(oracle):
    """Config 5, one GPU's shard of linearSplit(8): 125 000 x 1 000 int32 counts,
    32 pushes x 8 192 distinct rows, deltas in {-2..2}, init U{64..114} (no negatives)."""
    from distml_amd import DataDesc, _lib
    rows, cols, W, nrec = 125_000, 1000, 32, 8192
    fmt = DataDesc(1, 0, 0)
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    s.synth_fill(11)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    o.synth_fill(11)
    L = _lib.load()
    perms = [((4000 + b) * 2654435761 % rows | 1, b * 331 % rows) for b in range(W)]
    perms = [(pa if np.gcd(pa, rows) == 1 else pa + 2, pc) for pa, pc in perms]
    assert all(np.gcd(pa, rows) == 1 for pa, _ in perms)
    bufs = synth_device_buckets(L, fmt.to_c(), 0, rows, nrec, cols, [4000 + b for b in range(W)], perms)
    s.pushDevice([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
    s.flush()
    host = [oracle.synth_dense_bucket(0, 0, 0, rows, nrec, cols, 4000 + b, *perms[b]) for b in range(W)]
    assert o.push_many(host, threads=8) == 0
    assert kat.bits_equal(s.values(), o.data)


def test_config4_adagrad_rows_bit_exact(oracle):
    """Config 4 rows (AdaGrad Word2Vec store, 200 cols), reduced to 20 000 rows x 8 pushes;
    large gradients so delta crosses 1.0 and alpha/minAlpha paths run."""
    from distml_amd import DataDesc, encode_matrix_push
    rng = np.random.default_rng(44)
    rows, cols, W = 20_000, 200, 8
    fmt = DataDesc(1, 0, 1, False, True, True)
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    s.setAlpha(0.025, 0.0001, 1.5)
    o.set_alpha(0.025, 0.0001, 1.5)
    pushes = []
    for b in range(W):
        r = rng.permutation(rows)[: rows // 2]
        v = (rng.standard_normal((len(r), cols)) * 0.6).astype(np.float32)
        pushes.append(encode_matrix_push(r, v, 0, 1))
    for p in pushes:
        assert o.push(p) == 0
    s.handlePushBatch(fmt, pushes)
    assert kat.bits_equal(s.values(), o.data)
    a, d = s.adagrad_state()
    assert kat.bits_equal(a, o.alpha)
    assert kat.bits_equal(d, o.delta)
    assert s.maxDelta() == o.max_delta()


def test_shard_group_rccl_world1(oracle):
    """The multi-GPU full-range path (HIP pre-reduce -> RCCL reduce-scatter -> HIP owner
    apply) at world_size 1 on one MI355X; fp32 within the bound of tests/test_group_gloo.py."""
    import os
    import socket
    import torch.distributed as dist
    from distml_amd import DataDesc
    from distml_amd.group import ShardGroup
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rows, cols, W = 1000, 256, 6
        fmt = DataDesc(1, 0, 1)
        g = ShardGroup(fmt, rows, cols, 0, 1, device=0)
        g.store.synth_fill(3)
        pas = [1, 3, 7, 9, 11, 13]  # coprime with 1000: each push lists every row once
        host = [oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 50 + b, pas[b], b) for b in range(W)]
        dev = [torch.from_numpy(h).cuda() for h in host]
        torch.cuda.synchronize()
        g.push_full_range([d.data_ptr() for d in dev], [d.numel() for d in dev],
                          torch.cuda.current_stream().cuda_stream)
        g.flush()
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.synth_fill(3)
        init = o.data.copy()
        for h in host:
            assert o.push(h.tobytes()) == 0
        got = g.store.values().astype(np.float64)
        terms = np.abs(init.astype(np.float64))
        for h in host:
            rec = h.reshape(rows, 4 + 4 * cols)
            terms[rec[:, :4].copy().view("<i4").ravel()] += np.abs(rec[:, 4:].copy().view("<f4"))
        diff = np.abs(got - o.data.astype(np.float64))
        assert np.all(diff <= 2 * W * 2.0 ** -24 * terms)
    finally:
        dist.destroy_process_group()


def test_shard_group_oneshot_world1_consecutive(oracle):
    """The one-shot full-range path (> 64 pushes per call) at world 1, where the owner
    apply reads the partial itself: two calls back to back without a flush, so the second
    call's pre-reduce rewrites the partial right after the first call's apply was
    enqueued on the store's stream (it must wait for it). fp32 within the bound of
    tests/test_group_gloo.py."""
    import socket
    import torch.distributed as dist
    from distml_amd import DataDesc
    from distml_amd.group import ShardGroup
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rows, cols, W, calls = 1024, 256, 66, 2
        fmt = DataDesc(1, 0, 1)
        g = ShardGroup(fmt, rows, cols, 0, 1, device=0)
        g.store.synth_fill(5)
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.synth_fill(5)
        terms = np.abs(o.data.astype(np.float64))
        dev = []
        for c in range(calls):
            host = [oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 700 + 100 * c + b, 2 * b + 1, 3 * b)
                    for b in range(W)]
            for h in host:
                assert o.push(h.tobytes()) == 0
                rec = h.reshape(rows, 4 + 4 * cols)
                terms[rec[:, :4].copy().view("<i4").ravel()] += np.abs(rec[:, 4:].copy().view("<f4"))
            dev.append([torch.from_numpy(h).cuda() for h in host])  # alive until the flush
        torch.cuda.synchronize()
        for d in dev:
            g.push_full_range([t.data_ptr() for t in d], [t.numel() for t in d],
                              torch.cuda.current_stream().cuda_stream)
        g.flush()
        diff = np.abs(g.store.values().astype(np.float64) - o.data.astype(np.float64))
        assert np.all(diff <= 2 * calls * W * 2.0 ** -24 * terms)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("binding", ["torch", "native"])
@pytest.mark.parametrize("vt", [1, 0])
def test_sharded_speculation_world1(oracle, binding, vt):
    """The sharded path's speculative pre-reduce (dml_prectx) at world 1
    over RCCL: six calls of four full-range pushes (ascending, two fixed permutations,
    ascending), no flush between them. Calls 3 and 5 reuse the permutations their
    workspace kept three calls before; call 4's first push has two records swapped
    where k_ident_check's sample cannot see them, so its pieces fail verification and
    the call re-runs exactly with the key index before its reduce-scatter. int32 is
    exact; fp32 within the summation-order bound of tests/test_group_gloo.py."""
    import socket
    import torch.distributed as dist
    from distml_amd import DataDesc, encode_matrix_push
    from distml_amd.group import NativeShardGroup, ShardGroup
    rows, cols, calls, W = 1000, 256, 6, 4
    fmt = DataDesc(1, 0, vt)
    rng = np.random.default_rng(33 + vt)
    pa, pb = rng.permutation(rows), rng.permutation(rows)
    free = sorted(set(range(rows)) - _sampled_rows(oracle, 0, rows))
    host = []
    for c in range(calls):
        for b, keys in enumerate((np.arange(rows), pa, pb, np.arange(rows))):
            keys = keys.copy()
            if c == 4 and b == 0:
                i, j = free[len(free) // 2], free[len(free) // 2 + 1]
                keys[i], keys[j] = keys[j], keys[i]
            v = (rng.integers(-3, 4, size=(rows, cols)).astype(np.int32) if vt == 0
                 else (rng.standard_normal((rows, cols)) * 1e-3).astype(np.float32))
            host.append(encode_matrix_push(keys, v, 0, vt))
    dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in host]
    torch.cuda.synchronize()
    port = None
    if binding == "torch":
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        g = ShardGroup(fmt, rows, cols, 0, 1, device=0)
    else:
        g = NativeShardGroup(fmt, rows, cols, 0, 1, NativeShardGroup.unique_id(), device=0)
    try:
        g.store.synth_fill(3)
        for c in range(calls):
            sl = dev[c * W:(c + 1) * W]
            if binding == "torch":
                g.push_full_range([d.data_ptr() for d in sl], [d.numel() for d in sl],
                                  torch.cuda.current_stream().cuda_stream)
            else:
                g.push_full_range([d.data_ptr() for d in sl], [d.numel() for d in sl])
        g.flush()
        st = g.prereduce_stats()
        assert st["chunks"] == calls and st["spec_chunks"] == calls and st["spec_reruns"] == 1, st
        assert st["reused_pushes"] == 4 and st["identity_pushes"] == 2 * (calls - 1), st
        got = g.store.values()
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.synth_fill(3)
        init = o.data.copy()
        for h in host:
            assert o.push(h) == 0
        if vt == 0:
            assert np.array_equal(got, o.data)
            return
        terms = np.abs(init.astype(np.float64))
        for h in host:
            rec = np.frombuffer(h, np.uint8).reshape(rows, 4 + 4 * cols)
            terms[rec[:, :4].copy().view("<i4").ravel()] += np.abs(rec[:, 4:].copy().view("<f4"))
        diff = np.abs(got.astype(np.float64) - o.data.astype(np.float64))
        assert np.all(diff <= 2 * len(host) * 2.0 ** -24 * terms)
    finally:
        g.close()
        if port is not None:
            dist.destroy_process_group()


@pytest.mark.parametrize("binding", ["torch", "native"])
def test_adagrad_moments_world1(oracle, binding):
    """The two-moment AdaGrad path at world 1 over RCCL: three calls
    of four pushes (full-range ascending and permuted, and a key subset), no flush
    between; data, alpha, delta and maxDelta within 1e-6 of the sequential oracle
    (moments_within); maxDelta's (row, col) holds that value."""
    import socket
    import torch.distributed as dist
    from distml_amd import DataDesc, encode_matrix_push
    from distml_amd.group import NativeShardGroup, ShardGroup
    rows, cols, calls, W = 1000, 200, 3, 4
    ada = (0.025, 0.0001, 1.5)
    fmt = DataDesc(1, 0, 1, False, True, True)
    rng = np.random.default_rng(44)
    host = []
    for c in range(calls):
        for b in range(W):
            keys = (np.arange(rows) if b == 0 else rng.permutation(rows)[: rows if b < 3 else rows // 2])
            host.append(encode_matrix_push(keys, (rng.standard_normal((len(keys), cols)) * 0.6).astype(np.float32),
                                           0, 1))
    dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in host]
    torch.cuda.synchronize()
    port = None
    if binding == "torch":
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        g = ShardGroup(fmt, rows, cols, 0, 1, device=0, exchange_only=True)
    else:
        g = NativeShardGroup(fmt, rows, cols, 0, 1, NativeShardGroup.unique_id(), device=0)
    try:
        g.store.setAlpha(*ada)
        rng2 = np.random.default_rng(3)
        init = (rng2.standard_normal((rows, cols)) * 0.1).astype(np.float32)
        g.store.load_values(init)
        for c in range(calls):
            sl = dev[c * W:(c + 1) * W]
            g.push_moments([d.data_ptr() for d in sl], [d.numel() for d in sl])
        g.flush()
        a, d = g.store.adagrad_state()
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.set_alpha(*ada)
        o.data[:] = init
        for h in host:
            assert o.push(h) == 0
        kat.moments_within(g.store.values(), a.astype(np.float64), d.astype(np.float64), o, init, host, cols, binding)
        mv, mr, mc = g.store.maxDelta()
        ov = o.max_delta()[0]
        assert abs(mv - ov) <= 1e-6 * ov and d[mr, mc] == np.float32(mv), (mv, mr, mc, o.max_delta())
    finally:
        g.close()
        if port is not None:
            dist.destroy_process_group()


def test_prereduce_pieces_row_map(oracle):
    """dml_prereduce_{begin,piece,end}: slices laid out [rank][row] for a 3-way
    linearSplit of 1000 rows (step 334, last shard 332 rows + 2 padding rows),
    bit-exact vs an oracle store that starts at zero (0 + g0 + g1 + ...)."""
    import ctypes as C
    from distml_amd import DataDesc
    from distml_amd.group import HipOps
    rows, cols, W, world, P = 1000, 300, 5, 3, 2
    S = (rows - 1 + world) // world
    blk = S // P
    fmt = DataDesc(1, 0, 1)
    pas = [1, 3, 7, 9, 11]
    host = [oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 70 + b, pas[b], b) for b in range(W)]
    dev = [torch.from_numpy(h).cuda() for h in host]
    torch.cuda.synchronize()
    ops = HipOps()
    st = torch.cuda.current_stream().cuda_stream
    out = torch.full((P, world * blk, cols), float("nan"), dtype=torch.float32, device="cuda")
    h = ops.begin(fmt, 0, rows, cols, [d.data_ptr() for d in dev], [d.numel() for d in dev], st)
    for j in range(P):
        ops.piece(h, blk, S, j * blk, world * blk, out[j].data_ptr(), st)
    ops.end(h)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    for hb in host:
        assert o.push(hb.tobytes()) == 0
    got = out.cpu().numpy()
    for j in range(P):
        for t in range(world * blk):
            r = (t // blk) * S + j * blk + t % blk
            want = o.data[r] if r < rows else np.zeros(cols, np.float32)
            assert got[j, t].tobytes() == want.tobytes(), (j, t, r)


@pytest.mark.parametrize("vt", [1, 0])
def test_native_group_rccl_world1(oracle, vt):
    """dml_group_* (the C-ABI's own RCCL communicator, no torch.distributed) at world 1:
    two asynchronous full-range calls + flush. fp32 within the summation-order bound of
    tests/test_group_gloo.py, int32 exact."""
    from distml_amd import DataDesc
    from distml_amd.group import NativeShardGroup
    rows, cols, W = 1000, 256, 5
    fmt = DataDesc(1, 0, vt)
    g = NativeShardGroup(fmt, rows, cols, 0, 1, NativeShardGroup.unique_id(), device=0, pieces=4)
    try:
        g.store.synth_fill(3)
        pas = [1, 3, 7, 9, 11]  # coprime with 1000: each push lists every row once
        host = [oracle.synth_dense_bucket(0, vt, 0, rows, rows, cols, 70 + b, pas[b], 3 * b) for b in range(W)]
        dev = [torch.from_numpy(h).cuda() for h in host]
        torch.cuda.synchronize()
        ptrs, lens = [d.data_ptr() for d in dev], [d.numel() for d in dev]
        g.push_full_range(ptrs[:3], lens[:3])
        g.push_full_range(ptrs[3:], lens[3:])
        g.flush()
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.synth_fill(3)
        init = o.data.copy()
        for h in host:
            assert o.push(h.tobytes()) == 0
        got = g.store.values()
        if vt == 0:
            assert np.array_equal(got, o.data)
            return
        terms = np.abs(init.astype(np.float64))
        for h in host:
            rec = h.reshape(rows, 4 + 4 * cols)
            terms[rec[:, :4].copy().view("<i4").ravel()] += np.abs(rec[:, 4:].copy().view("<f4"))
        diff = np.abs(got.astype(np.float64) - o.data.astype(np.float64))
        assert np.all(diff <= 2 * W * 2.0 ** -24 * terms)
    finally:
        g.close()


def test_native_group_int32_negative_final_counter():
    """IntMatrixStore's negativity check on the sharded full-range path:
    the owner apply checks the final counters (IntMatrixStore.java:174-176); the
    first negative element (row-major) of the failing call becomes the store's
    IllegalStateException at flush(), with its key and column, and the store
    refuses later calls."""
    from distml_amd import DataDesc, IllegalStateException, encode_matrix_push
    from distml_amd.group import NativeShardGroup
    rows, cols = 64, 8
    fmt = DataDesc(1, 0, 0)
    g = NativeShardGroup(fmt, rows, cols, 0, 1, NativeShardGroup.unique_id(), device=0, pieces=4)
    try:
        g.store.fill(3)
        vals = np.zeros((rows, cols), np.int32)
        vals[40, 5] = -4   # final 3 - 4 = -1: the first negative in row-major order
        vals[41, 0] = -9
        vals[10, 2] = -3   # final 0: fine
        push = np.frombuffer(encode_matrix_push(np.arange(rows), vals, 0, 0), np.uint8).copy()
        dev = torch.from_numpy(push).cuda()
        torch.cuda.synchronize()
        g.push_full_range([dev.data_ptr()], [dev.numel()])
        with pytest.raises(IllegalStateException) as ei:
            g.flush()
        assert (ei.value.key, ei.value.col) == (40, 5)
        got = g.store.values()
        want = np.full((rows, cols), 3, np.int32) + vals
        assert np.array_equal(got, want)
        with pytest.raises(Exception):
            g.push_full_range([dev.data_ptr()], [dev.numel()])
            g.flush()
    finally:
        g.close()


def test_shard_group_orders_after_producer_stream(oracle):
    """ShardGroup.push_full_range right after the producers ran on the caller's
    stream, with no host synchronize: the key index (side stream) and the pieces
    must both order after them. Two back-to-back calls, bit-exact at
    world 1 for int32 (the reduce-scatter is a copy, the sum exact)."""
    import socket
    import torch.distributed as dist
    from distml_amd import DataDesc, _lib
    from distml_amd.group import ShardGroup
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rows, cols, W = 4096, 1000, 6
        fmt = DataDesc(1, 0, 0)
        L = _lib.load()
        g = ShardGroup(fmt, rows, cols, 0, 1, device=0)
        g.store.synth_fill(5)
        # a large first kernel on the caller's stream delays the producers behind it
        big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        bufs = [torch.empty(rows * (4 + 4 * cols), dtype=torch.uint8, device="cuda") for _ in range(2 * W)]
        torch.cuda.synchronize()
        st = torch.cuda.current_stream().cuda_stream
        pas = [1, 3, 5, 7, 9, 11, 13, 15, 17, 19, 21, 23]
        for call in range(2):
            big.fill_(call)
            for b in range(W):
                j = call * W + b
                assert L.dml_synth_dense_bucket(bufs[j].data_ptr(), C.byref(fmt.to_c()), 0, rows, rows, cols, 90 + j,
                                                pas[j], 7 * j, C.c_void_p(st)) == 0
            g.push_full_range([bufs[call * W + b].data_ptr() for b in range(W)], [bufs[0].numel()] * W, st)
        g.flush()
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.synth_fill(5)
        for j in range(2 * W):
            assert o.push(oracle.synth_dense_bucket(0, 0, 0, rows, rows, cols, 90 + j, pas[j], 7 * j).tobytes()) == 0
        assert np.array_equal(g.store.values(), o.data)
        g.close()
    finally:
        dist.destroy_process_group()


def _np_split(recs_list, K, total_rows, world):
    """Reference split for dml_shard_split: stable per-owner partition, dest-major."""
    from distml_amd.datadesc import KeyRange
    step = KeyRange(0, total_rows - 1).linearSplit(world)[0].size()
    kdt = "<i4" if K == 4 else "<i8"
    owners = []
    for r in recs_list:
        k = r[:, :K].copy().view(kdt).ravel().astype(np.int64)
        o = np.where((k >= 0) & (k < total_rows), k // max(step, 1), world)
        owners.append(np.minimum(o, world))
    out = b"".join(r[o == d].tobytes() for d in range(world) for r, o in zip(recs_list, owners))
    counts = [[int((o == d).sum()) for d in range(world)] for o in owners]
    return out, counts


@pytest.mark.parametrize("case", [
    # (data_type, key_type, value_type, cols, total_rows, world, n, nrec)
    (1, 0, 1, 200, 5000, 8, 3, 4000),   # config-4 record shape, 8 owners
    (1, 0, 0, 1000, 1000, 3, 2, 700),   # int32 counts, short last shard
    (1, 1, 3, 10, 784, 2, 4, 300),      # MLR DoubleMatrix (LONG keys)
    (0, 1, 1, 1, 10**9, 5, 2, 20000),   # sparse float array, long keys
    (1, 0, 1, 64, 100, 64, 1, 257),     # 64 owners, ragged last block
    (1, 0, 1, 200, 5003, 8, 3, 5003, "asc"),  # full-range ascending pushes: owner runs (vector copies)
    (0, 1, 1, 1, 40000, 3, 2, 40000, "asc"),  # 12-B records in owner runs
    (1, 0, 1, 200, 4000, 1, 2, 4000, "asc"),  # world 1: the split is one copy
])
def test_shard_split_kernel(case):
    """dml_shard_split against a numpy stable partition: counts and bytes equal; keys
    outside [0, total_rows) dropped. `asc`: every push lists the keys in ascending
    order (each owner's records form one run)."""
    from distml_amd import DataDesc
    from distml_amd.group import HipOps
    dtp, kt, vt, cols, total, world, n, nrec = case[:8]
    asc = len(case) > 8
    fmt = DataDesc(dtp, kt, vt)
    K, V = (4 if kt == 0 else 8), (4 if vt in (0, 1) else 8)
    stride = K + (V * cols if dtp == 1 else V)
    rng = np.random.default_rng(sum(case[:8]))
    recs = []
    for b in range(n):
        r = rng.integers(0, 256, size=(nrec + b, stride), dtype=np.uint8)
        keys = rng.integers(-3, total + 3, size=nrec + b).astype("<i4" if K == 4 else "<i8")
        if asc:
            keys = (np.arange(nrec + b) - b).astype(keys.dtype)  # push b: one key below 0 (dropped)
        r[:, :K] = keys.view(np.uint8).reshape(-1, K)
        recs.append(r)
    dev = [torch.from_numpy(r.reshape(-1)).cuda() for r in recs]
    cap = sum(d.numel() for d in dev)
    out = torch.zeros(cap + 16, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    counts = HipOps().split(fmt, cols, total, world, [d.data_ptr() for d in dev], [d.numel() for d in dev],
                            out.data_ptr(), cap, torch.cuda.current_stream().cuda_stream)
    exp, exp_counts = _np_split(recs, K, total, world)
    assert counts == exp_counts
    assert out[:len(exp)].cpu().numpy().tobytes() == exp


def test_shard_split_rejects_partial_records():
    from distml_amd import DataDesc, NativeError
    from distml_amd.group import HipOps
    d = torch.zeros(805, dtype=torch.uint8, device="cuda")
    with pytest.raises(NativeError):
        HipOps().split(DataDesc(1, 0, 1), 200, 100, 2, [d.data_ptr()], [805], d.data_ptr(), 805, 0)


@pytest.mark.parametrize("calls", [1, 4, "mixed"])
def test_exchange_rccl_world1_adagrad(oracle, calls):
    """ShardGroup.push_exchange at world 1 over RCCL: dml_shard_split, the all-to-all
    and the ordered AdaGrad apply; bit-exact (data, alpha, delta, maxDelta). With 4
    calls of different sizes back to back (no flush between), the pooled send /
    receive buffers are reused across calls of other sizes. `mixed`: pushes 0 and 3
    hold only keys inside the matrix, so calls 1 and 3 hand their pushes to the
    store as they are and calls 2 and 4 split, in one ordered sequence."""
    import socket
    import torch.distributed as dist
    from distml_amd import DataDesc, encode_matrix_push
    from distml_amd.group import ShardGroup
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rows, cols, W = 3000, 200, 5
        fmt = DataDesc(1, 0, 1, False, True, True)
        g = ShardGroup(fmt, rows, cols, 0, 1, device=0, exchange_only=calls != 1)
        g.store.setAlpha(0.025, 0.0001, 1.5)
        rng = np.random.default_rng(77)
        host = []
        for b in range(W):
            keys = rng.permutation(rows + 50)[: rows // 2] - 25  # some keys outside the matrix: dropped
            if calls == "mixed" and b in (0, 3):
                keys = rng.permutation(rows)[: rows // 2]
            vals = (rng.standard_normal((len(keys), cols)) * 0.6).astype(np.float32)
            host.append(encode_matrix_push(keys, vals, 0, 1))
        dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in host]
        torch.cuda.synchronize()
        cuts = [0, W] if calls == 1 else [0, 1, 3, 4, W]
        if calls == "mixed":
            torch.cuda.synchronize()
        for c0, c1 in zip(cuts, cuts[1:]):
            g.push_exchange([d.data_ptr() for d in dev[c0:c1]], [d.numel() for d in dev[c0:c1]])
        g.flush()
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.set_alpha(0.025, 0.0001, 1.5)
        for h in host:  # the client's split: out-of-matrix keys never reach the server
            r = np.frombuffer(h, np.uint8).reshape(-1, 4 + 4 * cols)
            k = r[:, :4].copy().view("<i4").ravel()
            assert o.push(r[(k >= 0) & (k < rows)].tobytes()) == 0
        assert kat.bits_equal(g.store.values(), o.data)
        a, d = g.store.adagrad_state()
        assert kat.bits_equal(a, o.alpha) and kat.bits_equal(d, o.delta)
        assert g.store.maxDelta() == o.max_delta()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("binding", ["torch", "native"])
@pytest.mark.parametrize("case", ["repeat_adagrad", "negative_int32"])
def test_exchange_buffer_reuse_after_retire(oracle, binding, case):
    """The exchange path's receive buffers are reused two calls later (native: two
    alternating sets; torch: a pool). A store chunk may read its pushes again when it
    retires on the host — the exact replay of a row a push repeats, the int32
    rollback past a negative counter — so a set is rewritten only after the store
    retired the call that read it (dml_store_retire). Six calls of two
    pushes at world 1 over RCCL, each push with keys outside the matrix (the split
    path, not the world-1 hand-through); call 1 repeats a row (AdaGrad: replayed) or
    drives a counter negative (IllegalStateException at a later call or the flush).
    Bit-exact against the oracle fed the client-split pushes in order, stopping where
    it throws (IntMatrixStore.java:174-176)."""
    import socket
    import torch.distributed as dist
    from distml_amd import DataDesc, DistMLException, encode_matrix_push
    from distml_amd.group import NativeShardGroup, ShardGroup
    rows, cols, calls, per = 1200, 64, 6, 2
    ada = case == "repeat_adagrad"
    fmt = DataDesc(1, 0, 1, False, True, True) if ada else DataDesc(1, 0, 0)
    rng = np.random.default_rng(17 if ada else 19)
    host = []
    for i in range(calls * per):
        keys = rng.permutation(rows + 40)[: rows // 2] - 20  # a few keys outside the matrix: dropped
        if ada:
            vals = (rng.standard_normal((len(keys), cols)) * 0.6).astype(np.float32)
            if i == per:  # call 1, push 0 lists one row twice
                inside = np.nonzero((keys >= 0) & (keys < rows))[0]
                keys[inside[7]] = keys[inside[300]]
        else:
            vals = rng.integers(-2, 3, size=(len(keys), cols)).astype(np.int32)
            if i == per:  # call 1, push 0: a counter goes negative
                j = int(np.nonzero((keys >= 0) & (keys < rows))[0][250])
                vals[j, 9] = -1000
        host.append(encode_matrix_push(keys, vals, 0, fmt.valueType))
    dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in host]  # alive until the end
    torch.cuda.synchronize()
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    if ada:
        o.set_alpha(0.025, 0.0001, 1.5)
    else:
        o.synth_fill(11)
    err = None
    for h in host:  # the client's split: out-of-matrix keys never reach the server
        r = np.frombuffer(h, np.uint8).reshape(-1, 4 + 4 * cols)
        k = r[:, :4].copy().view("<i4").ravel()
        if o.push(r[(k >= 0) & (k < rows)].tobytes()):
            err = o.error()
            break
    assert (err is None) == ada
    port = None
    if binding == "torch":
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        g = ShardGroup(fmt, rows, cols, 0, 1, device=0, exchange_only=True)
    else:
        g = NativeShardGroup(fmt, rows, cols, 0, 1, NativeShardGroup.unique_id(), device=0)
    try:
        if ada:
            g.store.setAlpha(0.025, 0.0001, 1.5)
        else:
            g.store.synth_fill(11)
        raised = None
        try:
            for c in range(calls):
                sl = dev[c * per:(c + 1) * per]
                g.push_exchange([d.data_ptr() for d in sl], [d.numel() for d in sl])
            g.flush()
        except DistMLException as e:
            raised = e
        if ada:
            assert raised is None, raised
            a, d = g.store.adagrad_state()
            assert kat.bits_equal(a, o.alpha) and kat.bits_equal(d, o.delta)
            assert g.store.maxDelta() == o.max_delta()
        else:
            assert raised is not None and (raised.code, raised.key, raised.col) == err
        assert kat.bits_equal(g.store.values(), o.data)
    finally:
        try:
            g.close()  # the torch group flushes first: the failed store raises again (it refuses pushes)
        except DistMLException:
            if ada:
                raise
        if port is not None:
            dist.destroy_process_group()


def test_native_group_exchange_world1(oracle):
    """dml_group_push_exchange at world 1 (native RCCL send/recv): two AdaGrad calls,
    then flush — bit-exact data, alpha, delta, maxDelta; then an int32-checked group
    whose second call drives a counter negative: the error surfaces at flush with the
    reference's key/col, and the shard holds the state the sequential oracle stops in."""
    from distml_amd import DataDesc, IllegalStateException, encode_matrix_push
    from distml_amd.group import NativeShardGroup
    rows, cols = 1500, 200
    fmt = DataDesc(1, 0, 1, False, True, True)
    g = NativeShardGroup(fmt, rows, cols, 0, 1, NativeShardGroup.unique_id(), device=0)
    rng = np.random.default_rng(91)
    try:
        g.store.setAlpha(0.025, 0.0001, 1.5)
        host = []
        for b in range(6):
            keys = rng.permutation(rows)[: rng.integers(100, rows)]
            host.append(encode_matrix_push(keys, (rng.standard_normal((len(keys), cols)) * 0.6).astype(np.float32),
                                           0, 1))
        dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in host]
        torch.cuda.synchronize()
        ptrs, lens = [d.data_ptr() for d in dev], [d.numel() for d in dev]
        g.push_exchange(ptrs[:4], lens[:4])
        g.push_exchange(ptrs[4:], lens[4:])
        g.flush()
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        o.set_alpha(0.025, 0.0001, 1.5)
        for h in host:
            assert o.push(h) == 0
        assert kat.bits_equal(g.store.values(), o.data)
        a, d = g.store.adagrad_state()
        assert kat.bits_equal(a, o.alpha) and kat.bits_equal(d, o.delta)
        assert g.store.maxDelta() == o.max_delta()
    finally:
        g.close()

    ifmt = DataDesc(1, 0, 0)
    g = NativeShardGroup(ifmt, rows, 16, 0, 1, NativeShardGroup.unique_id(), device=0)
    try:
        g.store.load_values(np.full((rows, 16), 3, np.int32))
        ok = encode_matrix_push(np.arange(rows), np.full((rows, 16), -1, np.int32), 0, 0)
        bad = encode_matrix_push(np.array([7, 5]), np.array([[0] * 16, [0] * 3 + [-9] + [0] * 12], np.int32), 0, 0)
        dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in (ok, bad)]
        torch.cuda.synchronize()
        g.push_exchange([dev[0].data_ptr()], [dev[0].numel()])
        g.push_exchange([dev[1].data_ptr()], [dev[1].numel()])
        with pytest.raises(IllegalStateException) as ei:
            g.flush()
        assert (ei.value.key, ei.value.col) == (5, 3)
        o = oracle.OracleStore(1, 0, 0, 0, rows - 1, 16)
        o.data[:] = 3
        assert o.push(ok) == 0
        assert o.push(bad) != 0
        assert np.array_equal(g.store.values(), o.data)
    finally:
        g.close()


def test_native_group_exchange_float_array(oracle):
    """The exact exchange path for a sparse FloatArrayStore (config 3's store type,
    LONG keys) through the native group at world 1: repeated and out-of-matrix keys,
    bit-exact against the oracle fed the in-matrix records in push order."""
    from distml_amd import DataDesc, encode_array_push
    from distml_amd.group import NativeShardGroup
    dim = 1_000_000
    fmt = DataDesc(0, 1, 1)
    g = NativeShardGroup(fmt, dim, 1, 0, 1, NativeShardGroup.unique_id(), device=0)
    rng = np.random.default_rng(123)
    try:
        host = []
        for b in range(5):
            keys = rng.integers(-10, dim + 10, size=50_000)  # repeats inside a push, some outside the matrix
            host.append(encode_array_push(keys, rng.standard_normal(len(keys)).astype(np.float32), 1, 1))
        dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in host]
        torch.cuda.synchronize()
        g.push_exchange([d.data_ptr() for d in dev], [d.numel() for d in dev])
        g.flush()
        o = oracle_store(oracle, fmt, 0, dim - 1)
        for h in host:
            r = np.frombuffer(h, np.uint8).reshape(-1, 12)
            k = r[:, :8].copy().view("<i8").ravel()
            assert o.push(r[(k >= 0) & (k < dim)].tobytes()) == 0
        assert kat.bits_equal(g.store.values(), o.data)
    finally:
        g.close()


@pytest.mark.parametrize("kind", ["f32_matrix", "i32_matrix", "adagrad", "f64_matrix", "f32_array", "i32_array",
                                  "f64_array"])
@pytest.mark.parametrize("api", ["batch", "sequential", "device"])
def test_empty_and_single_record_pushes(oracle, kind, api):
    """Zero-length pushes (handlePush's record loop never runs: a no-op in the reference,
    e.g. FloatMatrixStore.java:200-208) at the start, middle and end of a batch, and
    one-record pushes, leave exactly the oracle's state."""
    from distml_amd import DataDesc, encode_array_push, encode_matrix_push
    rng = np.random.default_rng(sum(map(ord, kind + api)))
    vt = {"f32": 1, "i32": 0, "f64": 3, "adagrad": 1}[kind.split("_")[0]]
    matrix = not kind.endswith("array")
    cols = 6 if matrix else 1
    first, rows = 50, 40
    fmt = DataDesc(1 if matrix else 0, 0, vt, False, True, kind == "adagrad")
    s, _ = mk_store(fmt, first, first + rows - 1, cols)
    o = oracle_store(oracle, fmt, first, first + rows - 1, cols)
    init = (rng.integers(100, 200, size=(rows, cols)).astype(np.int32) if vt == 0
            else rng.standard_normal((rows, cols)).astype(s.dtype))
    s.load_values(init)
    o.data[:] = init

    def push(keys):
        v = (rng.integers(-3, 4, size=(len(keys), cols)) if vt == 0 else rng.standard_normal((len(keys), cols)))
        if matrix:
            return encode_matrix_push(first + keys, v, 0, vt)
        return encode_array_push(first + keys, v[:, 0], 0, vt)

    pushes = [b"", push(np.array([7])), b"", push(rng.choice(rows, 25, replace=False)), push(np.array([rows - 1])),
              b""]
    for p in pushes:
        assert o.push(p) == 0
    if api == "batch":
        s.handlePushBatch(fmt, pushes)
    elif api == "sequential":
        for p in pushes:
            s.handlePush(fmt, p)
    else:
        bufs = [torch.frombuffer(bytearray(p), dtype=torch.uint8).cuda() if p else
                torch.empty(0, dtype=torch.uint8, device="cuda") for p in pushes]
        torch.cuda.synchronize()
        s.pushDevice([b.data_ptr() for b in bufs], [b.numel() for b in bufs])
        s.flush()
    assert kat.bits_equal(s.values(), o.data)
    s.close()


@pytest.mark.parametrize("case", ["no_error", "hidden_negative", "late_negative", "async_batches"])
def test_int_array_repeated_keys_exact_error_state(oracle, case):
    """IntArrayStore pushes that list a key several times (legal bytes, never produced by
    SparseArray.writeMap): the reference adds in record order and throws after the first add
    that leaves a counter negative (IntArrayStore.java:97-113) — e.g. 1 + (-2) + 5 is
    negative after the first add in record order, never in the order (+5, -2). int32 arrays
    take the ordered partition + leaf path: every row's adds in sequence order with the
    check after each (rows of ~25 records here: leaves beyond the LDS sort go to the exact
    replay, which checks too), the chunk's first negative (min sequence) bounds the rollback
    of every later add: data, error key and the no-further-pushes state equal the oracle's."""
    from distml_amd import DataDesc, DistMLException, encode_array_push
    rng = np.random.default_rng(hash(case) % 1000)
    first, rows = 10, 3000
    fmt = DataDesc(0, 0, 0)
    init = rng.integers(30, 40, size=(rows, 1)).astype(np.int32)  # random walks stay >= 0
    pushes = []
    for b in range(5):
        k = rng.integers(0, 400, size=2000)  # ~5 repeats of each key in every push
        v = rng.integers(-1, 2, size=len(k))
        pushes.append(encode_array_push(first + k, v, 0, 0))
    if case == "hidden_negative":
        init[2500, 0] = 1
        pushes[2] = pushes[2] + encode_array_push(first + np.array([2500, 2500]), np.array([-2, 5]), 0, 0)
    elif case == "late_negative":
        init[1500, 0] = 3
        k = np.array([1500] * 6 + [1501])
        pushes[4] = encode_array_push(first + k, np.array([-1, -1, -1, -1, -1, -1, -1]), 0, 0) + pushes[4]
    apis = ["batch", "sequential"] if case != "async_batches" else ["async"]
    o = oracle_store(oracle, fmt, first, first + rows - 1)
    o.data[:] = init
    rc = 0
    for p in pushes:
        rc = o.push(p)
        if rc:
            break
    assert (rc != 0) == (case in ("hidden_negative", "late_negative"))
    for api in apis:
        s, _ = mk_store(fmt, first, first + rows - 1, async_push=(api == "async"))
        s.load_values(init)
        if rc:
            with pytest.raises(DistMLException) as ei:
                if api == "batch":
                    s.handlePushBatch(fmt, pushes)
                else:
                    for p in pushes:
                        s.handlePush(fmt, p)
            assert (ei.value.code, ei.value.key, ei.value.col) == o.error()
        elif api == "async":
            for i in range(0, len(pushes), 2):
                s.handlePushBatch(fmt, pushes[i:i + 2])
            s.flush()
        else:
            s.handlePushBatch(fmt, pushes) if api == "batch" else [s.handlePush(fmt, p) for p in pushes]
        assert kat.bits_equal(s.values(), o.data)
        s.close()


@pytest.mark.parametrize("async_push", [False, True])
def test_pinned_push_matches_oracle(oracle, async_push):
    """Row f2 (wire ingest into pinned memory): pushes that sit in pinned host
    buffers (pinned_empty = dml_host_alloc, what the JNI DirectByteBuffer wraps) are
    DMA'd without staging, one at a time and as a batch, synchronous and
    DML_FLAG_ASYNC; bit-exact vs the oracle. The buffers are overwritten right
    after each call returns: the bytes are borrowed for the call only
    (PSAgent.java:278-281), so the store must have captured them by then."""
    from distml_amd import DataDesc, DataStore, KeyRange, encode_matrix_push, encode_array_push
    from distml_amd.store import pinned_empty
    rng = np.random.default_rng(11)
    for fmt, cols in ((DataDesc(1, 0, 1), 300), (DataDesc(0, 1, 0), 1)):
        rows = 777
        st = DataStore(fmt, KeyRange(0, rows - 1), cols, async_push=async_push)
        o = oracle_store(oracle, fmt, 0, rows - 1, cols)
        if fmt.valueType == 0:
            init = rng.integers(100, 200, size=(rows, cols)).astype(np.int32)
        else:
            init = rng.standard_normal((rows, cols)).astype(np.float32)
        st.load_values(init)
        o.data[:] = init
        pushes = []
        for b in range(5):
            keys = rng.permutation(rows)[: rows - 50 * b]
            if fmt.dataType == 1:
                v = (rng.standard_normal((len(keys), cols)) * 1e-3).astype(np.float32)
                pushes.append(encode_matrix_push(keys, v, fmt.keyType, fmt.valueType))
            else:
                v = rng.integers(-3, 4, size=len(keys)).astype(np.int32)
                pushes.append(encode_array_push(keys, v, fmt.keyType, fmt.valueType))
        pin = [pinned_empty(len(p)) for p in pushes]
        # one at a time
        for p, buf in zip(pushes[:2], pin[:2]):
            buf[:] = np.frombuffer(p, np.uint8)
            st.handlePush(fmt, buf)
            buf[:] = 0xAB  # the caller reuses its buffer at once
            assert o.push(p) == 0
        # as one batch
        for p, buf in zip(pushes[2:], pin[2:]):
            buf[:] = np.frombuffer(p, np.uint8)
        st.handlePushBatch(fmt, pin[2:])
        for buf in pin[2:]:
            buf[:] = 0xCD
        for p in pushes[2:]:
            assert o.push(p) == 0
        st.flush()
        assert st.values().tobytes() == o.data.tobytes()
        st.close()


def test_rand_reference_distributions(oracle):
    """DataStore.rand (dml_store_rand). DoubleMatrixStore: bit-exact against the
    oracle's restatement of DoubleMatrixStore.java:192-207 (java.util.Random(1L) per
    shard, fdlibm log in nextGaussian, |g| rows divided by their norm; the oracle's
    Random is pinned by Java's published outputs, tests/test_oracle_kat.py), on two
    shards of one matrix (both start from Random(1L)). FloatMatrixStore's
    (nextInt(100)/100f - 0.5f) / rowSize values (FloatMatrixStore.java:39-51; AdaGrad
    :55-66) come from an unseeded Random there: every value one of the 100 float
    results, each a near-uniform share, same seed same values. int / array stores
    unchanged (DataStore.rand is a no-op, DataStore.java:22)."""
    from distml_amd import DataDesc, DataStore, KeyRange
    rows, cols = 2000, 50
    allowed = {((np.float32(a) / np.float32(100.0)) - np.float32(0.5)) / np.float32(cols) for a in range(100)}
    for ada in (False, True):
        st = DataStore(DataDesc(1, 0, 1, False, True, ada), KeyRange(0, rows - 1), cols)
        st.rand(5)
        v = st.values()
        st2 = DataStore(DataDesc(1, 0, 1, False, True, ada), KeyRange(0, rows - 1), cols)
        st2.rand(5)
        assert v.tobytes() == st2.values().tobytes()
        uniq, cnt = np.unique(v, return_counts=True)
        assert set(uniq.tolist()) <= {float(x) for x in allowed} and len(uniq) == 100
        assert cnt.min() > 0.8 * v.size / 100 and cnt.max() < 1.2 * v.size / 100
        st.close()
        st2.close()
    # ragged shapes, a shard past 2^21 elements (the host generates blocks of rows)
    for first, last, c in ((0, 999, 10), (1000, 1536, 10), (0, 2, 1), (5, 9000, 300)):
        st = DataStore(DataDesc(1, 1, 3), KeyRange(first, last), c)
        st.rand(9)
        v = st.values()
        o = oracle.OracleStore(1, 1, 3, first, last, c)
        assert o.rand() == 0
        assert v.tobytes() == o.data.tobytes(), (first, last, c)
        assert np.all(v >= 0) and np.allclose(np.sqrt((v * v).sum(axis=1)), 1.0, rtol=1e-12)
        st.close()
    for fmt, c in ((DataDesc(1, 0, 0), 7), (DataDesc(0, 1, 1), 1), (DataDesc(0, 0, 0), 1)):
        st = DataStore(fmt, KeyRange(0, 99), c)
        st.rand(1)
        assert not st.values().any()
        st.close()


def test_zero_set_reference_semantics():
    """DataStore.zero() is a no-op on every store (DataStore.java:24; the float
    stores' zero(String) is an overload OP_ZERO never calls, FloatMatrixStore.java:57);
    set(String) fills the float matrix stores with Float.parseFloat
    (FloatMatrixStore.java:53-55, FloatMatrixStoreAdaGrad.java:69-71) and is a no-op
    on the others (DataStore.java:26)."""
    from distml_amd import DataDesc, DataStore, KeyRange
    for fmt, c in ((DataDesc(1, 0, 1), 5), (DataDesc(1, 0, 1, False, True, True), 5), (DataDesc(1, 0, 0), 5),
                   (DataDesc(1, 1, 3), 5), (DataDesc(0, 1, 1), 1), (DataDesc(0, 0, 3), 1), (DataDesc(0, 0, 0), 1)):
        st = DataStore(fmt, KeyRange(0, 63), c)
        st.fill(2)
        st.zero()
        assert np.all(st.values() == 2), fmt
        st.set("0.1")
        floatm = fmt.dataType == 1 and fmt.valueType == 1
        want = np.float32(0.1) if floatm else 2
        assert np.all(st.values() == want), fmt
        st.close()


@pytest.mark.parametrize("ada,asc", [(False, False), (False, True), (True, False)])
def test_config4_full_shard_bit_exact(oracle, ada, asc):
    """BASELINE config 4 at the full per-GPU shard bench.py --config 4 times:
    1 250 000 x 200 fp32 (linearSplit(8) of 10M rows), full-range pushes with every
    row permuted per push, device-resident, one batch — bit-exact against the oracle
    (VERDICT r1 #10). Plain sum: W = 8, oracle row-partitioned over 16 threads (each
    thread still applies its rows' adds in push order). AdaGrad (data, alpha, delta,
    maxDelta): W = 4, oracle single thread. Ascending rows take the identity-speculation
    path (no key index, every key verified by the reduce)."""
    import ctypes as C
    import math
    from distml_amd import DataDesc, DataStore, KeyRange, _lib
    rows, cols = 1_250_000, 200
    W = 4 if ada else 8
    fmt = DataDesc(1, 0, 1, False, True, ada)
    L = _lib.load()
    st = DataStore(fmt, KeyRange(0, rows - 1), cols)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    if ada:
        st.setAlpha(0.025, 0.0001, 1.0)
        o.set_alpha(0.025, 0.0001, 1.0)
    st.synth_fill(13)
    o.synth_fill(13)

    def perm(b):
        if asc:  # keys implicit = row: the identity-speculation path
            return 1, 0
        a = (3000 + b) * 2654435761 % rows | 1
        while math.gcd(a, rows) != 1:
            a += 1
        return a, b * 7919 % rows

    dev, host = [], []
    s0 = torch.cuda.current_stream().cuda_stream
    for b in range(W):
        pa, pc = perm(b)
        t = torch.empty(rows * (4 + 4 * cols), dtype=torch.uint8, device="cuda")
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows, rows, cols, 3000 + b, pa, pc,
                                        C.c_void_p(s0)) == 0
        dev.append(t)
        host.append(oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 3000 + b, pa, pc))
    torch.cuda.synchronize()
    st.pushDevice([t.data_ptr() for t in dev], [t.numel() for t in dev])
    st.flush()
    assert o.push_many(host, threads=1 if ada else 16) == 0
    assert st.values().tobytes() == o.data.tobytes()
    if ada:
        a, d = st.adagrad_state()
        assert a.tobytes() == o.alpha.tobytes() and d.tobytes() == o.delta.tobytes()
        assert st.maxDelta() == o.max_delta()
    st.close()


def _config4_rows(rows):
    """Sampled rows of the 10 M-row model: every 4 099th row, and every row of the last
    262 144, whose 800-B rows lie past 2^32 bytes of each array (and the pushes' 804-B
    records past 2^32 bytes of each push)."""
    return np.unique(np.concatenate([np.arange(0, rows, 4099), np.arange(rows - 262_144, rows)]))


def _perm10m(b, rows):
    import math
    a = (3000 + b) * 2654435761 % rows | 1
    while math.gcd(a, rows) != 1:
        a += 2
    return a, b * 7919 % rows


@pytest.mark.parametrize("case", ["sum_ascending", "sum_permuted", "adagrad", "adagrad_ascending", "prereduce_world8"])
def test_config4_model_size_sampled_rows(oracle, case):
    """The config-4 legs at the size bench.py times: the 10 M x 200 fp32
    model (8 GB per array; byte offsets past 2^32), device-resident full-range pushes,
    compared on sampled rows (_config4_rows) against the oracle fed the same rows'
    records (pyoracle.synth_dense_rows: a full-range push's per-element result does not
    depend on record order). sum_*: k_reduce_flat, 4 pushes (FloatMatrixStore.java:
    200-222), ascending (identity speculation) or permuted; adagrad: k_ada_flat, 2
    pushes, data / alpha / delta (FloatMatrixStoreAdaGrad.java:262-277), one ascending and
    one permuted (adagrad: k_ada_flat) or both ascending (adagrad_ascending: k_ada_ident,
    the bench's 4a leg); prereduce_world8:
    the kPreReduce partial a rank writes at N = 8 ([rank][row], 8 x 1 250 000 rows), one
    ascending and one permuted push summed in push order. All bit-exact."""
    import ctypes as C
    from distml_amd import DataDesc, DataStore, KeyList, KeyRange, _lib
    from distml_amd.group import HipOps
    rows, cols = 10_000_000, 200
    ada = case.startswith("adagrad")
    W = {"adagrad": 2, "adagrad_ascending": 2, "prereduce_world8": 2}.get(case, 4)
    fmt = DataDesc(1, 0, 1, False, True, ada)
    L = _lib.load()
    pick = _config4_rows(rows)
    s0 = torch.cuda.current_stream().cuda_stream
    dev = []
    for b in range(W):
        pa, pc = (1, 0) if case in ("sum_ascending", "adagrad_ascending") or (case != "sum_permuted" and b == 0) \
            else _perm10m(b, rows)
        t = torch.empty(rows * (4 + 4 * cols), dtype=torch.uint8, device="cuda")
        assert L.dml_synth_dense_bucket(t.data_ptr(), C.byref(fmt.to_c()), 0, rows, rows, cols, 3000 + b, pa, pc,
                                        C.c_void_p(s0)) == 0
        dev.append(t)
    torch.cuda.synchronize()
    o = oracle.OracleStore(1, 0, 1, 0, len(pick) - 1, cols, 1, int(ada))
    if case == "prereduce_world8":
        S = rows // 8
        part = torch.empty(8 * S * cols, dtype=torch.float32, device="cuda")
        ops = HipOps()
        h = ops.begin(fmt, 0, rows, cols, [t.data_ptr() for t in dev], [t.numel() for t in dev], s0)
        try:
            ops.piece(h, S, S, 0, 8 * S, part.data_ptr(), s0)
        finally:
            ops.end(h)
        torch.cuda.synchronize()
        got = part.view(-1, cols)[torch.from_numpy(pick).cuda()].cpu().numpy()
        del part
    else:
        st = DataStore(fmt, KeyRange(0, rows - 1), cols)
        if ada:
            st.setAlpha(0.025, 0.0001, 1.0)
            o.set_alpha(0.025, 0.0001, 1.0)
        st.synth_fill(13)
        o.synth_fill_rows(pick, 13)
        st.pushDevice([t.data_ptr() for t in dev], [t.numel() for t in dev])
        st.flush()
        if ada:
            want = "dml::k_ada_ident<" if case == "adagrad_ascending" else "dml::k_ada_flat<"
            assert st.kernel_name().startswith(want), (st.kernel_name(), want)
        if not ada:
            rec = np.frombuffer(st.handleFetch(fmt, KeyList(pick.tolist())), np.uint8).reshape(len(pick), 4 + 4 * cols)
            assert rec[:, :4].copy().view("<i4").ravel().tolist() == pick.tolist()
            got = rec[:, 4:].copy().view("<f4")
        else:  # (AdaGrad's fetch interleaves alpha, FloatMatrixStoreAdaGrad.java:150-174)
            got = st.values().reshape(rows, cols)[pick]
            a, d = st.adagrad_state()
            ga, gd = a.reshape(rows, cols)[pick], d.reshape(rows, cols)[pick]
            del a, d
        st.close()
    del dev
    torch.cuda.empty_cache()
    for b in range(W):
        assert o.push(oracle.synth_dense_rows(0, 1, pick, cols, 3000 + b).tobytes()) == 0
    assert got.tobytes() == o.data.tobytes(), case
    if ada:
        assert ga.tobytes() == o.alpha.tobytes() and gd.tobytes() == o.delta.tobytes()


def _sampled_rows(oracle, b, rows):
    """The record positions k_ident_check samples in push b of a chunk (32 evenly
    spaced + 32 hashed), so a test can corrupt records the sample does not see."""
    ev = {t * (rows - 1) // 31 for t in range(32)}
    hs = {oracle.splitmix64((b << 32) + t) % rows for t in range(32, 64)}
    return ev | hs


SPEC_SHAPES = [(256, 0, 1), (200, 0, 1), (100, 1, 3)]  # (cols, key type, value type)


@pytest.mark.parametrize("shape", SPEC_SHAPES, ids=["c256-i32-f32", "c200-i32-f32-flat", "c100-i64-f64-flat"])
@pytest.mark.parametrize("case", ["ascending", "swapped", "duplicate", "out_of_shard", "mixed_pipelined"])
def test_identity_speculation_exact(oracle, case, shape):
    """Identity speculation: full-range pushes whose sampled keys are
    ascending skip the key index; the reduce verifies every record's key and a
    chunk with a non-identity push re-runs exactly from its input buffer. Each case
    is bit-exact against the oracle, error state included: ascending pushes; an
    ascending push with two records swapped where the sample cannot see them; one
    with a row listed twice (and one missing: the repeated-row replay); one with an
    out-of-shard key (the cutoff: ArrayIndexOutOfBoundsException state); and
    several pipelined batches mixing all of them with permuted pushes. Shapes: whole
    1-KiB rows (k_reduce_rows FULL) and rows under 4 KiB (k_reduce_flat), int32 and
    int64 keys."""
    from distml_amd import DataDesc, DataStore, KeyRange, encode_matrix_push, ArrayIndexOutOfBoundsException
    cols, kt, vt = shape
    rows, W = 4000, 6
    fmt = DataDesc(1, kt, vt)
    vdt = np.float64 if vt == 3 else np.float32
    rng = np.random.default_rng(hash(case) % 2**32)
    st = DataStore(fmt, KeyRange(100, 100 + rows - 1), cols, async_push=True)
    o = oracle_store(oracle, fmt, 100, 100 + rows - 1, cols)
    init = rng.standard_normal((rows, cols)).astype(vdt)
    st.load_values(init)
    o.data[:] = init

    def push(b, kind):
        keys = np.arange(rows)
        free = sorted(set(range(rows)) - _sampled_rows(oracle, b % 64, rows))
        if kind == "permuted":
            keys = rng.permutation(rows)
        elif kind == "swapped":
            i = free[len(free) // 2]
            j = free[len(free) // 2 + 1]
            keys[i], keys[j] = keys[j], keys[i]
        elif kind == "duplicate":
            i = free[len(free) // 3]
            keys[i] = keys[free[len(free) // 3 + 5]]
        elif kind == "out_of_shard":
            keys = keys.copy()
            keys[free[len(free) // 2]] = rows + 7  # key - first outside the shard
        v = (rng.standard_normal((rows, cols)) * 1e-3).astype(vdt)
        return encode_matrix_push(keys + 100, v, kt, vt)

    if case == "mixed_pipelined":
        kinds = [["ascending"] * W, ["ascending", "permuted"] * 3, ["ascending", "swapped"] + ["ascending"] * 4,
                 ["ascending"] * W, ["duplicate"] + ["ascending"] * 5, ["permuted"] * W, ["ascending"] * W]
    else:
        kinds = [["ascending"] * 2 + [case] + ["ascending"] * (W - 3)]
    err = None
    dev_all = []
    for bi, ks in enumerate(kinds):
        host = [np.frombuffer(push(b, k), np.uint8).copy() for b, k in enumerate(ks)]
        dev = [torch.from_numpy(h).cuda() for h in host]
        dev_all.append(dev)
        torch.cuda.synchronize()
        st.pushDevice([d.data_ptr() for d in dev], [d.numel() for d in dev])
        if err is None:
            for h in host:
                rc = o.push(h.tobytes())
                if rc:
                    err = o.error()
                    break
    if err is None:
        st.flush()
    else:
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            st.flush()
        assert (ei.value.key, ei.value.col) == (err[1], err[2])
    assert st.values().tobytes() == o.data.tobytes()
    if case == "ascending":
        # the speculative path ran: a verified chunk commits the other shard buffer
        p0 = st.device_ptr()
        st.pushDevice([d.data_ptr() for d in dev_all[0]], [d.numel() for d in dev_all[0]])
        st.flush()
        assert st.device_ptr() != p0
        if cols * (8 if vt == 3 else 4) < 4096:
            # all-identity flat chunks run the lean kernel (chosen from the index's Ctrl)
            assert st.kernel_name().startswith("dml::k_flat_ident<"), st.kernel_name()
        for d in dev_all[0]:
            assert o.push(d.cpu().numpy().tobytes()) == 0
        assert st.values().tobytes() == o.data.tobytes()
    st.close()


@pytest.mark.parametrize("batched", [True, False])
def test_adagrad_maxdelta_tie_repeated_row(oracle, batched):
    """a push that lists row 5 twice reaches delta 2.0 at its second
    record, before row 2 reaches the same 2.0 at the third record. The reference's
    strict `deltas[i] > maxDelta` (FloatMatrixStoreAdaGrad.java:273-277) keeps row 5.
    Row 5 is replayed in layers; its candidate must still win the tie."""
    from distml_amd import DataDesc, encode_matrix_push
    rows, cols = 8, 4
    fmt = DataDesc(1, 0, 1, False, True, True)
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    s.setAlpha(0.025, 0.0001, 1.5)
    o.set_alpha(0.025, 0.0001, 1.5)
    one = np.zeros((1, cols), np.float32)
    one[0, 0] = 1.0
    p1 = encode_matrix_push([2], one, 0, 1)
    p2 = encode_matrix_push([5, 5, 2], np.repeat(one, 3, axis=0), 0, 1)
    for p in (p1, p2):
        assert o.push(p) == 0
    if batched:
        s.handlePushBatch(fmt, [p1, p2])
    else:
        s.handlePush(fmt, p1)
        s.handlePush(fmt, p2)
    assert o.max_delta() == (2.0, 5, 0)
    assert s.maxDelta() == o.max_delta()
    assert kat.bits_equal(s.values(), o.data)


@pytest.mark.parametrize("case", ["hot_line", "cutoff", "truncated", "push_repeat", "f64"])
def test_sparse_single_pass_partition_exact(oracle, case):
    """The single-pass sparse partition (fixed-capacity bins, atomic cursors; DESIGN.md
    §4) against the oracle, bit-exact, where it must fall back or cut: `hot_line` — 40
    pushes all list keys 777..778 (one 32-row line bucket of a leaf holds > 64
    records): the leaf kernel flags the leaf and the packed exact replay applies it;
    `cutoff` — a key outside the shard in the middle of push 3: records from it on
    are not applied (the sequence cut), error state as the reference's;
    `truncated` — the last push ends inside a record; `push_repeat` — push 2 lists
    one key twice (fp32 compact records order a row's adds by push only, so the leaf
    goes to the replay, which re-partitions with full sequence numbers); `f64` —
    DoubleArrayStore (full records) with cross-push repeats only."""
    from distml_amd import DataDesc, DistMLException, encode_array_push
    rng = np.random.default_rng(len(case))
    first, rows = 3, 2_000_000
    vt = 3 if case == "f64" else 1
    dt = np.float64 if vt == 3 else np.float32
    fmt = DataDesc(0, 1, vt)  # Float/DoubleArrayStore, LONG keys
    s, _ = mk_store(fmt, first, first + rows - 1)
    o = oracle_store(oracle, fmt, first, first + rows - 1)
    init = rng.standard_normal((rows, 1)).astype(dt)
    s.load_values(init)
    o.data[:] = init
    nb = 40 if case == "hot_line" else 6
    pushes = []
    for b in range(nb):
        keys = rng.choice(rows, size=20_000, replace=False) + first
        if case == "hot_line":
            keys[:2] = [777 + first, 778 + first]
        if case == "push_repeat" and b == 2:
            keys[17] = keys[5]
        vals = (rng.standard_normal(len(keys)) * 1e-2).astype(dt)
        p = encode_array_push(keys, vals, 1, vt)
        if case == "cutoff" and b == 3:
            bad = encode_array_push([rows + first + 5], [1.0], 1, 1)
            p = p[:12 * 9000] + bad + p[12 * 9000:]
        if case == "truncated" and b == nb - 1:
            p = p[:-7]
        pushes.append(p)
    err = None
    for p in pushes:
        rc = o.push(p)
        if rc:
            err = o.error()
            break
    if err is None:
        s.handlePushBatch(fmt, pushes)
    else:
        with pytest.raises(DistMLException) as ei:
            s.handlePushBatch(fmt, pushes)
        assert (ei.value.code, ei.value.key) == (err[0], err[1])
    assert s.values().tobytes() == o.data.tobytes()


@pytest.mark.parametrize("case", ["random", "lattice", "hot_big_leaf", "repeats", "push_repeat", "cutoff",
                                  "unbalanced"])
def test_sparse_big_leaves_exact(oracle, case):
    """The one-level partition (big leaves of 2^BL rows sorted in LDS)
    against the oracle, bit-exact (FloatArrayStore.java:110-122): a 4 M-row fp32 array
    shard and 16 pushes of 2 M keys — every row listed by ~8 pushes (owner chains in
    every bucket), big leaves as the planner sizes them for kSpBigBins / kSpBigCap.
    random — unique keys per push; lattice — the bench's config-3 key order
    ((a r + c) mod dim per push); hot_big_leaf — every push adds 1 000 keys inside one
    big leaf, over 32 pushes (past kSpBigCap: that leaf takes the exact replay); repeats — pushes
    drawn from half the rows (~10 adds per row); push_repeat — one push lists a key
    twice (the replay re-partitions with full sequence numbers); cutoff — a key outside
    the shard (the counted partition, sequence cut, error state); unbalanced — one push
    twice the others' size lands in one slice (the two-level path)."""
    from distml_amd import DataDesc, DistMLException, encode_array_push
    rng = np.random.default_rng(7 + len(case))
    first, rows = 11, 1 << 22
    # hot_big_leaf: 32 pushes of 1 M keys (same 32 M records), so one push per row
    # still overfills a big leaf whatever its size (a leaf holds <= pushes x rows)
    nb, per = (32, 1 << 20) if case == "hot_big_leaf" else (16, 1 << 21)
    fmt = DataDesc(0, 1, 1)  # FloatArrayStore, LONG keys
    s, _ = mk_store(fmt, first, first + rows - 1)
    o = oracle_store(oracle, fmt, first, first + rows - 1)
    init = rng.standard_normal((rows, 1)).astype(np.float32)
    s.load_values(init)
    o.data[:] = init
    pushes = []
    for b in range(nb):
        n = per * 12 if case == "unbalanced" and b == 0 else per
        if case == "lattice":
            a = (2 * b + 3) * 999_999_937 % rows | 1
            keys = (a * np.arange(n, dtype=np.int64) + b * 12_345_701) % rows
        elif case == "repeats":
            keys = np.unique(rng.choice(rows // 2, size=n, replace=True))
            rng.shuffle(keys)
        else:
            keys = rng.choice(rows, size=min(n, rows), replace=False)
        keys = keys + first
        if case == "hot_big_leaf":
            keys[:1000] = first + 5 * 1024 + rng.choice(1024, size=1000, replace=False)
            keys = np.concatenate([keys[:1000], np.setdiff1d(keys[1000:], keys[:1000])])
        if case == "push_repeat" and b == 5:
            keys[17] = keys[5]
        vals = (rng.standard_normal(len(keys)) * 1e-2).astype(np.float32)
        p = encode_array_push(keys, vals, 1, 1)
        if case == "cutoff" and b == 9:
            p = p[:12 * 9000] + encode_array_push([rows + first + 5], [1.0], 1, 1) + p[12 * 9000:]
        pushes.append(p)
    err = None
    for p in pushes:
        if o.push(p):
            err = o.error()
            break
    s.stats(reset=True)
    if err is None:
        s.handlePushBatch(fmt, pushes)
    else:
        with pytest.raises(DistMLException) as ei:
            s.handlePushBatch(fmt, pushes)
        assert (ei.value.code, ei.value.key) == (err[0], err[1])
    st = s.stats(reset=True)
    assert s.values().tobytes() == o.data.tobytes()
    big = case not in ("cutoff", "unbalanced")
    assert st["sparse_big_chunks"] == (1 if big else 0), st
    assert st["sparse_replays"] == (1 if case in ("hot_big_leaf", "push_repeat") else 0), st


@pytest.mark.parametrize("cols", [200, 64])
@pytest.mark.parametrize("W", [1, 2, 4])
@pytest.mark.parametrize("case", ["plain", "large", "cutoff", "repeat"])
def test_adagrad_flat_exact(oracle, case, W, cols):
    """k_ada_flat (AdaGrad chunks of <= 4 dense pushes, rows under 4 KiB)
    bit-exact against the oracle: data, alpha, delta, maxDelta/row/col and error
    state. `large`: gradients that drive delta past 1 (alpha written at write-back),
    plus a NaN and an Inf element; `cutoff`: a key outside the shard in the middle of
    the second push (ArrayIndexOutOfBoundsException state); `repeat`: the first push
    lists a row twice (the host's exact replay layers, maxDelta finalized after them)."""
    from distml_amd import DataDesc, DistMLException, encode_matrix_push
    rng = np.random.default_rng(1000 * W + cols + len(case))
    first, rows = 50, 3000
    fmt = DataDesc(1, 0, 1, False, True, True)
    s, _ = mk_store(fmt, first, first + rows - 1, cols)
    o = oracle_store(oracle, fmt, first, first + rows - 1, cols)
    s.setAlpha(0.025, 0.0001, 1.5)
    o.set_alpha(0.025, 0.0001, 1.5)
    init = rng.standard_normal((rows, cols)).astype(np.float32)
    s.load_values(init)
    o.data[:] = init
    pushes = []
    for b in range(W):
        keys = rng.permutation(rows)
        scale = 0.7 if case == "large" else 1e-2
        v = (rng.standard_normal((rows, cols)) * scale).astype(np.float32)
        if case == "large" and b == 0:
            v[10, 3], v[11, 5] = np.nan, np.inf
        if case == "repeat" and b == 0:
            keys[100] = keys[200]
        p = encode_matrix_push(keys + first, v, 0, 1)
        if case == "cutoff" and b == min(1, W - 1):
            rec = 4 + 4 * cols
            bad = encode_matrix_push([first + rows + 9], np.ones((1, cols), np.float32), 0, 1)
            p = p[:rec * 1500] + bad + p[rec * 1500:]
        pushes.append(p)
    err = None
    for p in pushes:
        if o.push(p):
            err = o.error()
            break
    if err is None:
        s.handlePushBatch(fmt, pushes)
    else:
        with pytest.raises(DistMLException):
            s.handlePushBatch(fmt, pushes)
        assert s.error_state() == (err[0], err[1], err[2])
    assert kat.bits_equal(s.values(), o.data)
    a, d = s.adagrad_state()
    assert kat.bits_equal(a, o.alpha) and kat.bits_equal(d, o.delta)
    assert s.maxDelta() == o.max_delta()
    s.close()


@pytest.mark.parametrize("cols", [200, 256, 48])
@pytest.mark.parametrize("W", [1, 2, 3, 4])
@pytest.mark.parametrize("case", ["plain", "large", "swapped", "partial", "tiny"])
def test_adagrad_ident_exact(oracle, case, W, cols):
    """k_ada_ident (AdaGrad chunks of full-range pushes whose records are rows in order,
    every key checked before the launch) bit-exact against the oracle:
    data, alpha, delta, maxDelta/row/col. The key check's threshold is lowered
    (DML_KNOB_IDENT_FULL_MIN_BYTES) so the path runs at this size. `large`: delta past 1
    (alpha written) plus a NaN and an Inf element; `swapped`: the last push has two
    records swapped (not identity: k_ada_flat takes the chunk); `partial`: the last push
    omits the last row (not full-range: the key index, k_ada_flat). Two batches, so the
    second starts from the first's delta and maxDelta. `tiny`: 5 rows, a grid rounded up
    past the rows (more candidate slots than k_reduce's count at 256 columns)."""
    from distml_amd import DataDesc, encode_matrix_push
    rng = np.random.default_rng(100 * W + cols + len(case))
    first, rows = 50, (5 if case == "tiny" else 2999)  # a short last wave
    fmt = DataDesc(1, 0, 1, False, True, True)
    s, _ = mk_store(fmt, first, first + rows - 1, cols)
    s.set_knob(1, 0)
    o = oracle_store(oracle, fmt, first, first + rows - 1, cols)
    s.setAlpha(0.025, 0.0001, 1.5)
    o.set_alpha(0.025, 0.0001, 1.5)
    init = rng.standard_normal((rows, cols)).astype(np.float32)
    s.load_values(init)
    o.data[:] = init
    for batch in range(2):
        pushes = []
        for b in range(W):
            keys = np.arange(rows)
            scale = 0.7 if case == "large" else 1e-2
            v = (rng.standard_normal((rows, cols)) * scale).astype(np.float32)
            if case == "large" and b == 0 and batch == 0:
                v[10, 3], v[2000, 5] = np.nan, np.inf
            if case == "tiny":
                v *= 100.0  # delta past 1: alpha written
            if b == W - 1 and case == "swapped":
                keys[[7, 1900]] = keys[[1900, 7]]
            if b == W - 1 and case == "partial":
                keys, v = keys[:-1], v[:-1]
            pushes.append(encode_matrix_push(keys + first, v, 0, 1))
        for p in pushes:
            assert o.push(p) == 0
        s.handlePushBatch(fmt, pushes)
        want = "dml::k_ada_ident<" if case in ("plain", "large", "tiny") else "dml::k_ada_flat<"
        assert s.kernel_name().startswith(want), (s.kernel_name(), want)
        assert kat.bits_equal(s.values(), o.data)
        a, d = s.adagrad_state()
        assert kat.bits_equal(a, o.alpha) and kat.bits_equal(d, o.delta)
        assert s.maxDelta() == o.max_delta()
    s.close()


@pytest.mark.parametrize("cols", [1024, 256, 200, 2048, 1280])
@pytest.mark.parametrize("case", ["same_order", "swapped_late", "duplicate_late", "out_of_shard_late", "order_change",
                                  "nb_change", "order_shuffled"])
def test_slot_reuse_exact(oracle, case, cols):
    """Slot reuse: a speculative k_reduce_rows chunk keeps its slot
    table, and the chunk three batches later in the same workspace takes a push's
    slots from the column of the push at the same position when its sampled keys
    match (k_ident_check); the reduce verifies every record's key and a mismatch
    re-runs the chunk exactly. Seven batches of six full-range permuted pushes (new
    values each batch), bit-exact against the oracle, error state included. Batch 3
    (the first that can reuse) varies by case: the same orders; push 2 with two
    records swapped where the sample cannot see them; with a row listed twice; with
    an out-of-shard key there; all new orders (batch 6 then repeats batch 3's); nine
    pushes (another slot-table stride, no reuse); from batch 3 on the six pushes in a
    new order every batch (arrival order: reuse is keyed by content, not position).
    Rows of whole 4 KiB (k_reduce_rows FULL; 8 KiB: two chunk groups per row), of 1
    KiB and 800 B (k_reduce_flat), and of 5 KiB (1280 cols: the pair-packed loop,
    which never speculates — ADVICE r2)."""
    from distml_amd import DataDesc, DataStore, KeyRange, encode_matrix_push, ArrayIndexOutOfBoundsException
    rows, W = 4000, 6
    fmt = DataDesc(1, 0, 1)
    rng = np.random.default_rng(len(case) * 7 + cols)
    st = DataStore(fmt, KeyRange(100, 100 + rows - 1), cols, async_push=True)
    o = oracle_store(oracle, fmt, 100, 100 + rows - 1, cols)
    init = rng.standard_normal((rows, cols)).astype(np.float32)
    st.load_values(init)
    o.data[:] = init
    perms = [rng.permutation(rows) for _ in range(9)]
    new_perms = [rng.permutation(rows) for _ in range(9)]
    err = raised = None
    keep = []
    for bi in range(7):
        n = 9 if (case == "nb_change" and bi == 3) else W
        order = new_perms if (case == "order_change" and bi in (3, 6)) else perms
        pos = rng.permutation(n) if (case == "order_shuffled" and bi >= 3) else np.arange(n)
        host = []
        for b in range(n):
            keys = order[pos[b]].copy()
            if bi == 3 and b == 2 and case.endswith("_late"):
                free = sorted(set(range(rows)) - _sampled_rows(oracle, b, rows))
                i, j = free[len(free) // 2], free[len(free) // 2 + 3]
                if case == "swapped_late":
                    keys[i], keys[j] = keys[j], keys[i]
                elif case == "duplicate_late":
                    keys[i] = keys[j]
                else:
                    keys[i] = rows + 11  # key - first outside the shard
            v = (rng.standard_normal((rows, cols)) * 1e-3).astype(np.float32)
            host.append(np.frombuffer(encode_matrix_push(keys + 100, v, 0, 1), np.uint8).copy())
        dev = [torch.from_numpy(h).cuda() for h in host]
        keep.append(dev)
        torch.cuda.synchronize()
        try:
            st.pushDevice([d.data_ptr() for d in dev], [d.numel() for d in dev])
        except ArrayIndexOutOfBoundsException as e:  # an earlier batch's error, surfaced at retire
            assert err is not None
            raised = e
            break
        if err is None:
            for h in host:
                if o.push(h.tobytes()):
                    err = o.error()
                    break
    if err is None:
        st.flush()
    elif raised is None:
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            st.flush()
        raised = ei.value
    if err is not None:
        assert (raised.key, raised.col) == (err[1], err[2])
    got = st.values()
    bad_rows = np.nonzero((got.view(np.uint32) != o.data.view(np.uint32)).any(axis=1))[0]
    assert len(bad_rows) == 0, (len(bad_rows), bad_rows[:8])
    stats = st.stats()
    if cols == 1280:
        assert stats["spec_chunks"] == 0, stats
    elif case in ("same_order", "order_shuffled"):
        # batches 3..6 take every push's slots from a kept column (chunk j-3's table)
        assert stats["reused_pushes"] == 4 * W and stats["spec_reruns"] == 0, stats
    st.close()


@pytest.mark.parametrize("rows,cols", [(3000, 1024), (2_200_000, 4), (2_200_000, 256)])
@pytest.mark.parametrize("case", ["ascending", "swapped", "rotated"])
def test_prereduce_verified_identity(case, rows, cols):
    """The sharded pre-reduce's identity pushes (dml_prereduce_begin): when the slot
    table is beyond the caches (rows x stride x 4 B > 64 MB: the 2.2 M-row cases),
    full-range pushes whose records are rows in order skip the key index after a
    complete key check, and the pieces take slot = row for them; the 3 000-row case
    keeps the index. The partial equals the ordered float32 sum of the pushes from
    zero, bit for bit: ascending pushes; push 1 with two records swapped (the check
    sends it to the index); push 1 rotated by one record. Rows of 16 B
    (k_reduce_flat) and 1 KiB (k_reduce_rows)."""
    from distml_amd import DataDesc, encode_matrix_push
    from distml_amd.group import HipOps
    W = 2
    fmt = DataDesc(1, 0, 1)
    rng = np.random.default_rng(len(case) + cols)
    expect = np.zeros((rows, cols), np.float32)
    dev = []
    for b in range(W):
        keys = np.arange(rows)
        if b == 1 and case == "swapped":
            i, j = rows // 3, rows // 3 + 11
            keys[i], keys[j] = keys[j], keys[i]
        elif b == 1 and case == "rotated":
            keys = np.roll(keys, 1)
        v = rng.standard_normal((rows, cols), dtype=np.float32)
        expect[keys] += v  # float32: one IEEE rounding per add, push order
        dev.append(torch.frombuffer(bytearray(encode_matrix_push(keys, v, 0, 1)), dtype=torch.uint8).cuda())
        del v
    out = torch.full((rows * cols,), 7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ops = HipOps()
    st = torch.cuda.current_stream().cuda_stream
    h = ops.begin(fmt, 0, rows, cols, [d.data_ptr() for d in dev], [d.numel() for d in dev], st)
    ops.piece(h, rows, rows, 0, rows, out.data_ptr(), st)
    torch.cuda.synchronize()
    ops.end(h)
    assert out.cpu().numpy().reshape(rows, cols).tobytes() == expect.tobytes()


@pytest.mark.parametrize("case", ["ascending", "rotated", "out_of_shard"])
def test_adagrad_identity_checked_large(oracle, case):
    """AdaGrad chunks of k_ada_flat with a slot table beyond the caches (2.2 M rows):
    full-range pushes whose records are rows in order skip the key index after a
    complete key check (Batch::ident_ok); bit-exact data, alpha, delta, maxDelta and
    error state against the oracle. `rotated`: push 1 rotated by one record (the check
    sends it to the index); `out_of_shard`: push 1's record 1 000 000 holds a key
    outside the shard (ArrayIndexOutOfBoundsException state)."""
    from distml_amd import DataDesc, encode_matrix_push, ArrayIndexOutOfBoundsException
    rows, cols, W = 2_200_000, 8, 2
    fmt = DataDesc(1, 0, 1, False, True, True)
    rng = np.random.default_rng(len(case))
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    s.setAlpha(0.025, 0.0001, 1.5)
    o.set_alpha(0.025, 0.0001, 1.5)
    init = rng.standard_normal((rows, cols)).astype(np.float32)
    s.load_values(init)
    o.data[:] = init
    pushes = []
    for b in range(W):
        keys = np.arange(rows)
        if b == 1 and case == "rotated":
            keys = np.roll(keys, 1)
        if b == 1 and case == "out_of_shard":
            keys = keys.copy()
            keys[1_000_000] = rows + 5
        v = (rng.standard_normal((rows, cols)) * 0.8).astype(np.float32)  # delta passes 1 for some elements
        pushes.append(encode_matrix_push(keys, v, 0, 1))
    err = None
    for p in pushes:
        if o.push(p):
            err = o.error()
            break
    if err is None:
        s.handlePushBatch(fmt, pushes)
    else:
        with pytest.raises(ArrayIndexOutOfBoundsException):
            s.handlePushBatch(fmt, pushes)
        assert s.error_state() == (err[0], err[1], err[2])
    assert kat.bits_equal(s.values(), o.data)
    a, d = s.adagrad_state()
    assert kat.bits_equal(a, o.alpha) and kat.bits_equal(d, o.delta)
    assert s.maxDelta() == o.max_delta()
    s.close()


@pytest.mark.parametrize("vt", [1, 3])
def test_sampled_timing_and_write_through_rows(oracle, vt):
    """dml_store_set_timing(s, every): one chunk in `every` carries start/stop events
    (the others only the in-packet completion event), and the whole-KiB-row reduce
    stores write-through (stg16_wt): 24 async calls of two full-range pushes (one
    ascending, one permuted) on 4-KiB / 8-KiB rows, f32 and f64, bytes-equal against the
    oracle, with 24 / 4 = 6 timed launches."""
    from distml_amd import DataDesc
    from distml_amd.store import DeviceBatch
    rows, cols, calls = 512, 1024, 24
    fmt = DataDesc(1, 0, vt)
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    s.synth_fill(9)
    o.synth_fill(9)
    host = [oracle.synth_dense_bucket(0, vt, 0, rows, rows, cols, 300 + b, 1 if b % 2 == 0 else 77, 0 if b % 2 == 0 else 5)
            for b in range(4)]
    dev = [torch.from_numpy(h).cuda() for h in host]
    torch.cuda.synchronize()
    s.set_timing(True, every=4)
    for c in range(calls):
        pair = dev[2 * (c % 2): 2 * (c % 2) + 2]
        s.pushDevice(DeviceBatch([t.data_ptr() for t in pair], [t.numel() for t in pair]))
        for h in host[2 * (c % 2): 2 * (c % 2) + 2]:
            assert o.push(h.tobytes()) == 0
    s.flush()
    ms, n = s.kernel_time(reset=True)
    s.set_timing(False)
    assert n == calls // 4 and ms > 0.0
    assert "k_reduce_rows" in s.kernel_name() and s.kernel_name().endswith(", 2>")
    assert kat.bits_equal(s.values(), o.data)


@pytest.mark.parametrize("vt,cols", [(1, 4), (1, 8), (1, 100), (1, 200), (1, 700), (1, 1020), (3, 2), (3, 250), (3, 510)])
def test_flat_kernel_widths_exact(oracle, vt, cols):
    """k_reduce_flat's row packing (R = min(16, JMAX * 64 / vectors per row) rows per
    wave, JMAX = 12) at widths from one vector to just under 4 KiB, on a row count
    that no R divides: host batches of dense pushes (ascending, permuted, half the
    rows, one push listing a row twice -> the exact replay) and device calls of
    full-range pushes (identity speculation, slot reuse on the second pair of
    calls). Bytes-equal against the oracle."""
    from distml_amd import DataDesc, encode_matrix_push
    from distml_amd.store import DeviceBatch
    rng = np.random.default_rng(1000 + cols)
    rows = 1237
    fmt = DataDesc(1, 0, vt)
    dt = np.float32 if vt == 1 else np.float64
    s, _ = mk_store(fmt, 0, rows - 1, cols)
    o = oracle_store(oracle, fmt, 0, rows - 1, cols)
    s.synth_fill(21)
    o.synth_fill(21)
    pushes = []
    for b in range(5):
        keys = np.arange(rows) if b == 0 else rng.permutation(rows)[: rows if b < 3 else rows // 2 + 40 * b]
        if b == 4:
            keys = keys.copy()
            keys[5] = keys[100]  # one push lists a row twice
        pushes.append(encode_matrix_push(keys, rng.standard_normal((len(keys), cols)).astype(dt), 0, vt))
    s.handlePushBatch(fmt, pushes)
    for p in pushes:
        assert o.push(p) == 0
    assert kat.bits_equal(s.values(), o.data)
    # device calls of full-range pushes: ascending + a fixed permutation, twice, so the
    # third and fourth calls find the permutation kept by the workspace ring
    perm = rng.permutation(rows)
    host = [encode_matrix_push(np.arange(rows) if j % 2 == 0 else perm,
                               rng.standard_normal((rows, cols)).astype(dt), 0, vt) for j in range(8)]
    dev = [torch.frombuffer(bytearray(h), dtype=torch.uint8).cuda() for h in host]
    torch.cuda.synchronize()
    for c in range(4):
        pair = dev[2 * c: 2 * c + 2]
        s.pushDevice(DeviceBatch([t.data_ptr() for t in pair], [t.numel() for t in pair]))
        for h in host[2 * c: 2 * c + 2]:
            assert o.push(h) == 0
    s.flush()
    assert kat.bits_equal(s.values(), o.data)
    # an all-identity call (two ascending pushes): k_flat_ident at this width, with the
    # row count no wave's rows divide
    idn = [dev[0], dev[2]]
    s.pushDevice(DeviceBatch([t.data_ptr() for t in idn], [t.numel() for t in idn]))
    for j in (0, 2):
        assert o.push(host[j]) == 0
    s.flush()
    assert s.kernel_name().startswith("dml::k_flat_ident<"), s.kernel_name()
    assert kat.bits_equal(s.values(), o.data)


def test_prectx_refuses_a_fourth_outstanding_call(oracle):
    """A pre-reduce context's ring holds three workspaces: a fourth
    _begin_ctx while three calls are begun and not ended is refused instead of
    rewriting a workspace under its pieces; once one ends, the next call proceeds."""
    from distml_amd import DataDesc, NativeError
    from distml_amd.group import HipOps
    rows, cols = 512, 64
    fmt = DataDesc(1, 0, 1)
    ops = HipOps()
    ctx = ops.ctx_create(fmt, 0, rows, cols, 0)
    push = torch.from_numpy(oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 5, 1, 0)).cuda()
    part = torch.zeros(rows * cols, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    hs = [ops.begin_ctx(ctx, [push.data_ptr()], [push.numel()], st) for _ in range(3)]
    with pytest.raises(NativeError):
        ops.begin_ctx(ctx, [push.data_ptr()], [push.numel()], st)
    for h in hs[:1]:
        ops.piece(h, rows, rows, 0, rows, part.data_ptr(), st)
        ops.verify(h)
        ops.end(h)
    h = ops.begin_ctx(ctx, [push.data_ptr()], [push.numel()], st)
    for h2 in hs[1:] + [h]:
        ops.piece(h2, rows, rows, 0, rows, part.data_ptr(), st)
        ops.verify(h2)
        ops.end(h2)
    torch.cuda.synchronize()
    want = oracle.synth_dense_bucket(0, 1, 0, rows, rows, cols, 5, 1, 0).reshape(rows, -1)[:, 4:].copy().view("<f4")
    assert part.view(rows, cols).cpu().numpy().tobytes() == want.tobytes()
    ops.ctx_destroy(ctx)
