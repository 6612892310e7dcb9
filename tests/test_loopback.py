"""Config-1 plumbing on CPU: the reference framing
(distml_amd.psnet) and the MNIST MLR sample with 2 worker processes and 1 server
over loopback TCP. Here the server's store is the CPU oracle (a8,
DoubleMatrixStore.java:163-175) behind the same handlePush / handleFetch calls;
tests/test_gpu_loopback.py puts the GPU DataStore there.

Golden bytes below are hand-derived from the reference's writers
(DataBusProtocol.java:148-165,194-203,262-304; DataDesc.java:62-69;
KeyList.java:31-43; KeyRange.java:43-54), not produced by this code.
"""
import struct

import numpy as np
import pytest

from distml_amd import loopback, psnet
from distml_amd.datadesc import ALL, EMPTY, DataDesc, KeyList, KeyRange


class OracleShard:
    """The CPU oracle behind the DataStore calls PSAgent makes (test-only)."""

    def __init__(self, oracle, fmt, keys: KeyRange, cols):
        self.keys = keys
        self.o = oracle.OracleStore(fmt.dataType, fmt.keyType, fmt.valueType, keys.firstKey, keys.lastKey, cols,
                                    int(fmt.denseColumn), int(fmt.adaGrad))

    def handlePush(self, fmt, data):
        rc = self.o.push(data)
        if rc != 0:
            raise RuntimeError(f"push failed: {self.o.error()}")

    def handleFetch(self, fmt, rows):
        ks = self.keys.intersect(rows)
        return self.o.fetch(list(ks))


def test_push_request_bytes():
    fmt = loopback.MLR_FORMAT
    data = struct.pack("<q", 5) + np.arange(10, dtype="<f8").tobytes()
    msg = psnet.push_request("weights", fmt, data)
    exp = (struct.pack(">i", 2)                       # MSG_PUSH_REQUEST
           + struct.pack(">6i", 1, 1, 3, 0, 1, 0)      # MATRIX, LONG, DOUBLE, !denseRow, denseColumn, !adaGrad
           + struct.pack(">i", len(data)) + data
           + struct.pack(">i", 7) + b"weights")
    assert msg == exp
    assert psnet.frame(msg)[:4] == struct.pack(">i", len(exp))


def test_fetch_request_bytes():
    fmt = loopback.MLR_FORMAT
    msg = psnet.fetch_request("w", fmt, KeyList([3, 1]))
    exp = (struct.pack(">i", 0) + struct.pack(">i", 1) + b"w"
           + struct.pack(">i", 3) + struct.pack(">i", 2) + struct.pack(">q", 3) + struct.pack(">q", 1)
           + struct.pack(">i", 0))                     # cols: KeyCollection.ALL
    assert msg == exp
    ifmt = DataDesc(1, DataDesc.KEY_TYPE_INT, 1)
    assert psnet.write_keys(KeyRange(4, 9), ifmt) == struct.pack(">iii", 2, 4, 9)
    assert psnet.write_keys(EMPTY, ifmt) == struct.pack(">i", 1)


@pytest.mark.parametrize("key_type", [0, 1])
@pytest.mark.parametrize("keys", [ALL, EMPTY, KeyRange(-3, 70), KeyList([9, 2, 2**31 - 1]), KeyList()])
def test_key_collections_round_trip(keys, key_type):
    fmt = DataDesc(1, key_type, 1)
    r = psnet._Reader(psnet.write_keys(keys, fmt))
    back = psnet.read_keys(r, fmt)
    assert r.pos == len(r.buf)
    if keys is ALL or keys is EMPTY:
        assert back is keys
    elif isinstance(keys, KeyRange):
        assert back == keys
    else:
        assert list(back) == list(keys)


def test_rows_codec_round_trip():
    rows = {7: np.linspace(-1, 1, 10), 0: np.full(10, 2.5)}
    back = loopback.decode_rows(loopback.encode_rows(rows))
    assert list(back) == [7, 0]
    for k in rows:
        assert np.array_equal(back[k], rows[k])


def test_mnist_lines_shape():
    lines = loopback.mnist_lines(20)
    assert lines == loopback.mnist_lines(20)       # seeded
    for l in lines:
        items = l.split(" ")
        assert len(items) == 785
        px = [int(v) for v in items[:-1]]
        assert all(0 <= v <= 255 for v in px) and 0 <= int(items[-1]) <= 9
    x, label = loopback.parse_line(lines[0])
    assert all(v != 0.0 for v in x.values()) and label.sum() == 1.0


def test_server_fetch_push_one_client(oracle):
    fmt = loopback.MLR_FORMAT
    shard = OracleShard(oracle, fmt, loopback.shard_range(), 10)
    with psnet.PSServer({"weights": (shard, fmt)}) as srv:
        cli = psnet.PSClient(srv.address)
        push = loopback.encode_rows({3: np.full(10, 0.5), 700: np.arange(10.0)})
        assert cli.push("weights", fmt, push)
        assert cli.push("weights", fmt, push)
        got = loopback.decode_rows(cli.fetch("weights", fmt, KeyList([700, 3, 4])))
        cli.close()
    assert set(got) == {700, 3, 4}
    assert np.array_equal(got[3], np.full(10, 1.0))
    assert np.array_equal(got[700], 2 * np.arange(10.0))
    assert np.array_equal(got[4], np.zeros(10))
    assert [n for n, _ in srv.pushes] == ["weights", "weights"]


def test_push_error_drops_connection(oracle):
    """A key outside the shard: handlePush throws, the server drops the channel
    (PSAgent.java:188-191); the client sees the connection end, not an ack."""
    fmt = loopback.MLR_FORMAT
    shard = OracleShard(oracle, fmt, loopback.shard_range(), 10)
    with psnet.PSServer({"weights": (shard, fmt)}) as srv:
        cli = psnet.PSClient(srv.address)
        with pytest.raises(ConnectionError):
            cli.push("weights", fmt, loopback.encode_rows({784: np.ones(10)}))
        cli.sock.close()
    assert len(srv.errors) == 1 and srv.pushes == []


def test_config1_two_workers_one_server(oracle):
    """2 worker processes x 1 server, 1 000 synthetic MNIST lines, batch 100: every
    push the workers sent arrives intact, and the server's shard equals a replay of
    the pushes in the server's arrival order."""
    fmt = loopback.MLR_FORMAT
    shard = OracleShard(oracle, fmt, loopback.shard_range(), 10)
    srv, results = loopback.run({"weights": (shard, fmt)}, n_lines=1000, workers=2, batch_size=100)
    assert [r[0] for r in results] == ["ok", "ok"], results
    assert srv.errors == []
    import hashlib
    sent = sorted(h for r in results for h in r[2])
    got = sorted(hashlib.sha256(d).hexdigest() for _, d in srv.pushes)
    assert len(sent) == 10 and sent == got
    replay = oracle.OracleStore(1, 1, 3, 0, 783, 10)
    for _, d in srv.pushes:
        assert replay.push(d) == 0
    assert replay.write_all() == shard.o.write_all()
    assert np.isfinite(shard.o.data).all() and np.abs(shard.o.data).sum() > 0
