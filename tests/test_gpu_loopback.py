"""Config-1 plumbing with the GPU store behind the server: 2 worker processes x
1 server over loopback TCP (reference framing), MNIST-shaped MLR pushes of
DoubleMatrix(784, 10) rows into an HBM-resident DataStore through the C-ABI.
The final shard must equal, bit for bit, a CPU-oracle replay of the pushes the
server received in arrival order; a whole-shard fetch over the wire must equal
the oracle's fetch bytes."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def test_config1_gpu_store_two_workers(oracle):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distml_amd import DataStore, loopback, psnet
    from distml_amd.datadesc import KeyRange

    fmt = loopback.MLR_FORMAT
    store = DataStore(fmt, loopback.shard_range(), loopback.OUTPUT_DIM)
    store.zero()
    srv, results = loopback.run({"weights": (store, fmt)}, n_lines=1000, workers=2, batch_size=100)
    assert [r[0] for r in results] == ["ok", "ok"], results
    assert srv.errors == []
    sent = sorted(h for r in results for h in r[2])
    assert len(sent) == 10 and sent == sorted(hashlib.sha256(d).hexdigest() for _, d in srv.pushes)

    replay = oracle.OracleStore(1, 1, 3, 0, 783, 10)
    for _, d in srv.pushes:
        assert replay.push(d) == 0
    vals = store.values()
    assert vals.dtype == np.float64 and vals.shape == replay.data.shape
    assert vals.tobytes() == replay.data.tobytes()

    # the whole shard back over the wire (FetchRequest with KeyRange rows)
    with psnet.PSServer({"weights": (store, fmt)}) as srv2:
        cli = psnet.PSClient(srv2.address)
        got = cli.fetch("weights", fmt, KeyRange(0, 783))
        cli.close()
    assert got == replay.fetch(np.arange(784))
    store.close()
