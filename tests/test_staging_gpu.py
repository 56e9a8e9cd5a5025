"""GPU: efl.staging, the pinned staging buffer the hex text of large messages crosses PCIe through
(received text -> HBM for efl_hex_parse; device hex text -> the outgoing request bytes). Bytes
must arrive unchanged at every size around the staging threshold, with the buffer reused, grown and
shared between threads."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def staging():
    import efl
    efl.lib.require_gpu()
    from efl import staging
    return staging


@pytest.mark.parametrize("n", [1, 4096, (1 << 20) - 1, 1 << 20, (1 << 20) + 7, 51 << 20, 3 << 20])
def test_round_trip(staging, n):
    rng = np.random.default_rng(n)
    host = rng.integers(0, 256, n, dtype=np.uint8)
    dev = staging.to_device(host, "cuda")
    assert dev.device.type == "cuda" and dev.dtype == torch.uint8 and dev.numel() == n
    back = np.empty(n, np.uint8)
    staging.to_host_into(back, dev)
    assert np.array_equal(back, host)
    offs = np.cumsum(rng.integers(0, 600, 300000)).astype(np.int64)      # an int64 array, 2.4 MB
    d = staging.to_device(offs, "cuda")
    assert d.dtype == torch.int64 and torch.equal(d.cpu(), torch.from_numpy(offs))


def test_threads_share_the_buffer(staging):
    errors = []

    def work(seed):
        rng = np.random.default_rng(seed)
        for _ in range(5):
            host = rng.integers(0, 256, int(rng.integers(1 << 20, 8 << 20)), dtype=np.uint8)
            dev = staging.to_device(host, "cuda")
            back = np.empty_like(host)
            staging.to_host_into(back, dev)
            if not np.array_equal(back, host):
                errors.append(seed)
    ts = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors
