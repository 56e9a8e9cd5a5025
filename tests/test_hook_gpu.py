"""GPU: the communicator's pre-send / post-recv hook with the real libefl_hip.so codec."""
import threading

import numpy as np
import pytest
import torch

from oracle import fxp
from test_communicator import free_port

pytestmark = pytest.mark.gpu


def test_fixed_point_hook_over_grpc():
    import efl
    pl, pf = free_port(), free_port()
    hl, hf = efl.privacy.FixedPointHook(return_device="cuda"), efl.privacy.FixedPointHook()
    leader = efl.Communicator("leader", 0, 1, f"127.0.0.1:{pf}", f"127.0.0.1:{pl}", hooks=[hl],
                              default_timeout_milliseconds=20000, connect_retry_seconds=0.1)
    follower = efl.Communicator("follower", 0, 1, f"127.0.0.1:{pl}", f"127.0.0.1:{pf}", hooks=[hf],
                                default_timeout_milliseconds=20000, connect_retry_seconds=0.1)
    t = threading.Thread(target=leader.initialize)
    t.start()
    follower.initialize()
    t.join()
    try:
        x = torch.randn(300, 77, generator=torch.Generator().manual_seed(2))
        x[0, :3] = torch.tensor([0.0, 1e-42, -8388608.0])
        h = follower.send("p_[x]", x.cuda())          # device tensor in, wire = M + E
        y = leader.recv("p_[x]", shape=(300, 77))      # decoded on the leader's GPU
        h.result(timeout=20)
        assert y.is_cuda
        M, E = fxp.encode(x.numpy())
        assert np.array_equal(y.cpu().numpy().view(np.uint32), fxp.decode(M, E).view(np.uint32))
        # non-float tensors pass through the hook untouched
        h = follower.send("ids", torch.arange(5))
        assert torch.equal(leader.recv("ids", dtype=torch.int64), torch.arange(5))
        h.result(timeout=20)
    finally:
        leader.shutdown()
        follower.shutdown()


def test_pipeline_slots_never_join_autograd():
    """a host activation that requires grad goes through the pinned pipeline (as
    FixedPointHook.pre_send sends it) twice; the cached device slots and pinned staging chunks stay
    plain buffers (no grad_fn chain across steps), and the bits equal the oracle."""
    import efl
    from efl.framework.host_pipeline import PinnedCodecPipeline
    pipe = PinnedCodecPipeline(chunk_elems=1 << 12)
    x = torch.randn(3 * 4096 + 17, generator=torch.Generator().manual_seed(5)).requires_grad_(True)
    for _ in range(2):
        M, E = pipe.encode(x)                                  # pageable source: staged chunks
        Mp, Ep = pipe.encode(x.detach().pin_memory())          # pinned source
        y = pipe.decode(M, E)
    for t in list(pipe._slots.values()) + list(pipe._stage.values()):
        assert not t.requires_grad and t.grad_fn is None
    assert not M.requires_grad and not y.requires_grad
    Mo, Eo = fxp.encode(x.detach().numpy())
    assert np.array_equal(M.numpy(), Mo) and np.array_equal(E.numpy(), Eo)
    assert np.array_equal(Mp.numpy(), Mo) and np.array_equal(Ep.numpy(), Eo)
    assert np.array_equal(y.numpy().view(np.uint32), fxp.decode(Mo, Eo).view(np.uint32))
    assert efl.lib.flush_denormal() in (True, False)
