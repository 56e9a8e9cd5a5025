"""CPU: the Stage-H communicator (gRPC TrainerService over loopback, 127.0.0.1).

* unit behaviour with two in-process communicators (threads): rendezvous by name + step, the send
  acknowledgement after the peer's recv, DataLoss on a step mismatch, DeadlineExceeded, strict
  names -> NotFound, string (HexTensor) payloads;
* BASELINE config 1 as two processes: the follower fixed-point-encodes a 1 MiB fp32 tensor and sends
  mantissa + exponent through the pre-send hook, the leader receives and decodes through the
  post-recv hook, comparing bits with the expected per-quirk output. No GPU: the hook's codec is the
  CPU oracle (injected; the product hook defaults to the libefl_hip.so ops).
"""
import multiprocessing as mp
import os
import socket
import threading

import numpy as np
import pytest
import torch

import efl
from conftest import GOLDEN


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pair(**kw):
    pl, pf = free_port(), free_port()
    leader = efl.Communicator("leader", 0, 1, f"127.0.0.1:{pf}", f"127.0.0.1:{pl}",
                              connect_retry_seconds=0.1, **kw)
    follower = efl.Communicator("follower", 0, 1, f"127.0.0.1:{pl}", f"127.0.0.1:{pf}",
                                connect_retry_seconds=0.1, **kw)
    t = threading.Thread(target=leader.initialize)
    t.start()
    follower.initialize()
    t.join()
    return leader, follower


@pytest.fixture
def comms():
    leader, follower = pair(default_timeout_milliseconds=5000)
    yield leader, follower
    leader.shutdown()
    follower.shutdown()


def test_send_recv_roundtrip(comms):
    leader, follower = comms
    x = torch.randn(17, 5)
    h = follower.send("act", x)
    y = leader.recv("act", shape=(17, 5))
    h.result(timeout=5)
    assert torch.equal(x, y)
    i = torch.arange(-6, 6, dtype=torch.int64).reshape(3, 4)
    h = leader.send("grad", i)
    assert torch.equal(follower.recv("grad", dtype=torch.int64), i)
    h.result(timeout=5)


def test_readonly_raw_recv_is_a_view(comms):
    """A hook that only reads the payload (FixedPointHook copying it to the GPU) gets a view of the
    received message bytes; a plain recv gets its own copy."""
    from efl.framework import wire
    leader, follower = comms
    m = torch.arange(1000, dtype=torch.int64) * 7
    h = follower.send("m", m)
    assert torch.equal(leader._recv_raw("m", readonly=True), m)
    h.result(timeout=5)
    h = follower.send("m", m)
    assert torch.equal(leader._recv_raw("m"), m)
    h.result(timeout=5)
    payload = m.numpy().tobytes()                         # immutable, like gRPC's request bytes
    msg = wire.TensorMsg(wire.DT_INT64, (1000,), memoryview(payload), [])
    base = np.frombuffer(payload, dtype=np.int64).ctypes.data
    view = efl.Communicator._materialize(msg, None, readonly=True)
    copy = efl.Communicator._materialize(msg, None)
    assert view.data_ptr() == base and copy.data_ptr() != base
    assert torch.equal(view, m) and torch.equal(copy, m)


def test_channel_of_is_stable_and_splits_pairs():
    from efl.framework.communicator import channel_of
    for n in ("act", "grad/0", "x_mantissa", "emb"):
        assert channel_of(n, 2) == channel_of(n, 2) and channel_of(n, 1) == 0
    for base in ("act", "dense_1/out", "y"):
        a, b = channel_of(base + "_mantissa", 2), channel_of(base + "_exponent", 2)
        assert {a, b} == {0, 1}


def test_same_name_back_to_back_keeps_order():
    """Several sends of one name in one step, over two connections: the receiver gets them in send
    order (one name always travels on one channel)."""
    leader, follower = pair(default_timeout_milliseconds=5000, channels=2)
    try:
        big = [torch.full((1 << 20,), float(i)) for i in range(4)]
        hs = [follower.send("dup", t) for t in (big[0], torch.ones(3), big[1], torch.full((5,), 2.0))]
        got = [leader.recv("dup") for _ in range(4)]
        for h in hs:
            h.result(timeout=5)
        assert torch.equal(got[0], big[0]) and torch.equal(got[1], torch.ones(3))
        assert torch.equal(got[2], big[1]) and torch.equal(got[3], torch.full((5,), 2.0))
    finally:
        leader.shutdown()
        follower.shutdown()


def test_send_completes_only_after_peer_recv(comms):
    leader, follower = comms
    h = follower.send("late", torch.ones(3))
    threading.Event().wait(0.3)
    assert not h.done()                       # the RPC is held open until the leader's recv
    leader.recv("late")
    h.result(timeout=5)
    assert h.done()


def test_steps_and_dataloss(comms):
    leader, follower = comms
    follower.add_step()                       # follower at step 1, leader at step 0
    h = follower.send("s", torch.zeros(2))
    with pytest.raises(efl.errors.DataLossError, match="expects step 0, but given step 1"):
        leader.recv("s")
    with pytest.raises(efl.errors.DataLossError):
        h.result(timeout=5)
    leader.add_step()
    h = follower.send("s", torch.full((2,), 3.0))
    assert torch.equal(leader.recv("s"), torch.full((2,), 3.0))
    h.result(timeout=5)


def test_recv_timeout():
    leader, follower = pair(default_timeout_milliseconds=300)
    try:
        with pytest.raises(efl.errors.DeadlineExceededError, match="Timeout"):
            leader.recv("never")
    finally:
        leader.shutdown()
        follower.shutdown()


def test_strict_names_not_found():
    leader, follower = pair(default_timeout_milliseconds=3000, strict_names=True)
    try:
        with pytest.raises(efl.errors.NotFoundError, match="not registed"):
            follower.send("unknown", torch.ones(1)).result(timeout=5)
    finally:
        leader.shutdown()
        follower.shutdown()


def test_hex_tensor_payload(comms):
    leader, follower = comms
    hx = efl.HexTensor.from_ints([0, -1, 2**1024 + 5, 255] * 3, shape=(3, 4))
    h = follower.send("ct", hx)
    got = leader.recv("ct", dtype="string")
    h.result(timeout=5)
    assert got == hx and got.to_ints()[2] == 2**1024 + 5


def test_not_connected():
    c = efl.Communicator("leader", 0, 1, "127.0.0.1:1", "127.0.0.1:0")
    with pytest.raises(efl.errors.FailedPreconditionError):
        c.send("x", torch.ones(1))
    with pytest.raises(ValueError):
        efl.Communicator("boss", 0, 1, "a", "b")


# ------------------------------------------------------------------ config 1, two processes

def _oracle_codec():
    from oracle import fxp

    def enc(t, decrease_precision=False):
        M, E = fxp.encode(t.numpy(), decrease_precision)
        return torch.from_numpy(M), torch.from_numpy(E)

    def dec(M, E, dtype=torch.float32):
        return torch.from_numpy(fxp.decode(M.numpy(), E.numpy(), np.float32))
    return enc, dec


def config1_tensor():
    special = np.load(os.path.join(GOLDEN, "fxp_golden.npz"))["f32_bits"][:4096].view(np.float32)
    x = torch.randn(512, 512, generator=torch.Generator().manual_seed(0))
    x.view(-1)[:4096] = torch.from_numpy(special.copy())
    return x


def _party(role, my_port, peer_port, q):
    try:
        enc, dec = _oracle_codec()
        hook = efl.privacy.FixedPointHook(encode=enc, decode=dec)
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer_port}", f"127.0.0.1:{my_port}",
                             default_timeout_milliseconds=60000, hooks=[hook], connect_retry_seconds=0.2)
        c.initialize()
        x = config1_tensor()
        if role == "follower":
            c.send("t_[x]", x).result(timeout=60)
            q.put(("follower", True))
        else:
            y = c.recv("t_[x]", shape=(512, 512))
            from oracle import fxp
            M, E = fxp.encode(x.numpy())
            want = fxp.decode(M, E).view(np.uint32)
            same = np.array_equal(y.numpy().view(np.uint32), want)
            changed = int((y.numpy().view(np.uint32) != x.numpy().view(np.uint32)).sum())
            q.put(("leader", same, changed))
        c.shutdown()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((role, "error", repr(e)))


def test_config1_two_process_loopback():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    procs = [ctx.Process(target=_party, args=("leader", pl, pf, q)),
             ctx.Process(target=_party, args=("follower", pf, pl, q))]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=30)
    assert res["follower"] == (True,), res
    same, changed = res["leader"]
    assert same, res
    # only the quirk classes of the special-value prefix change (zeros, denormals, 2^23 band)
    assert 0 < changed < 4096
