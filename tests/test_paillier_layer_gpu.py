"""GPU: the two-party Paillier Dense / Weight layers (paillier_layer.py protocol) end to end over
two communicators on loopback, with the key exchanged by efl.paillier.Hook. Checks the plaintext
meaning of every exchanged quantity against torch fp32 (tolerance from the reference's own
decrease_precision fixed-point encoding of W and dy: 13 dropped mantissa bits, rtol 1e-2)."""
import threading

import pytest
import torch

from test_communicator import free_port

pytestmark = pytest.mark.gpu


def run_pair(sender_fn, receiver_fn):
    import efl
    pl, pf = free_port(), free_port()
    comms = {}
    results, errs = {}, []

    def party(role, fn, my, peer):
        try:
            c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                                 default_timeout_milliseconds=120000, connect_retry_seconds=0.1)
            c.initialize()
            comms[role] = c
            results[role] = fn(c)
        except Exception as e:  # pragma: no cover
            errs.append((role, e))
            raise
    ts = [threading.Thread(target=party, args=("leader", receiver_fn, pl, pf)),
          threading.Thread(target=party, args=("follower", sender_fn, pf, pl))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    for c in comms.values():
        c.shutdown()
    assert not errs, errs
    return results


@pytest.mark.parametrize("kind", ["dense", "weight"])
def test_paillier_layer_two_party(kind):
    import efl
    g = torch.Generator().manual_seed(0)
    B, F = 8, 6
    units = 3 if kind == "dense" else F
    x = torch.randn(B, F, generator=g).cuda()
    dy_r = torch.randn(B, units, generator=g).cuda()
    dy_s = torch.randn(B, units, generator=g).cuda()
    Role = efl.privacy.Role

    def sender(c):
        kp = efl.paillier.Keypair()
        efl.paillier.Hook(kp, c, Role.SENDER, "k", n_bytes=64).after_create_session()
        xi = x.clone().requires_grad_(True)
        if kind == "dense":
            out, w = efl.paillier.sender.dense(xi, kp, c, "l1", units, seed=1)
        else:
            out, w = efl.paillier.sender.weight(xi, kp, c, "l1", units, seed=1)
        out.backward(dy_s)
        return out.detach(), xi.grad, w.grad

    def receiver(c):
        kp = efl.paillier.Keypair()
        efl.paillier.Hook(kp, c, Role.RECEIVER, "k", n_bytes=64).after_create_session()
        if kind == "dense":
            y, w = efl.paillier.recver.dense(None, kp, c, "l1", (B, F), units, seed=2)
        else:
            y, w = efl.paillier.recver.weight(None, kp, c, "l1", units, seed=2)
        y.backward(dy_r)
        return y.detach(), w.detach(), w.grad

    res = run_pair(sender, receiver)
    y, W, dW = res["leader"]
    out, dx, dws = res["follower"]
    if kind == "dense":
        want_y, want_dw, want_dx = x @ W, x.t() @ dy_r, dy_r @ W.t()
    else:
        want_y, want_dw, want_dx = x * W, (x * dy_r).sum(0), dy_r * W
    assert torch.allclose(y.cuda(), want_y, rtol=1e-2, atol=1e-2)
    assert torch.allclose(dW.cuda(), want_dw, rtol=1e-2, atol=1e-2)
    assert torch.allclose(dx.cuda(), want_dx, rtol=1e-2, atol=1e-2)
    assert dws is not None and torch.isfinite(dws).all()      # -nf noise for the sender's zero kernel
