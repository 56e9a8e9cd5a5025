"""GPU: efl.FederalModel's Paillier entry points (efls-train/python/efl/framework/model.py:543-677)
and their learning-rate update of the Paillier kernels (model.py:808-814) over three training steps
of two parties, each its own process, on loopback.

What is checked (in the parent, against float64 arithmetic of the same protocol):
  * step by step, W_recv + w_send moves by exactly -lr * x^T q(dy): the receiver applies
    lr * (dw + nf), the sender lr * (-nf) with the PEER's rate, and the masks cancel
    (q = the reference's decrease_precision fixed-point rounding of dy, paillier_layer.py:123);
  * each forward output equals x @ q(W_recv) + x @ w_send (the encrypted product with the
    receiver's kernel rounded the same way, plus the sender's local share), and the sender's own
    copy of it is masked by the receiver's noise n1;
  * W_recv + w_send tracks plaintext SGD of 0.5 |x W - t|^2 from the same start;
  * neither share alone is the model: the sender's share is non-zero and masked.
Dense and Weight layers both."""
import multiprocessing as mp
import weakref

import numpy as np
import pytest
import torch

from oracle import fxp
from test_communicator import free_port

pytestmark = pytest.mark.gpu

B, F, STEPS, LR = 16, 6, 3, 0.05


def data(kind):
    g = torch.Generator().manual_seed(11)
    units = 4 if kind == "dense" else F
    xs = [torch.randn(B, F, generator=g) for _ in range(STEPS)]
    t = torch.randn(B, units, generator=g)
    return units, xs, t


def party(role, kind, my, peer, q):
    try:
        import efl
        Role = efl.privacy.Role
        units, xs, t = data(kind)
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                             default_timeout_milliseconds=120000, connect_retry_seconds=0.1)
        model = efl.FederalModel(c)
        sender = role == "follower"
        model.create_keypair("kp", Role.SENDER if sender else Role.RECEIVER, n_bytes=64, seed=7)
        model.initialize()
        rec = []
        for step in range(STEPS):
            model.begin_step()
            if sender:
                if kind == "dense":
                    out = model.paillier_sender_dense(xs[step].cuda(), "kp", "l1", LR, units, seed=1)
                else:
                    out = model.paillier_sender_weight(xs[step].cuda(), "kp", "l1", LR, units, seed=1)
                (w, lr), = model.paillier_vars_and_lrs()
                before = w.detach().clone()
                model.minimize(None)                      # no loss of its own: the outputs pull dx
                rec.append((before, w.detach().clone(), out.detach()))
            else:
                if kind == "dense":
                    y = model.paillier_recver_dense(None, "kp", "l1", LR, units, (B, F), seed=2)
                else:
                    gw = torch.Generator().manual_seed(3)
                    y = model.paillier_recver_weight(None, "kp", "l1", LR, units, seed=2,
                                                     kernel_initializer=lambda v: v.copy_(torch.rand(v.shape, generator=gw) - 0.5))
                (W, lr), = model.paillier_vars_and_lrs()
                before = W.detach().clone()
                loss = 0.5 * ((y - t.cuda()) ** 2).sum()
                dy = (y - t.cuda()).detach()
                model.minimize(None, loss)
                assert W.grad is None
                rec.append((before, W.detach().clone(), y.detach(), dy))
            model.end_step()
        assert len(model.paillier_vars_and_lrs()) == 1          # registered once, not once per step
        c.shutdown()
        q.put((role, [tuple(a.cpu().numpy() for a in r) for r in rec], None))
    except BaseException as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((role, None, traceback.format_exc()[-3000:]))


ROT_STEPS, ROT_INTERVAL = 5, 2


def party_rotation(role, kind, my, peer, q):
    """Five dense steps with create_keypair(..., update_step_interval=2): the sender generates a new
    keypair before steps 0, 2 and 4 (PaillierHook.before_run, paillier.py:195-202) and the receiver
    installs it. Records per step: the key's n, device memory around the re-key, the layer values."""
    try:
        import efl
        from efl.privacy import paillier_cipher as pc      # table bytes live outside torch's allocator
        Role = efl.privacy.Role
        g = torch.Generator().manual_seed(12)
        units = 4
        xs = [torch.randn(B, F, generator=g) for _ in range(ROT_STEPS)]
        t = torch.randn(B, units, generator=g)
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                             default_timeout_milliseconds=120000, connect_retry_seconds=0.1)
        model = efl.FederalModel(c)
        sender = role == "follower"
        kp = model.create_keypair("kp", Role.SENDER if sender else Role.RECEIVER, update_step_interval=ROT_INTERVAL,
                                  n_bytes=128, seed=7)
        model.initialize()
        rec = []
        for step in range(ROT_STEPS):
            torch.cuda.synchronize()
            m0 = torch.cuda.memory_allocated() + pc.table_budget()[1]
            old = weakref.ref(kp.key) if step else None
            model.begin_step()                        # re-key on steps 0, 2, 4
            torch.cuda.synchronize()
            m1 = torch.cuda.memory_allocated() + pc.table_budget()[1]
            key_bytes = kp.key.block_bytes
            rekeyed = old is not None and old() is not kp.key
            old_alive = rekeyed and old() is not None
            if sender:
                out = model.paillier_sender_dense(xs[step].cuda(), "kp", "l1", LR, units, seed=1)
                (w, lr), = model.paillier_vars_and_lrs()
                before = w.detach().cpu().clone()
                model.minimize(None)
                vals = (before, w.detach().cpu().clone(), out.detach().cpu())
            else:
                y = model.paillier_recver_dense(None, "kp", "l1", LR, units, (B, F), seed=2)
                (W, lr), = model.paillier_vars_and_lrs()
                before = W.detach().cpu().clone()
                loss = 0.5 * ((y - t.cuda()) ** 2).sum()
                dy = (y - t.cuda()).detach()
                model.minimize(None, loss)
                vals = (before, W.detach().cpu().clone(), y.detach().cpu(), dy.cpu())
                del y, loss, dy
            subs = kp.key.crt_keys() if sender else None
            crt_bytes = sum(s.block_bytes for s in subs) if subs else 0
            model.end_step()
            rec.append(dict(n=kp.key.n, m0=m0, m1=m1, key_bytes=key_bytes, crt_bytes=crt_bytes, rekeyed=rekeyed,
                            old_alive=old_alive,
                            vals=tuple(a.numpy() for a in vals)))
        c.shutdown()
        q.put((role, rec, None))
    except BaseException:  # pragma: no cover - reported to the parent
        import traceback
        q.put((role, None, traceback.format_exc()[-3000:]))


def test_key_rotation_every_two_steps():
    """update_step_interval = 2 over five steps: both parties hold the same n on every step, n
    changes exactly on steps 2 and 4, the layer's values stay right across each switch, and device
    memory after a re-key is back at its level after the previous re-key (the old key block, its
    fixed-base table and the key owner's CRT sub-tables are released)."""
    res = run_parties("dense", target=party_rotation)
    recv, send = res["leader"], res["follower"]
    ns = [r["n"] for r in send]
    assert ns == [r["n"] for r in recv]
    assert ns[0] == ns[1] != ns[2] == ns[3] != ns[4] and ns[0] != ns[4]
    assert [r["rekeyed"] for r in send] == [False, False, True, False, True]
    assert [r["rekeyed"] for r in recv] == [False, False, True, False, True]
    assert not any(r["old_alive"] for r in send + recv)      # nothing holds the replaced KeyBlock
    g = torch.Generator().manual_seed(12)
    xs = [torch.randn(B, F, generator=g).numpy().astype(np.float64) for _ in range(ROT_STEPS)]
    for step in range(ROT_STEPS):
        W0, W1, y, dy = (a.astype(np.float64) for a in recv[step]["vals"])
        w0, w1, out = (a.astype(np.float64) for a in send[step]["vals"])
        x = xs[step]
        assert np.allclose(y, x @ qdp(W0) + x @ w0, rtol=1e-4, atol=1e-4), step
        assert np.allclose((W1 + w1) - (W0 + w0), -LR * x.T @ qdp(dy), rtol=1e-4, atol=2e-5), step
    for side in (send, recv):
        # the fixed-base tables dominate (MiB scale): the receiver's n^2 table, the key owner's two
        # CRT sub-tables (its n^2 table is never walked, so never built)
        key_bytes = side[2]["key_bytes"] + side[2]["crt_bytes"]
        assert key_bytes > 1 << 20
        # right after the re-keys of steps 2 and 4 the same bytes are live: nothing of the old key
        # stays behind (a leak would add at least one key block)
        assert abs(side[4]["m1"] - side[2]["m1"]) < key_bytes // 4, [r["m1"] for r in side]
        # at the start of steps 3 and 4 (before the second re-key) as at step 2: steady state
        assert abs(side[4]["m0"] - side[2]["m0"]) < key_bytes // 4, [r["m0"] for r in side]
    # the key owner's CRT sub-tables are rebuilt for each new key and the old ones released
    assert send[2]["crt_bytes"] > 0 and send[4]["crt_bytes"] == send[2]["crt_bytes"]


def run_parties(kind, target=party):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    procs = [ctx.Process(target=target, args=("leader", kind, pl, pf, q)),
             ctx.Process(target=target, args=("follower", kind, pf, pl, q))]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in procs:
            role, res, err = q.get(timeout=400)
            assert err is None, (role, err)
            results[role] = res
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    return results


def qdp(v):
    """decode(encode(v, decrease_precision=True)): the rounding the protocol applies to W and dy."""
    M, E = fxp.encode(np.ascontiguousarray(v, np.float32), decrease_precision=True)
    return fxp.decode(M, E).astype(np.float64)


@pytest.mark.parametrize("kind", ["dense", "weight"])
def test_federal_model_trains_the_shared_kernel(kind):
    res = run_parties(kind)
    units, xs, t = data(kind)
    t = t.numpy().astype(np.float64)
    recv, send = res["leader"], res["follower"]
    W_plain = recv[0][0].astype(np.float64) + send[0][0].astype(np.float64)
    for step in range(STEPS):
        W0, W1, y, dy = (a.astype(np.float64) for a in recv[step])
        w0, w1, out = (a.astype(np.float64) for a in send[step])
        x = xs[step].numpy().astype(np.float64)
        if kind == "dense":
            want_y = x @ qdp(W0) + x @ w0
            grad = x.T @ qdp(dy)
            plain_grad = x.T @ (x @ W_plain - t)
        else:
            want_y = x * qdp(W0) + x * w0
            grad = (x * qdp(dy)).sum(0)
            plain_grad = (x * (x * W_plain - t)).sum(0)
        assert np.allclose(y, want_y, rtol=1e-4, atol=1e-4), step          # receiver's output
        # the sender only ever sees z + n1 (paillier_layer.py:74-76): the receiver's noise masks it
        assert np.abs(out - want_y).mean() > 0.2, step
        # the masks cancel: the SUM of the two updates is -lr * x^T q(dy)
        assert np.allclose((W1 + w1) - (W0 + w0), -LR * grad, rtol=1e-4, atol=2e-5), step
        # each share moved by much more than the gradient alone (it carries the mask nf ~ N(10 s, 1))
        assert np.abs(w1 - w0).mean() > 0.1 * LR, step
        W_plain = W_plain - LR * plain_grad
        # the model the two parties hold together follows plaintext SGD (fixed-point rounding of
        # the encrypted product and of dy only)
        assert np.allclose(W1 + w1, W_plain, rtol=2e-2, atol=2e-3), step
        if step + 1 < STEPS:                       # next step starts from this step's result
            assert np.array_equal(recv[step + 1][0], recv[step][1])
            assert np.array_equal(send[step + 1][0], send[step][1])
    assert np.abs(send[-1][1]).mean() > 0.1 * LR              # the sender's share is not zero
