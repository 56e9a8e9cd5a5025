"""GPU: the two-party Paillier Dense / Weight layers (paillier_layer.py protocol) end to end over
two communicators on loopback, with the key exchanged by efl.paillier.Hook. Checks the plaintext
meaning of every exchanged quantity against torch fp32 (tolerance from the reference's own
decrease_precision fixed-point encoding of W and dy: 13 dropped mantissa bits, rtol 1e-2).

Each party runs in its own process, as in a federated deployment: the protocol blocks inside
backward() on messages the peer sends from ITS backward(), and torch runs every backward() of a
process on one autograd thread per device, so two parties sharing a process would wait on each
other forever."""
import multiprocessing as mp

import pytest
import torch

from test_communicator import free_port

pytestmark = pytest.mark.gpu

B, F = 8, 6


def data(kind):
    g = torch.Generator().manual_seed(0)
    units = 3 if kind == "dense" else F
    x = torch.randn(B, F, generator=g)
    dy_r = torch.randn(B, units, generator=g)
    dy_s = torch.randn(B, units, generator=g)
    return units, x, dy_r, dy_s


def party(role, kind, my, peer, q):
    try:
        import efl
        Role = efl.privacy.Role
        units, x, dy_r, dy_s = data(kind)
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                             default_timeout_milliseconds=120000, connect_retry_seconds=0.1)
        c.initialize()
        kp = efl.paillier.Keypair()
        if role == "follower":   # sender: owns the key, holds x
            efl.paillier.Hook(kp, c, Role.SENDER, "k", n_bytes=64).after_create_session()
            xi = x.cuda().requires_grad_(True)
            fn = efl.paillier.sender.dense if kind == "dense" else efl.paillier.sender.weight
            out, w = fn(xi, kp, c, "l1", units, seed=1)
            out.backward(dy_s.cuda())
            res = (out.detach(), xi.grad, w.grad)
        else:                    # receiver: holds W
            efl.paillier.Hook(kp, c, Role.RECEIVER, "k", n_bytes=64).after_create_session()
            if kind == "dense":
                y, w = efl.paillier.recver.dense(None, kp, c, "l1", (B, F), units, seed=2)
            else:
                gw = torch.Generator().manual_seed(3)
                y, w = efl.paillier.recver.weight(None, kp, c, "l1", units, seed=2,
                                                  kernel_initializer=lambda t: t.copy_(torch.rand(t.shape, generator=gw) - 0.5))
            y.backward(dy_r.cuda())
            res = (y.detach(), w.detach(), w.grad)
        c.shutdown()
        # numpy pickles by value (torch CPU tensors would travel as shared-memory handles that
        # die with this process)
        q.put((role, tuple(t.cpu().numpy() for t in res), None))
    except BaseException as e:  # pragma: no cover - reported to the parent
        q.put((role, None, repr(e)))


@pytest.mark.parametrize("kind", ["dense", "weight"])
def test_paillier_layer_two_party(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    procs = [ctx.Process(target=party, args=("leader", kind, pl, pf, q)),
             ctx.Process(target=party, args=("follower", kind, pf, pl, q))]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in procs:
            role, res, err = q.get(timeout=400)
            assert err is None, (role, err)
            results[role] = tuple(torch.from_numpy(a) for a in res)
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    y, W, dW = results["leader"]
    out, dx, dws = results["follower"]
    units, x, dy_r, _ = data(kind)
    if kind == "dense":
        want_y, want_dw, want_dx = x @ W, x.t() @ dy_r, dy_r @ W.t()
    else:
        want_y, want_dw, want_dx = x * W, (x * dy_r).sum(0), dy_r * W
    assert torch.allclose(y, want_y, rtol=1e-2, atol=1e-2)
    # the sender masks the revealed gradient with nf ~ N(10 sigmoid(sum x), 1) and keeps -nf for
    # its own zero kernel (reference paillier_layer.py:41-54): only the sum is dL/dW
    assert torch.allclose(dW + dws, want_dw, rtol=1e-2, atol=1e-2)
    assert (dW - want_dw).abs().mean() > 1.0          # the receiver's share really is masked
    assert torch.allclose(dx, want_dx, rtol=1e-2, atol=1e-2)


def party_two_steps(role, my, peer, q):
    """the receiver's dense with its own plaintext features, two training steps. The
    functional form must find its layers again on the second call (weights persist and train)."""
    try:
        import efl
        from efl.privacy import paillier_layer as pl
        Role = efl.privacy.Role
        units, x, dy_r, dy_s = data("dense")
        xr = torch.randn(B, 4, generator=torch.Generator().manual_seed(9))
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                             default_timeout_milliseconds=120000, connect_retry_seconds=0.1)
        c.initialize()
        kp = efl.paillier.Keypair()
        res = []
        if role == "follower":
            efl.paillier.Hook(kp, c, Role.SENDER, "k", n_bytes=64).after_create_session()
            for _ in range(2):
                xi = x.cuda().requires_grad_(True)
                out, w = efl.paillier.sender.dense(xi, kp, c, "l1", units, seed=1)
                out.backward(dy_s.cuda())
                c.add_step()
        else:
            efl.paillier.Hook(kp, c, Role.RECEIVER, "k", n_bytes=64).after_create_session()
            lins = []
            for _ in range(2):
                y, w = efl.paillier.recver.dense(xr.cuda(), kp, c, "l1", (B, F), units, seed=2)
                y.backward(dy_r.cuda())
                lin = pl.cached_layers(c)[("recver.dense.plain", "l1", None)]
                lins.append(lin)
                res.append((y.detach(), w.detach(), lin.weight.detach().clone(), lin.bias.detach().clone()))
                with torch.no_grad():           # one SGD step on the plaintext Dense only
                    for p in lin.parameters():
                        p -= 0.5 * p.grad
                        p.grad = None
                c.add_step()
            assert lins[0] is lins[1]
            assert len(pl.cached_layers(c)) == 2
        c.shutdown()
        q.put((role, [tuple(t.cpu().numpy() for t in r) for r in res], None))
    except BaseException as e:  # pragma: no cover - reported to the parent
        q.put((role, None, repr(e)))


def test_recver_dense_with_inputs_two_steps():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    procs = [ctx.Process(target=party_two_steps, args=("leader", pl, pf, q)),
             ctx.Process(target=party_two_steps, args=("follower", pf, pl, q))]
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
    units, x, dy_r, _ = data("dense")
    xr = torch.randn(B, 4, generator=torch.Generator().manual_seed(9))
    steps = [tuple(torch.from_numpy(a) for a in r) for r in results["leader"]]
    for y, W, Wl, bl in steps:
        assert torch.allclose(y, x @ W + xr @ Wl.t() + bl, rtol=1e-2, atol=1e-2)
    (_, W0, Wl0, b0), (_, W1, Wl1, b1) = steps
    assert torch.equal(W0, W1)                       # the Paillier kernel is the same parameter
    # the SGD step after step 1 is what step 2's plaintext Dense used
    g_w = dy_r.t() @ xr
    assert torch.allclose(Wl1, Wl0 - 0.5 * g_w, rtol=1e-4, atol=1e-5)
    assert torch.allclose(b1, b0 - 0.5 * dy_r.sum(0), rtol=1e-4, atol=1e-5)
