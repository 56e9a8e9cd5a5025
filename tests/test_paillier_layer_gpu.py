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
# the paillier_mnist example's dense layer: batch 256, 28 x 14 features, 128 units, 1024-bit key
# (efls-train/python/efl/example/paillier_mnist/follower_dense.py:23,39, leader_dense.py:44)
EXAMPLE = (256, 392, 128, 128)


def data(kind, B=B, F=F, units=None):
    g = torch.Generator().manual_seed(0)
    if units is None:
        units = 3 if kind == "dense" else F
    x = torch.randn(B, F, generator=g)
    dy_r = torch.randn(B, units, generator=g)
    dy_s = torch.randn(B, units, generator=g)
    return units, x, dy_r, dy_s


def party(role, kind, my, peer, q, shape=(B, F, None, 64)):
    try:
        import efl
        Role = efl.privacy.Role
        B, F, units, n_bytes = shape
        units, x, dy_r, dy_s = data(kind, B, F, units)
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                             default_timeout_milliseconds=120000, connect_retry_seconds=0.1)
        c.initialize()
        kp = efl.paillier.Keypair()
        if role == "follower":   # sender: owns the key, holds x
            efl.paillier.Hook(kp, c, Role.SENDER, "k", n_bytes=n_bytes).after_create_session()
            xi = x.cuda().requires_grad_(True)
            fn = efl.paillier.sender.dense if kind == "dense" else efl.paillier.sender.weight
            out, w = fn(xi, kp, c, "l1", units, seed=1)
            out.backward(dy_s.cuda())
            res = (out.detach(), xi.grad, w.grad)
        else:                    # receiver: holds W
            efl.paillier.Hook(kp, c, Role.RECEIVER, "k", n_bytes=n_bytes).after_create_session()
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


def run_two_parties(kind, shape=(B, F, None, 64)):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    procs = [ctx.Process(target=party, args=("leader", kind, pl, pf, q, shape)),
             ctx.Process(target=party, args=("follower", kind, pf, pl, q, shape))]
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
    return results


@pytest.mark.parametrize("kind", ["dense", "weight"])
def test_paillier_layer_two_party(kind):
    results = run_two_parties(kind)
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


def test_paillier_dense_example_shape():
    """The paillier_mnist example's dense layer at its own shape and key, checked against what the
    protocol computes exactly rather than against fp32 with a loose tolerance. Everything in between
    is integer arithmetic on fixed-point mantissas (encrypted sums, shifts, masks), so the layer's
    results are the exact products of the EXACT encodings, decrease_precision quantisation included,
    up to the float32 decodes and the float32 removal of the masks:
      y       = x @ Wq            Wq  = decode(encode(W,  decrease_precision)) (paillier_layer.py:136)
      dW+dw_s = x^T @ dyq         dyq = decode(encode(dy, decrease_precision)) (:147-150)
      dx      = fl32(dy @ W^T)    (the receiver's plaintext term, :158; the sender's kernel is 0)
    The oracle gives Wq and dyq; the references are float64. Tolerances: a few float32 ulp of the
    masked values (|n1|, |n2| ~ N(0, 1), |nf| ~ 10 + N(0, 1)), 1000x tighter than the small-shape
    test's 1e-2."""
    import numpy as np
    from oracle import fxp
    Bx, Fx, units, n_bytes = EXAMPLE
    results = run_two_parties("dense", EXAMPLE)
    y, W, dW = results["leader"]
    out, dx, dws = results["follower"]
    assert y.shape == (Bx, units) and dx.shape == (Bx, Fx)
    _, x, dy_r, _ = data("dense", Bx, Fx, units)

    def q(t):
        M, E = fxp.encode(t.numpy().astype(np.float32), decrease_precision=True)
        return fxp.decode(M, E).astype(np.float64)

    x64, W64, dy64 = x.double().numpy(), W.double().numpy(), dy_r.double().numpy()
    want_y = x64 @ q(W)
    want_dw = x64.T @ q(dy_r)
    want_dx = dy64 @ W64.T
    ulp = 2.0 ** -23
    err_y = np.abs(y.double().numpy() - want_y)
    assert (err_y <= 8 * ulp * (np.abs(want_y) + 8)).all(), err_y.max()
    err_dw = np.abs((dW + dws).double().numpy() - want_dw)
    assert (err_dw <= 8 * ulp * (np.abs(want_dw) + 16)).all(), err_dw.max()
    # the receiver's share is masked: nf = N(0, 1) + 10 sigmoid(sum x), E|nf| >= E|N(0, 1)| = 0.80
    assert np.abs(dW.double().numpy() - want_dw).mean() > 0.5
    err_dx = np.abs(dx.double().numpy() - want_dx)
    assert (err_dx <= 1e-5 + 1e-5 * np.abs(want_dx)).all(), err_dx.max()
    # the quantisation is real: W itself would miss y by far more than the tolerance above
    assert np.abs(x64 @ W64 - want_y).max() > 1e-4


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
