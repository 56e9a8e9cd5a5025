"""GPU: the secret-sharing protocol of efls-train/python/efl/privacy/secret_sharing.py end to end,
two parties in two processes over efl.Communicator on loopback (one GPU shared).

Checks the plaintext meaning of every exchange against float64 torch: modes A/B (z_A + z_B = a @ b),
mode C forward (the parties' z sum to (a_0 + a_1) @ (b_0 + b_1)) and its backward with and
without combine_gradients (da_0 + da_1 = dY @ B^T, db_0 + db_1 = A^T @ dY with A, B, dY the
summed shares), SecretSharingDense with noise_divisor, and share/reveal with their gradients.
Tolerance: fp32 matmuls of masked shares whose noise is up to |x|, rtol 1e-4 / atol 1e-4."""
import multiprocessing as mp

import pytest
import torch

from test_communicator import free_port

pytestmark = pytest.mark.gpu

R, C, N = 8, 6, 4


def inputs(p):
    g = torch.Generator().manual_seed(10 + p)
    return (torch.randn(R, C, generator=g), torch.randn(C, N, generator=g), torch.randn(R, N, generator=g))


def party(role, my, peer, q):
    try:
        import efl
        ss = efl.secret_sharing
        Mode = ss.matmul.Mode
        p = 0 if role == "leader" else 1
        ss.set_seed(1000 + p)
        a, b, dy = inputs(p)
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                             default_timeout_milliseconds=120000, connect_retry_seconds=0.1)
        c.initialize()
        out = {}
        # modes A / B: the leader holds a, the follower holds b
        if p == 0:
            out["zab"] = ss.matmul(a.cuda(), (C, N), c, "ab", Mode.A)
        else:
            out["zab"] = ss.matmul((R, C), b.cuda(), c, "ab", Mode.B)
        # mode C forward + backward, both gradient layouts
        for comb in (False, True):
            ai = a.cuda().requires_grad_(True)
            bi = b.cuda().requires_grad_(True)
            z = ss.matmul(ai, bi, c, f"mc{int(comb)}", Mode.C, combine_gradients=comb)
            z.backward(dy.cuda())
            out[f"z{int(comb)}"], out[f"da{int(comb)}"], out[f"db{int(comb)}"] = z.detach(), ai.grad, bi.grad
        # mode A has no gradient (the reference raises)
        if p == 0:
            ai = a.cuda().requires_grad_(True)
            z = ss.matmul(ai, (C, N), c, "ag", Mode.A)
            try:
                z.sum().backward()
                out["a_grad_raised"] = torch.tensor(0)
            except ValueError:
                out["a_grad_raised"] = torch.tensor(1)
        else:
            ss.matmul((R, C), b.cuda(), c, "ag", Mode.B)
        # SecretSharingDense with weight noise (the kernel shares are averaged with the peer's)
        gk = torch.Generator().manual_seed(50 + p)
        layer = ss.Dense(c, "dense", N, noise_divisor=2.0,
                         kernel_initializer=lambda t: t.copy_(torch.randn(t.shape, generator=gk)))
        xi = a.cuda().requires_grad_(True)
        y = layer(xi)
        y.backward(dy.cuda())
        out["dense_y"], out["dense_k"], out["dense_dx"] = y.detach(), layer.kernel.detach(), xi.grad
        out["dense_dk"] = layer.kernel.grad
        # share / reveal: the follower shares a (noise to the leader), the follower reveals its kept
        # share to the leader. Backward: the leader re-shares its gradient (reveal, RECEIVER) and
        # sends its noise share's gradient as sh_grad, which the follower's share() adds.
        if p == 1:
            xi = a.cuda().requires_grad_(True)
            kept = ss.share(xi, c, "sh")
            r = ss.reveal(kept, c, "rv", efl.privacy.Role.SENDER)
            r.backward(torch.zeros_like(r))
            out["share_kept"], out["share_dx"] = kept.detach(), xi.grad
        else:
            noise = c.recv("sh", shape=(R, C)).cuda().requires_grad_(True)
            r = ss.reveal(noise, c, "rv", efl.privacy.Role.RECEIVER)
            r.backward(torch.ones(R, C, device="cuda"))
            c.send("sh_grad", noise.grad).result()
            out["reveal"], out["reveal_dnoise"] = r.detach(), noise.grad
        c.shutdown()
        q.put((role, {k: v.cpu().numpy() for k, v in out.items()}, None))
    except BaseException as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((role, None, traceback.format_exc()))


def test_secret_sharing_two_party():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    procs = [ctx.Process(target=party, args=("leader", pl, pf, q)),
             ctx.Process(target=party, args=("follower", pf, pl, q))]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            role, r, err = q.get(timeout=300)
            assert err is None, (role, err)
            res[role] = {k: torch.from_numpy(v).double() for k, v in r.items()}
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    L, F = res["leader"], res["follower"]
    (a0, b0, dy0), (a1, b1, dy1) = [tuple(t.double() for t in inputs(p)) for p in (0, 1)]
    tol = dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(L["zab"] + F["zab"], a0 @ b1, **tol)
    A, B, DY = a0 + a1, b0 + b1, dy0 + dy1
    for comb in (0, 1):
        torch.testing.assert_close(L[f"z{comb}"] + F[f"z{comb}"], A @ B, **tol)
        torch.testing.assert_close(L[f"da{comb}"] + F[f"da{comb}"], DY @ B.t(), **tol)
        torch.testing.assert_close(L[f"db{comb}"] + F[f"db{comb}"], A.t() @ DY, **tol)
    assert int(L["a_grad_raised"]) == 1
    # Dense: side p multiplies by (k_p + n_p + k_q - n_q) / 2; the two effective kernels sum to
    # k0 + k1, so the outputs sum to A @ (k0 + k1), as with the reference's averaging (:137-143)
    K = L["dense_k"] + F["dense_k"]
    torch.testing.assert_close(L["dense_y"] + F["dense_y"], A @ K, **tol)
    torch.testing.assert_close(L["dense_dx"] + F["dense_dx"], DY @ K.t(), **tol)
    # share / reveal: the revealed sum is the follower's a; its kept share is masked
    torch.testing.assert_close(L["reveal"], a1, **tol)
    assert (F["share_kept"] - a1).abs().max() > 1e-3
    # gradients: the leader keeps 1 - a' (masked), the follower's input gradient is a' + (1 - a') = 1
    assert (L["reveal_dnoise"] - 1).abs().max() > 1e-3
    torch.testing.assert_close(F["share_dx"], torch.ones(R, C, dtype=torch.float64), **tol)
