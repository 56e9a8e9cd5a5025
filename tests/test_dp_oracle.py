"""CPU: the DP-SGD noise oracle (oracle/mask.py normal / dp_noise) and the DP optimisers' host
logic (efl.privacy.dp_optimizer: microbatch split, per-record clip, sum, division) with a noise-free
query, so no GPU is needed.

The reference (efls-train/python/efl/privacy/dp_optimizer.py) draws tf.random.normal from an
unseeded stream, so parity with it is statistical: the oracle's normals are checked for TF's
construction (Box-Muller on Philox word pairs, the 1e-7 clamp) and for their distribution."""
import math

import numpy as np
import pytest
import torch

from oracle import mask

# seed 12345, block 281852: word 2 has zero low 23 bits, so Box-Muller clamps u1 to 1e-7
CLAMP_SEED, CLAMP_BLOCK = 12345, 281852


def test_normal_is_box_muller_of_the_uniform_words():
    z = mask.normal(7, 100, 8)
    u = mask.uniform(7, 100, 8).astype(np.float64)
    for a, b in ((0, 1), (2, 3), (4, 5), (6, 7)):
        r = math.sqrt(-2.0 * math.log(max(u[a], 1e-7)))
        assert abs(z[a] - r * math.sin(2 * math.pi * u[b])) < 1e-5
        assert abs(z[b] - r * math.cos(2 * math.pi * u[b])) < 1e-5


def test_normal_clamp():
    w = mask.philox_blocks(CLAMP_SEED, CLAMP_BLOCK, 1)[0]
    assert w[2] & 0x7FFFFF == 0
    z = mask.normal(CLAMP_SEED, CLAMP_BLOCK, 4)
    r = math.sqrt(-2.0 * math.log(np.float32(1e-7)))
    assert abs(math.hypot(z[2], z[3]) - r) < 1e-5


def test_normal_distribution():
    from scipy import stats
    z = mask.normal(3, 0, 1 << 20).astype(np.float64)
    assert abs(z.mean()) < 5e-3 and abs(z.var() - 1) < 5e-3
    assert stats.kstest(z, "norm").pvalue > 1e-3
    # the counter layout: element i is normal i % 4 of block i / 4
    assert np.array_equal(mask.normal(3, 5, 8), mask.normal(3, 0, 28)[20:28])


def test_dp_noise_arithmetic():
    x = np.array([1.5, -2.0, 0.0, -0.0, 3e38, np.inf], np.float32)
    z = np.array([0.5, -1.0, 2.0, 1.0, 2.0, 0.0], np.float32)
    a = mask.dp_noise(x, 0, 0, 0, 2.0, 4.0, z=z)
    assert a[0] == np.float32((1.5 + 0.5 * 1.5 * 2.0) / 4)
    assert a[1] == np.float32((-2.0 + 2.0 * 2.0) / 4)
    assert a[4] == np.inf                    # (3e38 + 1.2e39) overflows as TF's ops do
    b = mask.dp_noise(x, 0, 0, 1, 2.0, 1.0, z=z)
    assert b[0] == np.float32(1.5 + 1.0) and b[2] == np.float32(4.0)
    assert np.signbit(b[5]) == False         # -0.0 * 2 + 0.0 = +0.0


class NoNoise:
    """A query with the Gaussian query's clip and no noise (host logic only)."""

    def __init__(self, clip=None):
        from efl.privacy import dp_optimizer as dp
        self.q = dp.GaussianSumQuery(clip, 0.0) if clip else dp.ElementWiseGaussianSumQuery(0.0)

    def __getattr__(self, k):
        return getattr(self.q, k)

    def get_noised_result(self, state, g, divisor=1.0):
        return [v / divisor for v in state], g


@pytest.mark.parametrize("clip", [None, 0.5])
@pytest.mark.parametrize("nm", [None, 2, 3])
def test_microbatches_clip_and_mean(clip, nm):
    import efl
    torch.manual_seed(0)
    w = torch.randn(4, 3, requires_grad=True)
    b = torch.randn(3, requires_grad=True)
    x = torch.randn(8, 4)
    opt = efl.privacy.make_optimizer_class(torch.optim.SGD)(NoNoise(clip), nm, False, [w, b], lr=0.1)
    loss = ((x @ w + b) ** 2).sum(dim=1)                   # per-example loss [8]
    got = opt.compute_gradients(loss, [w, b])
    rows = 8 if nm in (None, 3) else nm                    # 8 % 3 != 0: one microbatch per example
    want = [torch.zeros_like(w), torch.zeros_like(b)]
    for r in loss.reshape(rows, -1):
        gw, gb = torch.autograd.grad(r.sum(), [w, b], retain_graph=True)
        if clip:
            norm = torch.sqrt((gw * gw).sum() + (gb * gb).sum())
            s = clip * min(1 / norm.item(), 1 / clip)
            gw, gb = gw * s, gb * s
        want[0] += gw
        want[1] += gb
    for (g, v), e in zip(got, want):
        assert torch.allclose(g, e / rows, rtol=1e-5, atol=1e-6)
    opt.apply_gradients(got)
    assert w.grad is not None


def test_deferred_params_and_learning_rate_alias():
    import efl
    opt = efl.privacy.DPGradientDescentGaussianOptimizer(noise_multiplier=1.0, learning_rate=0.25)
    assert not opt._built
    w = torch.zeros(2, requires_grad=True)
    opt._dp_sum_query = NoNoise()
    loss = (w - torch.tensor([[1.0, 2.0], [3.0, 4.0]])).pow(2).sum(dim=1)
    opt.minimize(loss, [w])
    assert opt._built and opt.param_groups[0]["lr"] == 0.25
    # mean over 2 microbatches of d/dw (w - t)^2 = -2 t: (-2 - 6) / 2, (-4 - 8) / 2; w -= 0.25 g
    assert torch.allclose(w.detach(), torch.tensor([1.0, 1.5]))


def test_params_first_torch_style_and_float64():
    """`DPAdamGaussianOptimizer(model.parameters(), noise_multiplier=.., lr=..)` binds the
    parameters (not noise_multiplier); float64 variables train with a float64 clip norm."""
    import efl
    lin = torch.nn.Linear(3, 2).double()
    opt = efl.privacy.DPAdamGaussianOptimizer(lin.parameters(), noise_multiplier=0.7, l2_norm_clip=1.5, lr=0.01)
    assert opt._built and len(opt.param_groups[0]["params"]) == 2
    assert opt._dp_sum_query._stddev == pytest.approx(1.5 * 0.7)
    opt2 = efl.privacy.DPGradientDescentGaussianOptimizer(params=list(lin.parameters()), noise_multiplier=1.0, lr=0.1)
    assert opt2._built
    q = efl.privacy.make_optimizer_class(torch.optim.SGD)(list(lin.parameters()), dp_sum_query=NoNoise(0.5), lr=0.1)
    assert q._built and isinstance(q._dp_sum_query, NoNoise)
    with pytest.raises(TypeError, match="dp_sum_query"):
        efl.privacy.make_optimizer_class(torch.optim.SGD)(list(lin.parameters()), lr=0.1)
    # float64 records: clip in float64, gradients stay float64
    x = torch.randn(4, 3, dtype=torch.float64, generator=torch.Generator().manual_seed(1))
    opt3 = efl.privacy.make_optimizer_class(torch.optim.SGD)(NoNoise(0.5), 4, False, list(lin.parameters()), lr=0.1)
    got = opt3.compute_gradients((lin(x) ** 2).sum(dim=1), list(lin.parameters()))
    assert all(g.dtype == torch.float64 for g, _ in got)
    rows = [torch.autograd.grad((lin(x[i:i + 1]) ** 2).sum(), list(lin.parameters())) for i in range(4)]
    want = [torch.zeros_like(p) for p in lin.parameters()]
    for gr in rows:
        norm = torch.sqrt(sum((g * g).sum() for g in gr))
        s = 0.5 * min(1 / float(norm), 1 / 0.5)
        for w, g in zip(want, gr):
            w += g * s
    for (g, _), w in zip(got, want):
        assert torch.allclose(g, w / 4, rtol=1e-12, atol=1e-14)
