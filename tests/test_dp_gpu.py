"""GPU parity: the DP-SGD noise kernel (csrc/mask.hip efl_dp_noise through efl.privacy.dp_optimizer)
against the oracle (oracle/mask.py).

Tolerance. The normals use the device's logf / sincosf; the oracle rounds float64 log/sin/cos to
float32. They agree within 4 float32 ulp (stated below); everything after the normal is the same
sequence of float32 operations (fp contraction off in mask.hip), so with the kernel's own normals
fed to the oracle the outputs are equal bit for bit. The kernel's normals are read back exactly
from mode 1 with x = 0, sigma = 1, divisor = 1: 0 + (z * 1 + 0) / 1 = z."""
import numpy as np
import pytest
import torch

from oracle import mask
from test_dp_oracle import CLAMP_BLOCK, CLAMP_SEED

pytestmark = pytest.mark.gpu

ULP_TOL = 4


@pytest.fixture(scope="module")
def dp():
    import efl
    efl.lib.require_gpu()
    from efl.privacy import dp_optimizer
    return dp_optimizer


def kernel_normals(dp, seed, ctr0, n):
    from efl.privacy.secret_sharing import NoiseStream
    z = dp.dp_noise(torch.zeros(n, device="cuda"), 1, 1.0, 1.0, NoiseStream(seed, ctr0))
    return z.cpu().numpy()


def ulps(a, b):
    a = a.astype(np.float32).view(np.int32).astype(np.int64)
    b = b.astype(np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    return np.abs(a - b)


@pytest.mark.parametrize("n", [1, 3, 4, 7, 4096, 262147])
def test_normals_vs_oracle(dp, n):
    z = kernel_normals(dp, 99, 17, n)
    assert ulps(z, mask.normal(99, 17, n)).max() <= ULP_TOL


def test_normals_clamp(dp):
    z = kernel_normals(dp, CLAMP_SEED, CLAMP_BLOCK, 4)
    assert ulps(z, mask.normal(CLAMP_SEED, CLAMP_BLOCK, 4)).max() <= ULP_TOL
    assert abs(np.hypot(z[2], z[3]) - np.sqrt(-2 * np.log(np.float32(1e-7)))) < 1e-4


@pytest.mark.parametrize("mode,sigma,div", [(0, 1.0, 1.0), (0, 0.7, 256.0), (1, 1.5, 3.0), (1, 0.0, 1.0),
                                            (0, 1.1, 3.0), (1, 1.1, 256.0), (0, 1.0, -0.5), (1, 1.0, 2.0 ** 120)])
@pytest.mark.parametrize("n", [5, 1000, 65539])
def test_noise_bit_exact_given_normals(dp, mode, sigma, div, n):
    from efl.privacy.secret_sharing import NoiseStream
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32) * 3
    x[:5] = [0.0, -0.0, 1e-40, 3e38, -np.inf][:min(5, n)]
    got = dp.dp_noise(torch.from_numpy(x).cuda(), mode, sigma, div, NoiseStream(5, 40)).cpu().numpy()
    z = kernel_normals(dp, 5, 40, n)
    want = mask.dp_noise(x, 5, 40, mode, sigma, div, z=z)
    g, w = got.view(np.uint32), want.view(np.uint32)
    same = (g == w) | (np.isnan(got) & np.isnan(want))
    assert same.all(), np.nonzero(~same)[0][:8]
    # and within the stated tolerance of the oracle's own normals: a normal off by ULP_TOL ulp moves
    # the output by |x sigma z| ULP_TOL 2^-23 / div (mode 0; |sigma z| ... in mode 1), plus the
    # output's own rounding
    ref = mask.dp_noise(x, 5, 40, mode, sigma, div)
    zr = mask.normal(5, 40, n)
    fin = np.isfinite(ref)
    scale = (np.abs(x.astype(np.float64)) if mode == 0 else 1.0) * sigma * np.abs(zr) / abs(div)
    bound = scale * ULP_TOL * 2.0 ** -23 + 2 * np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    assert (err[fin] <= bound[fin]).all()


def test_in_place_and_stream_advance(dp):
    from efl.privacy.secret_sharing import NoiseStream
    import efl
    s = NoiseStream(8, 0)
    x = torch.ones(10, device="cuda")
    a = dp.dp_noise(x, 0, 1.0, 1.0, s)
    assert s.counter == 3                                    # ceil(10 / 4) blocks
    b = dp.dp_noise(x, 0, 1.0, 1.0, s)
    assert not torch.equal(a, b)
    y = x.clone()
    efl.lib.check(efl.lib.raw().efl_dp_noise(y.data_ptr(), y.data_ptr(), 10, 0, 1.0, 1.0, 8, 0,
                                             efl.lib.stream_handle(y.device)))
    assert torch.equal(y, a)
    assert efl.lib.raw().efl_dp_noise(y.data_ptr(), y.data_ptr(), 10, 2, 1.0, 1.0, 8, 0, None) < 0
    assert efl.lib.raw().efl_dp_noise(y.data_ptr(), y.data_ptr(), 10, 0, 1.0, 0.0, 8, 0, None) < 0


def test_normal_moments_large(dp):
    from scipy import stats
    z = kernel_normals(dp, 2024, 0, 1 << 24).astype(np.float64)
    assert abs(z.mean()) < 1e-3 and abs(z.var() - 1) < 1e-3
    assert stats.kstest(z[: 1 << 20], "norm").pvalue > 1e-3


@pytest.mark.parametrize("clip", [None, 1.0])
def test_optimizer_step_matches_oracle(dp, clip):
    """DPGradientDescentGaussianOptimizer on a small model (the dp_mnist examples' optimiser:
    dp_cnn.py:85-86 with l2_norm_clip, leader.py:89-90 without): the applied gradient equals the
    oracle's per-microbatch sum (clipped) + noise from the same stream positions, / microbatches."""
    import efl
    torch.manual_seed(1)
    w = torch.randn(6, 4, device="cuda", requires_grad=True)
    b = torch.zeros(4, device="cuda", requires_grad=True)
    x = torch.randn(16, 6, device="cuda")
    w0 = w.detach().clone()
    efl.privacy.set_noise_seed(77, 0)
    opt = efl.privacy.DPGradientDescentGaussianOptimizer(noise_multiplier=1.1, l2_norm_clip=clip, num_microbatches=4,
                                                         learning_rate=0.5)
    loss = torch.nn.functional.cross_entropy(x @ w + b, torch.arange(16, device="cuda") % 4, reduction="none")
    sums = [torch.zeros_like(w), torch.zeros_like(b)]
    for r in loss.reshape(4, -1):
        gw, gb = torch.autograd.grad(r.sum(), [w, b], retain_graph=True)
        if clip:
            norm = torch.sqrt((gw * gw).sum() + (gb * gb).sum())
            s = clip * torch.minimum(1 / norm, torch.tensor(1 / clip, device="cuda"))
            gw, gb = gw * s, gb * s
        sums[0] += gw
        sums[1] += gb
    opt.minimize(loss, [w, b])
    ctr = 0
    for v, sm, v0 in ((w, sums[0], w0), (b, sums[1], torch.zeros(4, device="cuda"))):
        n = sm.numel()
        mode, sigma = (0, 1.1) if clip is None else (1, clip * 1.1)
        g = mask.dp_noise(sm.detach().cpu().numpy().reshape(-1), 77, ctr, mode, sigma, 4.0)
        ctr += (n + 3) // 4
        want = v0.cpu().numpy().reshape(-1) - 0.5 * g
        assert np.allclose(v.detach().cpu().numpy().reshape(-1), want, rtol=1e-4, atol=1e-5)


def test_float64_and_half_gradients_take_the_float32_noise(dp):
    """float64 (and bf16) gradients are noised, not rejected: the kernel's float32 noise
    of the float32 value, cast back to the gradient's dtype (same stream position, same bits)."""
    from efl.privacy.secret_sharing import NoiseStream
    x = torch.randn(1001, dtype=torch.float64, generator=torch.Generator().manual_seed(3)).cuda()
    got = dp.dp_noise(x, 0, 0.9, 4.0, NoiseStream(12, 5))
    assert got.dtype == torch.float64
    want = dp.dp_noise(x.float(), 0, 0.9, 4.0, NoiseStream(12, 5)).double()
    assert torch.equal(got, want)
    xb = x.to(torch.bfloat16)
    gb = dp.dp_noise(xb, 1, 1.0, 1.0, NoiseStream(12, 5))
    assert gb.dtype == torch.bfloat16
    assert torch.equal(gb, dp.dp_noise(xb.float(), 1, 1.0, 1.0, NoiseStream(12, 5)).to(torch.bfloat16))
    with pytest.raises(Exception, match="floating-point"):
        dp.dp_noise(torch.ones(4, dtype=torch.int32, device="cuda"), 0, 1.0, 1.0, NoiseStream(1, 0))


@pytest.mark.parametrize("n", [1, 5, 1023, 1024, 4097, 262147, 1 << 20])
def test_blocks_per_lane_layouts_agree(dp, n):
    """efl_fxp_tune(20, nb): 1, 2 or 4 Philox blocks per lane give the same bits, in place too, for
    sizes that leave every kind of ragged last workgroup (the kernel's full-tile and tail paths)."""
    import efl
    from efl.privacy.secret_sharing import NoiseStream
    lib = efl.lib.raw()
    x = torch.randn(n, generator=torch.Generator().manual_seed(n)).cuda()
    outs = []
    old = lib.efl_fxp_tune(20, 1)
    try:
        for nb in (1, 2, 4):
            lib.efl_fxp_tune(20, nb)
            outs.append(dp.dp_noise(x, 0, 1.3, 7.0, NoiseStream(11, 3)).cpu())
            y = x.clone()
            efl.lib.check(lib.efl_dp_noise(y.data_ptr(), y.data_ptr(), n, 1, 0.9, 256.0, 11, 3,
                                           torch.cuda.current_stream().cuda_stream))
            outs.append(y.cpu())
    finally:
        lib.efl_fxp_tune(20, old)
    for a, b in ((outs[0], outs[2]), (outs[0], outs[4]), (outs[1], outs[3]), (outs[1], outs[5])):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    assert lib.efl_fxp_tune(20, 3) < 0      # only 1, 2, 4
