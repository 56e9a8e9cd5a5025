"""GPU parity: the secret-sharing mask kernels (csrc/mask.hip, through the C ABI via
efl.secret_sharing) against the numpy oracle (oracle/mask.py), bit for bit, on ragged, aligned
and unaligned shapes; at 64 Mi elements through size-independent properties (shares sum back to
the input, |noise| <= |x|, uniform moments)."""
import numpy as np
import pytest
import torch

from oracle import mask

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ss():
    import efl
    efl.lib.require_gpu()
    return efl.secret_sharing


def nbits(a):
    """uint32 bit patterns, every NaN mapped to one pattern: x86 (the oracle) produces the negative
    default NaN for inf - inf, the GPU the positive one; payloads are not part of the contract."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    return np.where(np.isnan(a), np.uint32(0x7FC00000), a.view(np.uint32))


def bits(t):
    return nbits(t.detach().cpu().numpy())


def rand(shape, seed):
    x = np.random.default_rng(seed).standard_normal(shape).astype(np.float32)
    flat = x.reshape(-1)
    special = np.array([0.0, -0.0, 1e-40, -1e-40, 3.4e38, -3.4e38, np.inf, -np.inf, np.nan], np.float32)
    flat[: min(flat.size, special.size)] = special[: flat.size]
    return x


@pytest.mark.parametrize("n", [1, 3, 4, 5, 1023, 4096, 262147])
@pytest.mark.parametrize("op,div", [(0, 1.0), (1, 1.0), (2, 1.0), (2, 3.0), (0, 7.5)])
def test_noise_matches_oracle(ss, n, op, div):
    x = rand(n, n)
    st = ss.NoiseStream(0xC0FFEE ^ n, 17)
    got = ss._noise(torch.from_numpy(x).cuda(), op, div, stream=st)
    want = mask.noise(x, 0xC0FFEE ^ n, 17, op, div)
    got = got if isinstance(got, tuple) else (got,)
    want = want if isinstance(want, tuple) else (want,)
    for g, w in zip(got, want):
        assert np.array_equal(bits(g), nbits(w))
    assert st.counter == 17 + (n + 3) // 4


def test_stream_counter_continues(ss):
    x = rand(1000, 1)
    st = ss.NoiseStream(99, 0)
    a = ss.generate_suitable_noise(torch.from_numpy(x[:500]).cuda(), stream=st)
    b = ss.generate_suitable_noise(torch.from_numpy(x[500:]).cuda(), stream=st)
    assert np.array_equal(bits(a), nbits(mask.noise(x[:500], 99, 0)))
    assert np.array_equal(bits(b), nbits(mask.noise(x[500:], 99, 125)))


def test_unaligned_view_and_host_tensor(ss):
    x = rand(1025, 2)
    t = torch.from_numpy(x).cuda()[1:]          # 4-byte offset view: staged through an aligned copy
    st = ss.NoiseStream(5, 0)
    a, kept = ss.split_share(t, stream=st)
    wa, wk = mask.noise(x[1:], 5, 0, 1)
    assert np.array_equal(bits(a), nbits(wa)) and np.array_equal(bits(kept), nbits(wk))
    st = ss.NoiseStream(5, 0)
    h = ss.generate_suitable_noise(torch.from_numpy(x[1:].copy()), stream=st)   # host in, host out
    assert h.device.type == "cpu" and np.array_equal(bits(h), nbits(wa))


@pytest.mark.parametrize("R,C", [(1, 2), (3, 6), (4, 8), (7, 12), (5, 16), (33, 100), (256, 392), (129, 1030)])
def test_mask_cols_matches_oracle(ss, R, C):
    a = rand((R, C), R * 1000 + C)
    st = ss.NoiseStream(R + C, 3)
    got = ss.mask_cols(torch.from_numpy(a).cuda(), stream=st)
    want = mask.mask_cols(a, R + C, 3)
    for g, w in zip(got, want):
        assert g.shape == w.shape
        assert np.array_equal(bits(g), nbits(w))


@pytest.mark.parametrize("K,N", [(2, 1), (2, 4), (6, 3), (8, 8), (10, 13), (392, 256), (1030, 129)])
def test_mask_rows_matches_oracle(ss, K, N):
    b = rand((K, N), K * 1000 + N)
    st = ss.NoiseStream(K * N, 8)
    got = ss.mask_rows(torch.from_numpy(b).cuda(), stream=st)
    want = mask.mask_rows(b, K * N, 8)
    for g, w in zip(got, want):
        assert g.shape == w.shape
        assert np.array_equal(bits(g), nbits(w))


def test_mask_argument_errors(ss):
    import efl
    with pytest.raises(efl.errors.InvalidArgumentError):
        ss.mask_cols(torch.zeros(4, 5, device="cuda"))
    with pytest.raises(efl.errors.InvalidArgumentError):
        ss.mask_rows(torch.zeros(5, 4, device="cuda"))
    with pytest.raises(efl.errors.InvalidArgumentError):
        ss.generate_suitable_noise(torch.zeros(4, dtype=torch.float64, device="cuda"))
    assert ss.generate_suitable_noise(torch.zeros(0, device="cuda")).numel() == 0


def test_share_full_size_properties(ss):
    """BASELINE-size tensor (64 Mi fp32): a + (x - a) == x up to one rounding, 0 <= a/x < 1, and
    the sampled uniform has the right moments; plus a 1 % sampled bit compare to the oracle."""
    n = 1 << 26
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, device="cuda", generator=g)
    st = ss.NoiseStream(2024, 0)
    a, kept = ss.split_share(x, stream=st)
    err = ((a + kept) - x).abs()
    assert float((err - x.abs() * 2**-22).clamp(min=0).max()) == 0.0
    nz = x != 0
    r = a[nz] / x[nz]
    assert float(r.min()) >= 0.0 and float(r.max()) <= 1.0   # U < 1, U * x may round to x
    assert abs(float(r.double().mean()) - 0.5) < 1e-3
    idx = torch.randint(0, n // 4, (n // 400,), device="cuda", generator=g)
    idx = (idx[:, None] * 4 + torch.arange(4, device="cuda")).reshape(-1)
    xs = x[idx].cpu().numpy()
    u = np.stack([mask.uniform(2024, int(b), 4) for b in (idx[::4] // 4).cpu().numpy()[:2000]])
    want = (u.reshape(-1) * xs[: u.size]).astype(np.float32)
    assert np.array_equal(bits(a[idx][: u.size]), nbits(want))


@pytest.mark.parametrize("nb", [1, 2, 4])
@pytest.mark.parametrize("st", [0, 2, 7])
def test_mask_variants_identical(ss, nb, st):
    """Every lane-group count (efl_fxp_tune 25) and store flavour (28) of the mask kernels gives the
    oracle's bits, at sizes whose last lane groups are partial (the per-group tail path) and at sizes
    that fill every group."""
    import efl
    lib = efl.lib.raw()
    old = lib.efl_fxp_tune(25, nb), lib.efl_fxp_tune(28, st)
    assert min(old) >= 0
    try:
        for n in (5, 4096 * 4 + 12, 4 * 256 * 4 * 3 + 4):
            x = rand(n, n + nb)
            for op, div in ((0, 1.0), (1, 1.0), (2, 3.0)):
                got = ss._noise(torch.from_numpy(x).cuda(), op, div, stream=ss.NoiseStream(n, 9))
                want = mask.noise(x, n, 9, op, div)
                got = got if isinstance(got, tuple) else (got,)
                want = want if isinstance(want, tuple) else (want,)
                for g, w in zip(got, want):
                    assert np.array_equal(bits(g), nbits(w)), (n, op)
        for R, C in ((3, 8), (257, 1024), (100, 392)):
            a = rand((R, C), R + C)
            for g, w in zip(ss.mask_cols(torch.from_numpy(a).cuda(), stream=ss.NoiseStream(R, 1)),
                            mask.mask_cols(a, R, 1)):
                assert np.array_equal(bits(g), nbits(w)), (R, C)
        for K, N in ((2, 4), (514, 1024), (392, 256)):
            b = rand((K, N), K + N)
            for g, w in zip(ss.mask_rows(torch.from_numpy(b).cuda(), stream=ss.NoiseStream(K, 2)),
                            mask.mask_rows(b, K, 2)):
                assert np.array_equal(bits(g), nbits(w)), (K, N)
    finally:
        lib.efl_fxp_tune(25, -2)
        lib.efl_fxp_tune(28, -2)


@pytest.mark.parametrize("half", [0, 1])
@pytest.mark.parametrize("nb", [1, 2, 4])
@pytest.mark.parametrize("st", [0, 2, 7])
def test_mask_rows_layouts_identical(ss, half, nb, st):
    """mask_rows with the row pair over the halves of a wave (efl_fxp_tune 29 = 1, the default) and in
    one lane (0), at every lane-group count and store flavour, gives the oracle's bits: one lane
    group, partial waves (33 groups a row pair), and full ones."""
    import efl
    lib = efl.lib.raw()
    assert lib.efl_fxp_tune(29, -1) == 1                       # the halves by default
    assert lib.efl_fxp_tune(29, 2) < 0
    lib.efl_fxp_tune(29, half)
    lib.efl_fxp_tune(25, nb)
    lib.efl_fxp_tune(28, st)
    try:
        for K, N in ((2, 4), (6, 132), (514, 1024), (392, 256), (130, 4 * 33 * 3)):
            b = rand((K, N), K * 7 + N)
            for g, w in zip(ss.mask_rows(torch.from_numpy(b).cuda(), stream=ss.NoiseStream(K, 2)),
                            mask.mask_rows(b, K, 2)):
                assert np.array_equal(bits(g), nbits(w)), (K, N)
    finally:
        lib.efl_fxp_tune(29, 1)
        lib.efl_fxp_tune(25, -2)
        lib.efl_fxp_tune(28, -2)


@pytest.mark.parametrize("half", [0, 1])
@pytest.mark.parametrize("st", [0, 2, 7])
def test_noise_halves_identical(ss, half, st):
    """share and weight noise with the two outputs over the halves of a wave (efl_fxp_tune 30 = 1, the
    default) and both in one lane (0) give the oracle's bits, at sizes ending in a partial group, a partial wave, and full waves."""
    import efl
    lib = efl.lib.raw()
    assert lib.efl_fxp_tune(30, -1) == 1                       # the halves by default
    assert lib.efl_fxp_tune(30, 2) < 0
    prev = lib.efl_fxp_tune(30, half)
    lib.efl_fxp_tune(28, st)
    try:
        for n in (5, 4 * 33 + 2, 4096 * 4 + 12, 4 * 256 * 4 * 3 + 4):
            x = rand(n, n + 3)
            for op, div in ((1, 1.0), (2, 3.0), (1, 4.0)):
                got = ss._noise(torch.from_numpy(x).cuda(), op, div, stream=ss.NoiseStream(n, 9))
                want = mask.noise(x, n, 9, op, div)
                for g, w in zip(got, want):
                    assert np.array_equal(bits(g), nbits(w)), (n, op, div)
    finally:
        lib.efl_fxp_tune(30, prev)
        lib.efl_fxp_tune(28, -2)
