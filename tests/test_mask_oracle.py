"""CPU: the secret-sharing mask oracle (oracle/mask.py) against Philox4x32-10 known answers, the
uniform's distribution (the only thing the unseeded reference pins, secret_sharing.py:26-27), and
the protocol algebra of secret_sharing.py:30-77 (the two parties' results sum to the product).
Also the C-ABI argument checks of the mask entry points (no compute without a GPU)."""
import ctypes

import numpy as np
import pytest

from oracle import mask, philox

# Random123 known-answer vectors for philox4x32_10 (kat_vectors: ctr, key -> out)
KATS = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,out", KATS)
def test_philox_kat(ctr, key, out):
    assert philox.philox4x32_10(ctr, key) == out


def test_vectorised_blocks_match_scalar():
    seed, ctr0 = 0x0123456789ABCDEF, (1 << 32) - 3      # crosses the 32-bit counter word
    b = mask.philox_blocks(seed, ctr0, 7)
    for i in range(7):
        c = ctr0 + i
        want = philox.philox4x32_10((c & 0xFFFFFFFF, c >> 32, 0, 0), (seed & 0xFFFFFFFF, seed >> 32))
        assert tuple(int(v) for v in b[i]) == want
    assert tuple(int(v) for v in mask.philox_blocks(0, 0, 1)[0]) == KATS[0][2]


def test_uniform_is_tf_uint32_to_float():
    w = mask.philox_blocks(5, 9, 2).reshape(-1)
    u = mask.uniform(5, 9, 8)
    want = np.array([(int(x) & 0x7FFFFF) / 2.0**23 for x in w], dtype=np.float32)
    assert np.array_equal(u, want)
    # a call over n elements is the first n of a longer one (word i % 4 of block i / 4)
    assert np.array_equal(mask.uniform(5, 9, 5), u[:5])


def test_uniform_distribution():
    u = mask.uniform(123, 0, 1 << 20).astype(np.float64)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 3e-3
    assert abs(u.var() - 1 / 12) < 1e-3
    hist, _ = np.histogram(u, bins=64, range=(0, 1))
    expected = u.size / 64
    chi2 = ((hist - expected) ** 2 / expected).sum()
    assert chi2 < 120          # 63 dof; p ~ 1e-5 bound


def test_noise_ops_algebra():
    x = np.random.default_rng(0).standard_normal(1001).astype(np.float32)
    n = mask.noise(x, 7, 0, 0)
    a, kept = mask.noise(x, 7, 0, 1)
    assert np.array_equal(a, n)
    assert np.allclose(a + kept, x, rtol=0, atol=1e-6)
    assert np.all(np.abs(n) <= np.abs(x))
    sent, kept = mask.noise(x, 7, 0, 2, divisor=4.0)
    n4 = (n / np.float32(4)).astype(np.float32)
    assert np.array_equal(sent, (x - n4).astype(np.float32))
    assert np.allclose((sent + kept) / 2, x, atol=1e-6)


@pytest.mark.parametrize("R,C,N", [(4, 6, 3), (5, 8, 7), (16, 32, 8)])
def test_modes_a_b_reconstruct_product(R, C, N):
    """Party A holds a, party B holds b: z_A + z_B = a @ b (secret_sharing.py:30-53)."""
    g = np.random.default_rng(R * C)
    a = g.standard_normal((R, C)).astype(np.float32)
    b = g.standard_normal((C, N)).astype(np.float32)
    a_send, a_minus_e, eo_minus_ee = mask.mask_cols(a, 1, 0)
    b_send, half_plus_f, fo_plus_fe = mask.mask_rows(b, 2, 0)
    b1, f1 = b_send[:C], b_send[C:]
    a1, e1 = a_send[:, :C], a_send[:, C:]
    z_a = a_minus_e.astype(np.float64) @ b1 + eo_minus_ee.astype(np.float64) @ f1
    z_b = a1.astype(np.float64) @ half_plus_f - e1.astype(np.float64) @ fo_plus_fe
    np.testing.assert_allclose(z_a + z_b, a.astype(np.float64) @ b, rtol=1e-5, atol=1e-5)


def test_mask_layouts():
    a = np.arange(24, dtype=np.float32).reshape(4, 6) + 1
    send, k0, k1 = mask.mask_cols(a, 3, 11)
    e = (mask.uniform(3, 11, a.size).reshape(a.shape) * a).astype(np.float32)
    assert send.shape == (4, 9) and k0.shape == (4, 6) and k1.shape == (4, 3)
    assert np.array_equal(send[:, 6:], e[:, 0::2] + e[:, 1::2])
    assert np.array_equal(k1, e[:, 1::2] - e[:, 0::2])
    send, k0, k1 = mask.mask_rows(a, 3, 11)
    assert send.shape == (6, 6) and k1.shape == (2, 6)
    assert np.array_equal(send[:4], (a / 2 - e).astype(np.float32))
    assert np.array_equal(k0, (a / 2 + e).astype(np.float32))


def test_mask_abi_argument_errors():
    import efl
    lib = efl.lib.raw()
    p = ctypes.c_void_p(4096)
    assert lib.efl_ss_noise(p, p, p, 0, 1, 0, 0, 1.0, None) == 0            # empty: no-op
    assert lib.efl_ss_noise(p, p, p, 8, 3, 0, 0, 1.0, None) == -3           # bad op
    assert lib.efl_ss_noise(p, p, p, 8, 0, 0, 0, 0.0, None) == -3           # zero divisor
    assert lib.efl_ss_noise(ctypes.c_void_p(4100), p, p, 8, 0, 0, 0, 1.0, None) == -3   # unaligned
    assert lib.efl_ss_mask_cols(p, p, p, p, 3, 5, 0, 0, None) == -3         # odd columns
    assert "even" in lib.efl_last_error().decode()
    assert lib.efl_ss_mask_rows(p, p, p, p, 3, 4, 0, 0, None) == -3         # odd rows
    assert lib.efl_ss_mask_rows(p, p, p, p, 0, 4, 0, 0, None) == 0
