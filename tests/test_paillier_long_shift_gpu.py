"""Shifts past one launch's squarings (MAX_SHIFT = 2^16 per element), against the Python-int oracle.

The reference has no cap: PaillierMulExp2 is mpz_mul_2exp(1, y) + mpz_powm, y squarings
(paillier.cc:724-731), FixedPointTensor.__add__ composes two of them (paillier.py:116-133) and
PaillierMatmul shifts every term by 2^(xe + ye - min) (paillier.cc:1008-1034). The build cuts longer
shifts into bounded launches (PaillierKeypair._exp2_chunked) and runs a matmul whose exponents
spread past MATMUL_MAX_SPREAD term by term (_matmul_composed); both must give the reference's
ciphertexts bit for bit."""
import numpy as np
import pytest
import torch

from oracle import paillier as P
from test_paillier_gpu import ALL, ENC_KEYS, family, fams, keypair  # noqa: F401
from test_paillier_scalar_gpu import ciphertexts, okeypair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


@pytest.fixture
def pc():
    from efl.privacy import paillier_cipher
    return paillier_cipher


def test_mul_exp2_past_one_launch(efl):
    """y = 2^16 + 1 and 70,000 squarings beside short shifts: two launches, the oracle's values."""
    k = ENC_KEYS[0]
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    cs = ciphertexts(k, 4, 4)
    ys = [1, 0, (1 << 16) + 1, 70000]
    got = kp.mul_exp2(efl.HexTensor.from_ints(cs), torch.tensor(ys)).to_hex().to_ints()
    assert got == [P.mul_exp2(okp, c, y) for c, y in zip(cs, ys)]
    with pytest.raises(efl.errors.InvalidArgumentError, match="y should be a positive tensor"):
        kp.mul_exp2(efl.HexTensor.from_ints(cs), torch.tensor([1, 70000, -1, 0]))


@pytest.mark.parametrize("k,c", fams(ALL))
def test_chunked_shifts_every_family(efl, pc, monkeypatch, k, c):
    """_exp2_chunked with 3 squarings per launch (7 launches for y = 20): x^(2^a) then ^(2^b) is
    x^(2^(a+b)) in every kernel family, elements with no squarings left passing through unchanged."""
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    ys = [0, 1, 2, 3, 4, 7, 10, 20]
    cs = ciphertexts(k, len(ys), 9)
    monkeypatch.setattr(pc, "_SHIFT_CHUNK", 3)
    with family(k["n_bytes"] // 4, False, c):
        x = kp._cipher(efl.HexTensor.from_ints(cs))
        out = kp._exp2_chunked(x.limbs, torch.tensor(ys, device=x.limbs.device))
    got = pc.CipherTensor(out, (len(ys),), kp.key).to_hex().to_ints()
    assert got == [P.mul_exp2(okp, c_, y) for c_, y in zip(cs, ys)]


def test_fxp_add_past_one_launch(efl):
    """FixedPointTensor.__add__ with an exponent gap of 70,000: the fused launch reports the
    element, and the op falls back to the reference's composition with chunked shifts."""
    k = ENC_KEYS[0]
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    xs, ys = ciphertexts(k, 3, 12), ciphertexts(k, 3, 13)
    xe, ye = [0, 70000, -5], [0, 0, 66000]
    z, ze = kp.shift_add(efl.HexTensor.from_ints(xs), torch.tensor(xe), efl.HexTensor.from_ints(ys),
                         torch.tensor(ye))
    want = [P.fixedpoint_add(okp, a, ea, b, eb) for a, ea, b, eb in zip(xs, xe, ys, ye)]
    assert z.to_hex().to_ints() == [w[0] for w in want]
    assert ze.cpu().tolist() == [w[1] for w in want]


def _matmul_inputs(kp, seed, u=3, v=5, w=4):
    rng = np.random.default_rng(seed)
    xm_plain = rng.integers(-2**20, 2**20, (u, v))
    ct = kp.encrypt(torch.from_numpy(xm_plain))
    xe = rng.integers(-30, -10, (u, v))
    ym = rng.integers(-2**20, 2**20, (v, w))
    ym[0, 0] = 0
    ym[1, 1] = -1
    ye = rng.integers(-25, -12, (v, w))
    return ct, xe, ym, ye


@pytest.mark.parametrize("k,c", fams(ALL))
def test_matmul_composed_equals_the_kernel(efl, pc, monkeypatch, k, c):
    """The term-by-term matmul (forced with MATMUL_MAX_SPREAD = 0) gives efl_pl_matmul's ciphertexts
    and exponents bit for bit, in every family, in one row chunk and one row per chunk; an odd
    inner size exercises the product tree's carried column."""
    kp = keypair(efl, k)
    ct, xe, ym, ye = _matmul_inputs(kp, 31, v=5)
    args = (ct.tensor, torch.from_numpy(xe), torch.from_numpy(ym), torch.from_numpy(ye))
    with family(k["n_bytes"] // 4, False, c):
        zk, ek = kp.matmul(*args)
        monkeypatch.setattr(pc, "MATMUL_MAX_SPREAD", 0)
        zc, ec = kp.matmul(*args)
        monkeypatch.setattr(pc, "_COMPOSED_CHUNK_BYTES", 1)     # one row per chunk
        zr, er = kp.matmul(*args)
    assert torch.equal(ek.cpu(), ec.cpu()) and torch.equal(ek.cpu(), er.cpu())
    assert zk.to_hex().to_ints() == zc.to_hex().to_ints() == zr.to_hex().to_ints()


def test_matmul_wide_exponent_spread(efl, pc):
    """Exponents spread by 70,000 (past one launch's squarings): the composed path against the
    oracle, ciphertexts and exponents."""
    k = ENC_KEYS[0]
    kp, okp = keypair(efl, k), okeypair(k)
    ct, xe, ym, ye = _matmul_inputs(kp, 32, u=2, v=3, w=2)
    xe[0, 1] += 70000
    zm, ze = kp.matmul(ct.tensor, torch.from_numpy(xe), torch.from_numpy(ym), torch.from_numpy(ye))
    xs = [[int(s, 16) for s in row] for row in np.array(ct.tensor.to_hex().strings()).reshape(2, 3)]
    om, oe = P.matmul(okp, xs, xe.tolist(), ym.tolist(), ye.tolist())
    assert ze.cpu().tolist() == oe
    assert zm.to_hex().to_ints() == [c_ for row in om for c_ in row]
