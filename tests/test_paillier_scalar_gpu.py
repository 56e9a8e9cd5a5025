"""GPU parity of the device-side scalar ops of Stage P against the Python-int oracle (which the
GMP known answers pin, tests/test_paillier_oracle.py):

  PaillierMulExp2<int64>      (paillier.cc:680-751)  -> efl_pl_mul_exp2
  PaillierMulScalar<int64>    (paillier.cc:197-237)  -> efl_pl_mul_scalar
  PaillierMulScalar<string>   (paillier.cc:239-248)  -> efl_hex_parse + efl_pl_mul_scalar_big
  FixedPointTensor.__add__    (paillier.py:116-133)  -> efl_pl_fxp_add (one fused launch)
  PaillierPassiveWeight's row reduction (paillier_layer.py:297-310) -> one efl_pl_matmul by ones

Bar: bit-exact ciphertexts for every kernel family, the reference's errors for bad operands."""
import random

import numpy as np
import pytest
import torch

from oracle import paillier as P
from test_paillier_gpu import ALL, ENC_KEYS, KAT, family, fams, keypair  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


def okeypair(k):
    return P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))


def ciphertexts(k, count, seed):
    """count valid ciphertexts (< n^2): the KAT ciphertexts, then products of them."""
    okp = okeypair(k)
    base = [int(v["c"], 16) for v in k["vectors"]]
    rng = random.Random(seed)
    out = list(base[:count])
    while len(out) < count:
        out.append(rng.choice(base) * rng.choice(base) % okp.n2)
    return out


@pytest.mark.parametrize("k,c", fams(ALL))
def test_mul_exp2_int64_on_device(efl, k, c):
    """y squarings per element, y from 0 (x mod n^2) to a few hundred, mixed within every wave."""
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    n = 70 if k["n_bytes"] < 512 else 24
    cs = ciphertexts(k, n, 1)
    rng = random.Random(2)
    ys = [0, 1, 2, 31, 32, 33, 64, 300] + [rng.randrange(0, 160) for _ in range(n - 8)]
    with family(k["n_bytes"] // 4, False, c):
        got = kp.mul_exp2(efl.HexTensor.from_ints(cs), torch.tensor(ys)).to_hex().to_ints()
    assert got == [P.mul_exp2(okp, x, y) for x, y in zip(cs, ys)]


def test_mul_exp2_int32_and_broadcast(efl):
    k = ENC_KEYS[1]
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    cs = ciphertexts(k, 6, 3)
    x = efl.HexTensor.from_ints(cs, (2, 3))
    got = kp.mul_exp2(x, torch.tensor([4, 0, 9], dtype=torch.int32))          # y [3] over x [2, 3]
    assert got.shape == (2, 3)
    assert got.to_hex().to_ints() == [P.mul_exp2(okp, c, y) for c, y in zip(cs, [4, 0, 9] * 2)]
    got = kp.mul_exp2(efl.HexTensor.from_ints(cs[:1]), np.array([[1], [2], [3]]))   # x [1] over y [3, 1]
    assert got.shape == (3, 1) and got.to_hex().to_ints() == [P.mul_exp2(okp, cs[0], y) for y in (1, 2, 3)]
    # the operator form (paillier.py:48-50)
    pt = efl.paillier.Tensor(kp, kp._cipher(efl.HexTensor.from_ints(cs[:3])))
    assert (pt << torch.tensor([2, 5, 7])).tensor.to_hex().to_ints() == \
        [P.mul_exp2(okp, c, y) for c, y in zip(cs[:3], (2, 5, 7))]


def test_mul_exp2_errors(efl):
    k = ENC_KEYS[0]
    kp = keypair(efl, k, private=False)
    x = efl.HexTensor.from_ints(ciphertexts(k, 4, 4))
    with pytest.raises(efl.errors.InvalidArgumentError, match="y should be a positive tensor"):
        kp.mul_exp2(x, torch.tensor([1, 2, -3, 4]))
    with pytest.raises(efl.errors.InvalidArgumentError, match="int32 or int64"):
        kp.mul_exp2(x, ["1", "2", "3", "4"])
    with pytest.raises(efl.errors.InvalidArgumentError, match="dtype"):
        kp.mul_exp2(x, torch.tensor([1.0, 2.0, 3.0, 4.0]))
    # the largest one-launch shift (65536 squarings of one element; longer ones: test_paillier_long_shift_gpu.py)
    assert kp.mul_exp2(efl.HexTensor.from_ints([2]), torch.tensor([1 << 16])).to_hex().to_ints() == \
        [pow(2, 1 << (1 << 16), kp.key.n ** 2)]


@pytest.mark.parametrize("k,c", fams(ALL))
def test_mul_scalar_int64_on_device(efl, k, c):
    """|y| powm + an inversion restricted to the negative scalars, int64 extremes included."""
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    n = 40 if k["n_bytes"] < 512 else 16
    cs = ciphertexts(k, n, 5)
    rng = random.Random(6)
    ys = [0, 1, -1, 2**63 - 1, -2**63, 7, -7, 2**32] + [rng.randrange(-2**40, 2**40) for _ in range(n - 8)]
    with family(k["n_bytes"] // 4, False, c):
        got = kp.mul_scalar(efl.HexTensor.from_ints(cs), torch.tensor(ys)).to_hex().to_ints()
        pos = kp.mul_scalar(efl.HexTensor.from_ints(cs), torch.tensor([abs(y) % 1000 for y in ys]))
    assert got == [P.mul_scalar(okp, x, y) for x, y in zip(cs, ys)]
    assert pos.to_hex().to_ints() == [P.mul_scalar(okp, x, abs(y) % 1000) for x, y in zip(cs, ys)]


@pytest.mark.parametrize("k,c", fams(ENC_KEYS))
def test_mul_scalar_string_is_signed_hex(efl, k, c):
    """PaillierMulScalar<string> parses the scalars with mpz_init_set_str(op, y, 16): "12" is 18,
    "-ff" is -255, and scalars wider than int64 work (round-2 VERDICT: the build parsed decimal)."""
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    cs = ciphertexts(k, 8, 7)
    ys = ["12", "-ff", "0", "1", "-1", "FFFFFFFFFFFFFFFFFFFF", "-123456789abcdef0123456789", "7fffffffffffffff"]
    with family(k["n_bytes"] // 4, False, c):
        got = kp.mul_scalar(efl.HexTensor.from_ints(cs), ys).to_hex().to_ints()
        hx = kp.mul_scalar(efl.HexTensor.from_ints(cs), efl.HexTensor.from_strings(ys)).to_hex().to_ints()
        one = kp.mul_scalar(efl.HexTensor.from_ints(cs), "12").to_hex().to_ints()     # broadcast scalar
    want = [P.mul_scalar_hex(okp, x, y) for x, y in zip(cs, ys)]
    assert got == want and hx == want
    assert want[0] == P.mul_scalar(okp, cs[0], 18)
    assert one == [P.mul_scalar(okp, x, 0x12) for x in cs]


def test_mul_scalar_wide_python_ints_and_errors(efl):
    k = ENC_KEYS[1]
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    cs = ciphertexts(k, 3, 8)
    ys = [1 << 100, -(1 << 70) - 5, 3]                # beyond int64: carried as big integers
    assert kp.mul_scalar(efl.HexTensor.from_ints(cs), ys).to_hex().to_ints() == \
        [P.mul_scalar(okp, x, y) for x, y in zip(cs, ys)]
    with pytest.raises(efl.errors.InvalidArgumentError, match="hex"):
        kp.mul_scalar(efl.HexTensor.from_ints(cs), ["12", "zz", "1"])
    with pytest.raises(efl.errors.InvalidArgumentError, match="hex"):
        kp.mul_scalar(efl.HexTensor.from_ints(cs), ["12", "", "1"])
    with pytest.raises(efl.errors.InvalidArgumentError, match="no inverse"):
        kp.mul_scalar(efl.HexTensor.from_ints([okp.n, cs[0]]), torch.tensor([-1, 2]))
    # a non-invertible x with a non-negative scalar is fine (no inversion needed)
    assert kp.mul_scalar(efl.HexTensor.from_ints([okp.n]), torch.tensor([2])).to_hex().to_ints() == \
        [okp.n * okp.n % okp.n2]


@pytest.mark.parametrize("k,c", fams(ALL))
def test_fxp_add_fused_equals_composition(efl, k, c):
    """efl_pl_fxp_add == PaillierAdd(PaillierMulExp2(x, dl), PaillierMulExp2(y, dr)) bit for bit,
    for either side shifted, equal exponents and int64 exponents far from zero."""
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    n = 48 if k["n_bytes"] < 512 else 16
    xs, ys = ciphertexts(k, n, 9), ciphertexts(k, n, 10)
    rng = random.Random(11)
    xe = [rng.randrange(-300, 100) for _ in range(n)]
    ye = [e + rng.choice([0, 1, -1, 17, -17, 130, -130]) for e in xe]
    xe[:3] = [-(2**62), 2**62, 5]
    ye[:3] = [-(2**62) + 3, 2**62, 5]
    with family(k["n_bytes"] // 4, False, c):
        z, ze = kp.shift_add(efl.HexTensor.from_ints(xs), torch.tensor(xe), efl.HexTensor.from_ints(ys),
                             torch.tensor(ye))
    want = [P.fixedpoint_add(okp, a, ea, b, eb) for a, ea, b, eb in zip(xs, xe, ys, ye)]
    assert z.to_hex().to_ints() == [w[0] for w in want]
    assert ze.cpu().tolist() == [w[1] for w in want]


def test_fxp_add_errors_and_broadcast(efl):
    k = ENC_KEYS[0]
    kp, okp = keypair(efl, k, private=False), okeypair(k)
    xs, ys = ciphertexts(k, 6, 12), ciphertexts(k, 3, 13)
    z, ze = kp.shift_add(efl.HexTensor.from_ints(xs, (2, 3)), torch.tensor([[0, 5, -5], [1, 2, 3]]),
                         efl.HexTensor.from_ints(ys), torch.tensor(2))        # y [3], exponent scalar
    assert z.shape == (2, 3) and tuple(ze.shape) == (2, 3)
    xe = [0, 5, -5, 1, 2, 3]
    assert z.to_hex().to_ints() == [P.fixedpoint_add(okp, a, ea, ys[i % 3], 2)[0] for i, (a, ea) in enumerate(zip(xs, xe))]
    # a gap past one launch's squarings: tests/test_paillier_long_shift_gpu.py


def test_fixed_point_tensor_add_is_the_fused_op(efl):
    """FixedPointTensor + FixedPointTensor / + plaintext (paillier.py:116-133) through the fused op:
    ciphertexts equal the oracle's composition given the same encryption randomness."""
    k = ENC_KEYS[1]
    kp, okp = keypair(efl, k, seed=77), okeypair(k)
    g = torch.Generator().manual_seed(3)
    a = torch.randn(5, 7, generator=g).cuda()
    b = torch.randn(5, 7, generator=g).cuda()
    a[0, 0] = 0.0                                          # E = -127: a 100-odd squaring shift
    fa = efl.paillier.fixedpoint.encode(a)
    fb = efl.paillier.fixedpoint.encode(b)
    ca = kp.encrypt(fa.mantissa)
    cb = kp.encrypt(fb.mantissa)
    s = efl.paillier.fixedpoint.Tensor(ca, fa.exponent) + efl.paillier.fixedpoint.Tensor(cb, fb.exponent)
    xs, ys = ca.tensor.to_hex().to_ints(), cb.tensor.to_hex().to_ints()
    want = [P.fixedpoint_add(okp, x, int(ea), y, int(eb)) for x, ea, y, eb in
            zip(xs, fa.exponent.reshape(-1).tolist(), ys, fb.exponent.reshape(-1).tolist())]
    assert s.mantissa.tensor.to_hex().to_ints() == [w[0] for w in want]
    assert s.exponent.reshape(-1).cpu().tolist() == [w[1] for w in want]
    y = efl.paillier.fixedpoint.decode(efl.paillier.fixedpoint.Tensor(kp.decrypt(s.mantissa), s.exponent))
    assert torch.allclose(y, a + b)


@pytest.mark.parametrize("rows,cols", [(1, 5), (2, 3), (9, 4), (64, 3)])
def test_weight_column_sum_one_launch_equals_sequential(efl, rows, cols):
    """PaillierPassiveWeight's dw reduction as one matmul by ones == the reference's row-by-row
    FixedPointTensor.__add__ loop (paillier_layer.py:297-310), ciphertext bits and exponents."""
    from efl.privacy import paillier_layer as L
    k = ENC_KEYS[1]
    kp, okp = keypair(efl, k, seed=5), okeypair(k)
    g = torch.Generator().manual_seed(rows * 100 + cols)
    x = torch.randn(rows, cols, generator=g).cuda()
    dy = torch.randn(rows, cols, generator=g).cuda()
    fx = efl.paillier.fixedpoint.encode(x)
    cx = efl.paillier.fixedpoint.Tensor(kp.encrypt(fx.mantissa), fx.exponent)
    dw = cx * efl.paillier.fixedpoint.encode(dy, decrease_precision=True)
    got = L.column_sum(kp, dw)
    seq = L.sequential_column_sum(kp, dw)
    assert got.mantissa.tensor.to_hex().to_ints() == seq.mantissa.tensor.to_hex().to_ints()
    assert torch.equal(got.exponent.cpu(), seq.exponent.cpu())
    m = dw.mantissa.tensor.to_hex().to_ints()
    e = dw.exponent.cpu().tolist()
    om, oe = P.column_sum(okp, [m[r * cols:(r + 1) * cols] for r in range(rows)], e)
    assert got.mantissa.tensor.to_hex().to_ints() == om and got.exponent.cpu().tolist() == oe
    # and it decrypts to the column sums of x * dy
    val = efl.paillier.fixedpoint.decode(efl.paillier.fixedpoint.Tensor(kp.decrypt(got.mantissa), got.exponent))
    want = (x.double() * efl.paillier.fixedpoint.decode(efl.paillier.fixedpoint.encode(dy, True)).double()).sum(0)
    assert torch.allclose(val.double(), want, rtol=1e-5, atol=1e-6)
