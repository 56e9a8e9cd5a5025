"""The reference's own Paillier test (efls-train/test/paillier_test.py:20-79) at its own settings:
`PaillierKeypair().generate_keypair()` with the default 4096-bit n (n_bytes 512, a_bytes 256,
group size 1: paillier.py:173-176, paillier.cc:799-805) on [100, 100] tensors, the four cases
encode -> encrypt -> decrypt -> decode, encrypted + plain, encrypted * plain, encrypted @ plain.

The reference asserts np.allclose; these tests keep that check and add the exact one: the decrypted
integers equal the exact integer results of the oracle's fixed-point encodings (sums aligned as
paillier.py:119-132, products as :135-138, matmul sums as paillier.cc:941-1051), and the decoded
floats equal the oracle's GMP-pinned hex decode of those integers bit for bit."""
import numpy as np
import pytest
import torch

from oracle import fxp
from oracle import paillier as P

pytestmark = pytest.mark.gpu

SHAPE = (100, 100)


@pytest.fixture(scope="module")
def kp():
    import efl
    efl.lib.require_gpu()
    k = efl.paillier.Keypair()
    k.generate_keypair()                     # reference defaults: 4096-bit n, 2048-bit a, g = 1
    # two 2048-bit primes: n has 4095 or 4096 bits (paillier.cc:851-877), the 4096-bit limb class
    assert k.key.n.bit_length() in (4095, 4096) and k.key.ln == 128
    assert k.key.a_bits == 2048 and k.key.group_size == 1
    return k


def _pair(seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*SHAPE, generator=g), torch.randn(*SHAPE, generator=g)


def _decode_exact(ints, E):
    return fxp.decode_hex([P.hx(v) for v in ints], np.asarray(E, dtype=np.int64).reshape(-1))


def test_encrypt_decrypt_encode_decode(kp):
    import efl
    a, _ = _pair(0)
    b = efl.paillier.fixedpoint.encode(a.cuda())
    m0 = b.mantissa.clone()
    b.mantissa = kp.encrypt(b.mantissa)
    b.mantissa = b.mantissa.decrypt()
    assert b.mantissa.to_ints() == m0.cpu().reshape(-1).tolist()      # decrypt() gives hex text
    y = efl.paillier.fixedpoint.decode(b).cpu()
    assert np.allclose(a.numpy(), y.numpy())
    Mo, Eo = fxp.encode(a.numpy())
    assert np.array_equal(y.numpy().view(np.uint32), fxp.decode(Mo, Eo).view(np.uint32))


def test_add(kp):
    import efl
    a, b = _pair(1)
    c1 = a + b
    fa = efl.paillier.fixedpoint.encode(a.cuda())
    fa.mantissa = kp.encrypt(fa.mantissa)
    c2 = fa + b.cuda()
    c2.mantissa = c2.mantissa.decrypt()
    ints = c2.mantissa.to_ints()
    c2 = efl.paillier.fixedpoint.decode(c2).cpu()
    assert np.allclose(c1.numpy(), c2.numpy())
    Ma, Ea = fxp.encode(a.numpy())
    Mb, Eb = fxp.encode(b.numpy())
    E = np.minimum(Ea, Eb).reshape(-1)
    sums = [(int(ma) << int(ea - e)) + (int(mb) << int(eb - e))
            for ma, ea, mb, eb, e in zip(Ma.reshape(-1), Ea.reshape(-1), Mb.reshape(-1), Eb.reshape(-1), E)]
    assert ints == sums
    assert np.array_equal(c2.numpy().reshape(-1).view(np.uint32), _decode_exact(sums, E).view(np.uint32))


def test_mul_scalar(kp):
    import efl
    a, b = _pair(2)
    c1 = a * b
    fa = efl.paillier.fixedpoint.encode(a.cuda())
    fa.mantissa = kp.encrypt(fa.mantissa)
    c2 = fa * b.cuda()
    c2.mantissa = c2.mantissa.decrypt()
    ints = c2.mantissa.to_ints()
    E2 = c2.exponent.cpu().numpy().reshape(-1)
    c2 = efl.paillier.fixedpoint.decode(c2).cpu()
    assert np.allclose(c1.numpy(), c2.numpy())
    Ma, Ea = fxp.encode(a.numpy())
    Mb, Eb = fxp.encode(b.numpy())
    assert np.array_equal(E2, (Ea + Eb).reshape(-1))
    prods = [int(x) * int(y) for x, y in zip(Ma.reshape(-1), Mb.reshape(-1))]
    assert ints == prods
    assert np.array_equal(c2.numpy().reshape(-1).view(np.uint32), _decode_exact(prods, E2).view(np.uint32))


def test_matmul(kp):
    import efl
    a, b = _pair(3)
    c1 = a @ b
    fa = efl.paillier.fixedpoint.encode(a.cuda())
    fa.mantissa = kp.encrypt(fa.mantissa)
    c2 = fa @ b.cuda()
    c2.mantissa = c2.mantissa.decrypt()
    ints = c2.mantissa.to_ints()
    Ez = c2.exponent.cpu().numpy()
    c2 = efl.paillier.fixedpoint.decode(c2).cpu()
    assert np.allclose(c1.numpy(), c2.numpy(), 1e-5, 1e-4)
    Ma, Ea = fxp.encode(a.numpy())
    Mb, Eb = fxp.encode(b.numpy())
    ex = Ea[:, :, None] + Eb[None, :, :]                       # [u, v, w]
    assert np.array_equal(Ez, ex.min(axis=1))
    u, v = Ma.shape
    w = Mb.shape[1]
    Ma_l, Mb_l = Ma.tolist(), Mb.tolist()
    sh = (ex - ex.min(axis=1, keepdims=True)).tolist()
    sums = [sum((Ma_l[i][j] * Mb_l[j][q]) << sh[i][j][q] for j in range(v)) for i in range(u) for q in range(w)]
    assert ints == sums
    assert np.array_equal(c2.numpy().reshape(-1).view(np.uint32), _decode_exact(sums, Ez).view(np.uint32))
