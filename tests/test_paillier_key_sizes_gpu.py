"""Key sizes between and past the round-3 limb classes. The reference takes any n_bytes
(GeneratePaillierKeypair, paillier.cc:799-913: primes of n_bytes * 4 bits); the build runs a key in
the smallest limb class that holds n and p^2 (512 / 1024 / 2048 / 4096 / 8192-bit n: KeyBlock's
_LIMB_CLASSES), the numbers zero-padded to it, so 768-, 1000-, 1536- and 3072-bit keys (3072 bits is
the usual 128-bit security level) run in the 1024-, 1024-, 2048- and 4096-bit kernels. Montgomery
arithmetic only needs the modulus below R, so the results must be the oracle's bit for bit: fresh
randomness encryption by the public path and by CRT, decryption, the homomorphic ops and matmul.
8192-bit keys (round 4) run their n^2 ops over 16 lanes per number and decrypt over 8."""
import random

import numpy as np
import pytest
import torch

from oracle import paillier as P
from oracle import philox

pytestmark = pytest.mark.gpu

# (n_bytes, limb class of n)
SIZES = [(96, 32), (125, 32), (192, 64), (384, 128), (1024, 256)]


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


@pytest.fixture(scope="module", params=SIZES, ids=[f"n{8 * s[0]}" for s in SIZES])
def keys(request, efl):
    n_bytes, ln = request.param
    owner = efl.paillier.Keypair(seed=17)
    owner.generate_keypair(n_bytes=n_bytes, a_bytes=n_bytes // 2, rng=random.Random(n_bytes))
    k = owner.key
    assert k.ln == ln and k.n.bit_length() in (8 * n_bytes - 1, 8 * n_bytes)
    public = efl.paillier.Keypair(seed=17)
    public.set_keys_ints(k.n, k.hs, n_bytes // 2, 1)
    okp = P.Keypair(k.n, k.hs, n_bytes // 2, 1, k.p, k.q)
    return owner, public, okp


def _ms(count, seed):
    rng = np.random.default_rng(seed)
    m = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, count, dtype=np.int64))
    m[:4] = torch.tensor([0, -1, 2**63 - 1, -2**63])
    return m


def test_encrypt_public_and_crt_match_the_oracle(keys):
    owner, public, okp = keys
    m = _ms(200, 1)
    ct_pub = public.encrypt(m, counter_base=300)
    ct_own = owner.encrypt(m, counter_base=300)      # the key owner's CRT path
    got = ct_pub.tensor.to_hex().strings()
    assert ct_own.tensor.to_hex().strings() == got
    a_bits = public.key.a_bits
    for i in (0, 1, 2, 3, 50, 199):
        a = philox.draw_a(17, 300 + i, a_bits)
        assert got[i] == P.hx(P.encrypt(okp, int(m[i]), P.fbpowm(okp.hs, okp.n2, a, 1))), i
    assert torch.equal(owner.decrypt(ct_pub, dtype=torch.int64).cpu(), m)
    assert owner.decrypt(ct_pub).strings()[:4] == [P.hx(v) for v in (0, -1, 2**63 - 1, -2**63)]


def test_decrypt_every_family(keys):
    from test_paillier_gpu import SLICINGS, family
    owner, public, okp = keys
    m = _ms(64, 2)
    ct = public.encrypt(m)
    ln = owner.key.ln
    for c in SLICINGS[ln][1]:
        with family(ln, True, c):
            assert torch.equal(owner.decrypt(ct, dtype=torch.int64).cpu(), m), c


def test_homomorphic_ops_match_the_oracle(keys):
    owner, public, okp = keys
    m = _ms(6, 3)
    ct = public.encrypt(m)
    cs = ct.tensor.to_hex().to_ints()
    ys = [5, -3, 0, 1, 2**40, -(2**33)]
    assert public.add(ct.tensor, ct.tensor).to_hex().to_ints() == [P.add(okp, c, c) for c in cs]
    assert public.mul_scalar(ct.tensor, torch.tensor(ys)).to_hex().to_ints() == \
        [P.mul_scalar(okp, c, y) for c, y in zip(cs, ys)]
    sh = [0, 1, 7, 64, 130, 3]
    assert public.mul_exp2(ct.tensor, torch.tensor(sh)).to_hex().to_ints() == \
        [P.mul_exp2(okp, c, y) for c, y in zip(cs, sh)]
    assert public.invert(ct.tensor).to_hex().to_ints() == [P.invert(okp, c) for c in cs]
    xe, ye = [0, 5, -5, 70, 2, 3], [0, 0, 1, 2, 9, -9]
    z, ze = public.shift_add(ct.tensor, torch.tensor(xe), ct.tensor, torch.tensor(ye))
    want = [P.fixedpoint_add(okp, c, a, c, b) for c, a, b in zip(cs, xe, ye)]
    assert z.to_hex().to_ints() == [w[0] for w in want] and ze.cpu().tolist() == [w[1] for w in want]


def test_matmul_matches_the_oracle(keys):
    owner, public, okp = keys
    rng = np.random.default_rng(4)
    u, v, w = 3, 4, 2
    m = torch.from_numpy(rng.integers(-2**20, 2**20, (u, v)))
    ct = public.encrypt(m)
    xe = rng.integers(-30, -10, (u, v))
    ym = rng.integers(-2**20, 2**20, (v, w))
    ye = rng.integers(-25, -12, (v, w))
    zm, ze = public.matmul(ct.tensor, torch.from_numpy(xe), torch.from_numpy(ym), torch.from_numpy(ye))
    xs = [[int(s, 16) for s in row] for row in np.array(ct.tensor.to_hex().strings()).reshape(u, v)]
    om, oe = P.matmul(okp, xs, xe.tolist(), ym.tolist(), ye.tolist())
    assert ze.cpu().tolist() == oe
    assert zm.to_hex().to_ints() == [c for row in om for c in row]
    dec = owner.decrypt(zm, dtype="string").to_ints()
    assert dec == [sum(int(m[i, j]) * int(ym[j, q]) * 2 ** int(xe[i, j] + ye[j, q] - oe[i][q]) for j in range(v))
                   for i in range(u) for q in range(w)]
