"""GPU: the row-split fixed-base walks (efl_pl_tune(ln, 4, P); csrc/paillier_sliced.hip
k_walk28_part / k_walk28_join). A launch below 4 waves per SIMD splits every element's walk over P
disjoint ranges of table rows and multiplies the parts in a second launch; the ciphertexts and
hs^(a') must be those of the unsplit walk, bit for bit, for every P, group size, table window, the
public-key path and the key owner's CRT sub-keys (the reference: FixedBasePowm::mpz_fbpowm,
gmp_utils.cc:107-144, and Encrypt, paillier.cc:103-131), including exponents whose windows are zero
over a whole part (a = 0, 1, powers of two)."""
import contextlib
import json
import os
import random

import pytest
import torch

from conftest import GOLDEN
from oracle import paillier as P
from oracle import philox

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


@contextlib.contextmanager
def parts(efl, ln, p):
    lib = efl.lib.raw()
    prev = lib.efl_pl_tune(ln, 4, p)
    assert prev >= 0
    try:
        yield
    finally:
        lib.efl_pl_tune(ln, 4, prev)


def test_tune_knob(efl):
    lib = efl.lib.raw()
    assert lib.efl_pl_tune(32, 4, -1) == 0               # chosen per launch by default
    assert lib.efl_pl_tune(32, 4, 6) == -3
    prev = lib.efl_pl_tune(32, 4, 3)
    assert lib.efl_pl_tune(32, 4, prev) == 3


@pytest.mark.parametrize("k", [k for k in KAT["keys"] if k["n_bytes"] in (64, 128, 256)],
                         ids=lambda k: f"n{8 * k['n_bytes']}")
def test_every_split_gives_the_unsplit_walk(efl, k):
    ln = k["n_bytes"] // 4
    rng = random.Random(k["n_bytes"])
    a_bits = k["a_bits"]
    avals = [0, 1, 2, 1 << (a_bits - 1), (1 << a_bits) - 1, 1 << (a_bits // 2)] + \
        [rng.getrandbits(a_bits) for _ in range(120)]
    m = torch.tensor([0, -1, 2**63 - 1, -2**63] + list(range(-60, 60)), dtype=torch.int64)
    for g in (1, 3):
        for owner in (False, True):
            kp = efl.paillier.Keypair(seed=31)
            kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), a_bits // 8, g,
                             int(k["p"], 16) if owner else None, int(k["q"], 16) if owner else None)
            out = {}
            for p in (1, 2, 3, 4, 5, 0):
                with parts(efl, ln, p), parts(efl, ln // 2 if ln > 16 else 16, p):
                    f1 = kp.fbpowm(a=avals).to_hex().strings()
                    f2 = kp.fbpowm(n=200, counter_base=7).to_hex().strings()
                    c = kp.encrypt(m, counter_base=500).tensor.to_hex().strings()
                out[p] = (f1, f2, c)
            for p in (2, 3, 4, 5, 0):
                assert out[p] == out[1], (g, owner, p)
            okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), a_bits // 8, g)
            for j in (0, 1, 3, 5, 77):
                assert out[1][0][j] == P.hx(P.fbpowm(okp.hs, okp.n2, avals[j], g))
            for j in (0, 199):
                assert out[1][1][j] == P.hx(P.fbpowm(okp.hs, okp.n2, philox.draw_a(31, 7 + j, a_bits), g))
            for j in (0, 3, 50):
                want = P.encrypt(okp, int(m[j]), P.fbpowm(okp.hs, okp.n2, philox.draw_a(31, 500 + j, a_bits), g))
                assert out[1][2][j] == P.hx(want)


def test_mnist_shape_split_round_trip(efl):
    """The paillier_mnist activation ([256, 392], 100,352 mantissas), 1024-bit key: the split chosen
    per launch (P = 3 on 256 CUs for the public-key holder's two-lane n^2 walk; the key owner's
    one-lane CRT walks stay whole) gives the unsplit ciphertexts, which decrypt to the plaintext."""
    k = next(k for k in KAT["keys"] if k["n_bytes"] == 128)
    ln = 32
    g = torch.Generator(device="cuda").manual_seed(5)
    m = torch.randint(-2**40, 2**40, (256 * 392,), dtype=torch.int64, device="cuda", generator=g)
    owner = efl.paillier.Keypair(seed=9)
    owner.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), 64, 10, int(k["p"], 16), int(k["q"], 16))
    holder = efl.paillier.Keypair(seed=9)
    holder.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), 64, 10)
    c_auto = owner.encrypt(m, counter_base=1000).tensor.limbs
    h_auto = holder.encrypt(m, counter_base=1000).tensor.limbs
    with parts(efl, ln, 1), parts(efl, 16, 1):
        c_one = owner.encrypt(m, counter_base=1000).tensor.limbs
        h_one = holder.encrypt(m, counter_base=1000).tensor.limbs
    assert torch.equal(c_auto, c_one) and torch.equal(h_auto, h_one) and torch.equal(c_auto, h_auto)
    back = owner.decrypt(efl.privacy.paillier_cipher.CipherTensor(c_auto, (m.numel(),), owner.key), dtype=torch.int64)
    assert torch.equal(back, m)
