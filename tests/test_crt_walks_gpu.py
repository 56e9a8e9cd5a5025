"""GPU: the key owner's CRT encryption with an element's two walks in one wave (efl_pl_tune(ln, 5, 2),
the default's choice; csrc/paillier_sliced.hip k_crt_pair_whole / k_crt_pair_part /
k_crt_pair_tjoin): each lane makes its walk start, the CRT join is done at the wave's end, and only
the waves past the launch's whole rounds are split over table rows and joined. The ciphertexts and hs^(a') must be those of the
per-key walks and efl_pl_crt_join (efl_pl_tune(ln, 5, 1)), bit for bit, at
every element count: no tail, a tail split P ways, an element count below one round (everything
split), counts that leave the last wave of each key partly empty. The reference: Encrypt,
paillier.cc:103-131, and FixedBasePowm::mpz_fbpowm, gmp_utils.cc:107-144."""
import contextlib
import json
import os

import pytest
import torch

from conftest import GOLDEN
from oracle import paillier as P
from oracle import philox

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)
K1024 = next(k for k in KAT["keys"] if k["n_bytes"] == 128)


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


@pytest.fixture(scope="module")
def owner(efl):
    kp = efl.paillier.Keypair(seed=11)
    kp.set_keys_ints(int(K1024["n"], 16), int(K1024["hs"], 16), 64, 10, int(K1024["p"], 16), int(K1024["q"], 16))
    return kp


@contextlib.contextmanager
def mode(efl, v):
    lib = efl.lib.raw()
    prev = lib.efl_pl_tune(16, 5, v)
    assert prev >= 0
    try:
        yield
    finally:
        lib.efl_pl_tune(16, 5, prev)


def test_tune_knob(efl):
    lib = efl.lib.raw()
    assert lib.efl_pl_tune(16, 5, -1) == 0               # chosen per launch by default
    assert lib.efl_pl_tune(16, 5, 3) < 0
    prev = lib.efl_pl_tune(16, 5, 1)
    assert lib.efl_pl_tune(16, 5, prev) == 1


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4097, 32768, 50176, 100352, 100352 + 5 * 64 + 3, 131072 + 17,
                               262144])
def test_paired_lanes_equal_per_key(efl, owner, n):
    g = torch.Generator(device="cuda").manual_seed(n)
    m = torch.randint(-2**40, 2**40, (n,), dtype=torch.int64, device="cuda", generator=g)
    out = {}
    for v in (0, 1, 2):                                   # chosen, per key, paired lanes
        with mode(efl, v):
            out[v] = (owner.encrypt(m, counter_base=3 * n).tensor.limbs, owner.fbpowm(n=n, counter_base=5).limbs)
    for v in (0, 2):
        assert torch.equal(out[v][0], out[1][0]) and torch.equal(out[v][1], out[1][1]), v


def test_paired_lanes_match_oracle_and_decrypt(efl, owner):
    """The paillier_mnist activation ([256, 392]): ciphertexts from the split tail's elements (the
    last ones) and from whole walks equal the oracle's Encrypt, and the tensor decrypts."""
    n = 256 * 392
    g = torch.Generator(device="cuda").manual_seed(3)
    m = torch.randint(-2**40, 2**40, (n,), dtype=torch.int64, device="cuda", generator=g)
    with mode(efl, 0):
        ct = owner.encrypt(m, counter_base=900)
    hexes = ct.tensor.to_hex().strings()
    okp = P.Keypair(int(K1024["n"], 16), int(K1024["hs"], 16), 64, 10)
    a_bits = 8 * 64
    for j in (0, 1, 4095, n - 4096, n - 2049, n - 2048, n - 65, n - 64, n - 1):   # tail from n - 2048
        want = P.encrypt(okp, int(m[j]), P.fbpowm(okp.hs, okp.n2, philox.draw_a(11, 900 + j, a_bits), 10))
        assert hexes[j] == P.hx(want), j
    back = owner.decrypt(ct, dtype=torch.int64)
    assert torch.equal(back, m)


def test_given_exponents(efl, owner):
    """fbpowm of given a (the hsa path of efl_pl_ctx_fbpowm) through the paired lanes: zero, one, powers of
    two and all-ones exponents, whose windows vanish over whole parts."""
    a_bits = 512
    base = [0, 1, 2, 1 << (a_bits - 1), (1 << a_bits) - 1, 1 << 256, (1 << 64) - 1]
    avals = (base * 200)[:1300]
    with mode(efl, 1):
        f1 = owner.fbpowm(a=avals).to_hex().strings()
    for v in (0, 2):
        with mode(efl, v):
            assert owner.fbpowm(a=avals).to_hex().strings() == f1, v
    f0 = f1
    okp = P.Keypair(int(K1024["n"], 16), int(K1024["hs"], 16), 64, 10)
    for j in range(len(base)):
        assert f0[j] == P.hx(P.fbpowm(okp.hs, okp.n2, avals[j], 10)), j


def test_extreme_plaintexts(efl, owner):
    """int64 extremes and zero through the paired lanes' in-kernel starts ((1 +- |m| n) mod x^2 with
    |m| up to 2^63): the per-key path's ciphertexts, and the plaintexts back."""
    ext = [0, 1, -1, 2**63 - 1, -2**63, -2**63 + 1, 2**62, -2**62, 2**40, -2**40]
    m = torch.tensor((ext * 500)[:4999], dtype=torch.int64, device="cuda")
    out = {}
    for v in (1, 2):
        with mode(efl, v):
            out[v] = owner.encrypt(m, counter_base=77)
    assert torch.equal(out[1].tensor.limbs, out[2].tensor.limbs)
    assert torch.equal(owner.decrypt(out[2], dtype=torch.int64), m)


@pytest.mark.parametrize("tail", [0, 1, 2, 4, 8, 16])
# tails of 1 to 2,371 elements (S = 16 or 8 in mode 0), 8,192 (S = 4), 16,384 (S = 2) and 17,408
# (no split: every wave whole) past 32,768 elements (the whole rounds of 1,024 SIMDs)
@pytest.mark.parametrize("n", [1, 17, 65, 2048, 32769, 40960, 49152, 50176, 100352, 100352 + 5 * 64 + 3])
def test_tree_tail_equals_per_key(efl, owner, tail, n):
    """The tail past the whole rounds as a product tree across lanes, in the whole rounds' launch
    (efl_pl_tune(ln, 6, 0), the default) or after it (2-16, a fixed S), or as the round-5
    split-and-join launches (1): ciphertexts and
    hs^(a') equal the per-key walks' bit for bit, for tails of every size (a lone element, a part-empty
    wave, the MNIST activation's 2,048 elements, and a count whose tail is neither)."""
    lib = efl.lib.raw()
    g = torch.Generator(device="cuda").manual_seed(n + 1)
    m = torch.randint(-2**40, 2**40, (n,), dtype=torch.int64, device="cuda", generator=g)
    with mode(efl, 1):
        want = (owner.encrypt(m, counter_base=7).tensor.limbs, owner.fbpowm(n=n, counter_base=9).limbs)
    prev = lib.efl_pl_tune(16, 6, tail)
    assert prev >= 0
    try:
        with mode(efl, 2):
            got = (owner.encrypt(m, counter_base=7).tensor.limbs, owner.fbpowm(n=n, counter_base=9).limbs)
    finally:
        lib.efl_pl_tune(16, 6, prev)
    assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1])


def test_tree_tail_knob(efl):
    lib = efl.lib.raw()
    assert lib.efl_pl_tune(16, 6, -1) == 0               # the tree waves inside the whole launch by default
    assert lib.efl_pl_tune(16, 6, 3) < 0 and lib.efl_pl_tune(16, 6, 32) < 0
