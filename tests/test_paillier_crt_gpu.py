"""The key owner's CRT encryption (efl_pl_crt_join, KeyBlock.crt_keys): hs^(a') mod n^2 from the
fixed-base exponentiations mod p^2 and mod q^2 and a Garner join must give the public-key path's
ciphertexts bit for bit (the reference's Encrypt, paillier.cc:103-131, works mod n^2 only)."""
import json
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import paillier as P
from oracle import philox

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)
CRT_KEYS = [k for k in KAT["keys"] if k["n_bytes"] >= 128]   # 512-bit n: 256-bit primes, no CRT class


def ids(k):
    return f"n{8 * k['n_bytes']}"


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


def keypair(efl, k, g=1, seed=1234, private=True):
    kp = efl.paillier.Keypair(seed=seed)
    kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, g,
                     int(k["p"], 16) if private else None, int(k["q"], 16) if private else None)
    return kp


def limbs(vals, L):
    return torch.from_numpy(np.stack([np.frombuffer(v.to_bytes(4 * L, "little"), "<u4") for v in vals])
                            .view(np.int32)).cuda()


def ints(t):
    a = t.cpu().numpy().view("<u4")
    return [int.from_bytes(r.tobytes(), "little") for r in a]


@pytest.mark.parametrize("k", CRT_KEYS, ids=ids)
def test_crt_join(efl, k):
    """z = q^2 yp + p^2 yq mod n^2, including sums at and above n^2 and above 2^(64 ln)."""
    from efl.privacy import paillier_cipher as pc
    kp = keypair(efl, k)
    key = kp.key
    p, q = key.p, key.q                       # as the key block orders them (q < 2p)
    p2, q2, n2 = p * p, q * q, key.n * key.n
    rng = random.Random(k["n_bytes"])
    yp = [0, 1, p2 - 1, 0, p2 - 1, 5, 0] + [rng.randrange(p2) for _ in range(250)]
    yq = [0, 1, q2 - 1, q2 - 1, 0, 7, 1] + [rng.randrange(q2) for _ in range(250)]
    z = torch.empty((len(yp), key.lc), dtype=torch.int32, device="cuda")
    Yp, Yq = limbs(yp, key.ln), limbs(yq, key.ln)
    rc = pc._lib.efl_pl_crt_join(*key.args(), Yp.data_ptr(), Yq.data_ptr(), None, z.data_ptr(), len(yp),
                                 torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    got = ints(z)
    over = 0
    for a, b, g in zip(yp, yq, got):
        s = q2 * a + p2 * b
        over += s >= n2
        assert g == s % n2
    assert over > 0
    # x -> (x (q^2)^-1 mod p^2, x (p^2)^-1 mod q^2) -> x
    xs = [0, 1, n2 - 1] + [rng.randrange(n2) for _ in range(100)]
    ip, iq = pow(q2, -1, p2), pow(p2, -1, q2)
    Yp, Yq = limbs([x % p2 * ip % p2 for x in xs], key.ln), limbs([x % q2 * iq % q2 for x in xs], key.ln)
    z = torch.empty((len(xs), key.lc), dtype=torch.int32, device="cuda")
    assert pc._lib.efl_pl_crt_join(*key.args(), Yp.data_ptr(), Yq.data_ptr(), None, z.data_ptr(), len(xs), None) == 0
    assert ints(z) == xs
    # with the plaintext: v is hsa R, z = (1 + |m| n)^(sign) hsa mod n^2 (in place of z's own words)
    R = 1 << (32 * key.lc)
    ms = [rng.randrange(-2**63, 2**63) for _ in xs]
    ms[:4] = [0, -1, 2**63 - 1, -2**63]
    m = torch.tensor(ms, dtype=torch.int64, device="cuda")
    assert pc._lib.efl_pl_crt_join(*key.args(), Yp.data_ptr(), Yq.data_ptr(), m.data_ptr(), z.data_ptr(), len(xs),
                                   None) == 0
    Rinv = pow(R, -1, n2)
    for x, mi, got in zip(xs, ms, ints(z)):
        gm = (1 + abs(mi) * key.n) % n2
        if mi < 0:
            gm = pow(gm, -1, n2)
        assert got == gm * x * Rinv % n2


@pytest.mark.parametrize("k", CRT_KEYS, ids=ids)
def test_crt_encrypt_equals_public_path(efl, k):
    g = 3 if k["n_bytes"] <= 128 else 1
    rng = np.random.default_rng(k["n_bytes"])
    m = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, 777, dtype=np.int64))
    m[:4] = torch.tensor([0, -1, 2**63 - 1, -2**63])
    kp = keypair(efl, k, g=g, seed=77)
    assert kp.key.crt_keys() is not None
    crt = kp.encrypt(m, counter_base=11).tensor.to_hex().strings()
    kp.crt_encrypt = False
    pub = kp.encrypt(m, counter_base=11).tensor.to_hex().strings()
    assert crt == pub
    kp.crt_encrypt = True
    assert torch.equal(kp.decrypt(kp.encrypt(m), dtype=torch.int64).cpu(), m)
    # fbpowm: Philox draws and given exponents
    f1 = kp.fbpowm(n=300, counter_base=3).to_hex().strings()
    ra = random.Random(5)
    a = [ra.getrandbits(k["a_bits"]) for _ in range(40)] + [0, 1]
    f2 = kp.fbpowm(a=a).to_hex().strings()
    kp.crt_encrypt = False
    assert kp.fbpowm(n=300, counter_base=3).to_hex().strings() == f1
    assert kp.fbpowm(a=a).to_hex().strings() == f2
    okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, g)
    for i in (0, 123, 299):
        assert f1[i] == P.hx(P.fbpowm(okp.hs, okp.n2, philox.draw_a(77, 3 + i, k["a_bits"]), g))


@pytest.mark.parametrize("c", [0, 8, 16, 32])
def test_crt_encrypt_every_family(efl, c):
    """The join's g(m) product runs the main key's encryption kernel with hsa in Montgomery form:
    every kernel family of the 1024-bit key (one lane, sliced C = 8 / 16 / 32) gives the n^2 path's
    ciphertexts."""
    from efl.privacy import paillier_cipher as pc
    k = CRT_KEYS[0]
    ln = k["n_bytes"] // 4
    m = torch.tensor([0, 1, -1, 2**63 - 1, -2**63] + list(range(-60, 60, 7)), dtype=torch.int64)
    prev = pc.set_kernel_slicing(ln, False, c)
    try:
        kp = keypair(efl, k, seed=5)
        crt = kp.encrypt(m, counter_base=9).tensor.to_hex().strings()
        kp.crt_encrypt = False
        assert kp.encrypt(m, counter_base=9).tensor.to_hex().strings() == crt
    finally:
        pc.set_kernel_slicing(ln, False, prev)


def test_crt_mixed_hsa_rows(efl):
    """hsa given for some rows, "0" for others: the zero rows draw their own index's counter
    through the CRT path and equal the public path's."""
    k = CRT_KEYS[0]
    kp = keypair(efl, k, seed=4321)
    N = 50
    zero_rows = [0, 3, 4, 5, 31, 49]
    given = kp.fbpowm(a=[999 + i for i in range(N)]).to_hex().strings()
    hsa = ["0" if i in zero_rows else given[i] for i in range(N)]
    m = torch.arange(-25, 25, dtype=torch.int64)
    c1 = kp.encrypt(m, hsa=hsa, counter_base=100).tensor.to_hex().strings()
    kp.crt_encrypt = False
    c2 = kp.encrypt(m, hsa=hsa, counter_base=100).tensor.to_hex().strings()
    assert c1 == c2
    assert kp.decrypt(efl.HexTensor.from_strings(c1), dtype=torch.int64).cpu().tolist() == m.tolist()


def test_crt_not_used_without_private_key_or_class(efl, monkeypatch):
    assert keypair(efl, CRT_KEYS[0], private=False).key.crt_keys() is None
    assert keypair(efl, KAT["keys"][0]).key.crt_keys() is None       # 512-bit n
    monkeypatch.setenv("EFL_PL_CRT_ENCRYPT", "0")
    assert keypair(efl, CRT_KEYS[0]).key.crt_keys() is None


def test_crt_not_used_for_private_key_not_factoring_n(efl):
    """A private key whose p q != n: the reference's Encrypt (mod n^2 only) still gives valid
    ciphertexts of n, so the key owner's encryption must take the public-key path, not the CRT
    join (which would be wrong mod n^2)."""
    from efl import errors
    from efl.privacy import paillier_cipher as pc
    k = CRT_KEYS[0]
    _, _, p2, q2 = pc.generate_keypair_ints(k["n_bytes"], 24, random.Random(99))
    kp = efl.paillier.Keypair(seed=8)
    kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, p2, q2)
    assert kp.key.crt_keys() is None
    m = torch.tensor([0, 5, -7, 2**62, -2**63], dtype=torch.int64)
    got = kp.encrypt(m, counter_base=3).tensor.to_hex().strings()
    pub = keypair(efl, k, g=1, seed=8, private=False)
    assert got == pub.encrypt(m, counter_base=3).tensor.to_hex().strings()
    with pytest.raises(errors.InvalidArgumentError):
        efl.paillier.Keypair(seed=1).set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1,
                                                   p2, p2)


def test_owner_table_deferred_until_walked(efl):
    """The key owner's encryptions go by CRT, so its n^2 fixed-base table is built only when the
    public-key path is asked for (crt_encrypt = False here): the raw ABI refuses the walk before
    that (no table, no fault), and both paths give the same ciphertexts after it."""
    from efl.privacy import paillier_cipher as pc
    k = CRT_KEYS[0]
    kp = keypair(efl, k, seed=21)
    key = kp.key
    assert not key.has_table and key.crt_capable()
    m = torch.tensor([3, -4, 2**40, 0], dtype=torch.int64)
    crt = kp.encrypt(m, counter_base=5).tensor.to_hex().strings()
    assert not key.has_table                                   # CRT needs only the sub-tables
    subs = key.crt_keys()
    budget = pc.table_max_bytes()
    assert all(sk.block_bytes <= budget // 2 + (1 << 20) for sk in subs)     # half of the cap each
    ct = torch.empty((4, key.lc), dtype=torch.int32, device="cuda")
    md = m.cuda()
    rc = pc._lib.efl_pl_encrypt(*key.args(), md.data_ptr(), None, ct.data_ptr(), 4, 21, 5, None)
    assert rc != 0                                             # ABORTED: no fixed-base table yet
    kp.crt_encrypt = False
    pub = kp.encrypt(m, counter_base=5).tensor.to_hex().strings()
    assert key.has_table and pub == crt
    assert pc._lib.efl_pl_encrypt(*key.args(), md.data_ptr(), None, ct.data_ptr(), 4, 21, 5, None) == 0
    # a public-key holder builds its table at once
    assert keypair(efl, k, private=False).key.has_table


def test_crt_keys_survive_set_private_key(efl):
    k = CRT_KEYS[0]
    kp = keypair(efl, k)
    subs = kp.key.crt_keys()
    kp.set_private_key(k["p"], k["q"])
    assert kp.key.crt_keys() is subs


def test_crt_join_errors(efl):
    from efl.privacy import paillier_cipher as pc
    kp = keypair(efl, CRT_KEYS[0], private=False)
    z = torch.empty((1, kp.key.lc), dtype=torch.int32, device="cuda")
    rc = pc._lib.efl_pl_crt_join(*kp.key.args(), z.data_ptr(), z.data_ptr(), None, z.data_ptr(), 1, None)
    assert rc != 0
