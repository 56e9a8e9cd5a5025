"""CPU: pin the Paillier oracle (oracle/paillier.py, oracle/philox.py).

* tests/golden/paillier_kat.json was produced by GMP 6.2.1 in the reference's call order
  (make_paillier_golden.py); the Python-int restatement must reproduce every vector, and the GMP
  harness must reproduce a sample again at test time.
* Philox4x32-10 against the Random123 known-answer vectors (Salmon et al., SC'11).
* The survey's fbpowm finding: g = 1 gives hs^a; g > 1 gives
  hs^(groupwise bit-reversed a).
"""
import json
import os
import random

import pytest

from conftest import GOLDEN
from oracle import paillier as P
from oracle import philox

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)


def kp_of(k):
    return P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))


@pytest.mark.parametrize("k", KAT["keys"], ids=lambda k: f"n{8 * k['n_bytes']}")
def test_kat_restatement(k):
    kp = kp_of(k)
    for v in k["vectors"]:
        hsa = int(v["hsa"], 16)
        assert P.fbpowm(kp.hs, kp.n2, int(v["a"], 16), v["g"]) == hsa
        c = P.encrypt(kp, v["m"], hsa)
        assert P.hx(c) == v["c"]
        assert P.hx(P.decrypt(kp, c)) == v["d"] and P.decrypt(kp, c) == v["m"]
    c0, c1 = int(k["vectors"][5]["c"], 16), int(k["vectors"][6]["c"], 16)
    assert P.hx(P.add(kp, c0, c1)) == k["ops"]["add"]
    assert P.hx(P.mul_scalar(kp, c0, 7)) == k["ops"]["mul_scalar_7"]
    assert P.hx(P.mul_exp2(kp, c1, 5)) == k["ops"]["mul_exp2_5"]
    assert P.decrypt(kp, int(k["ops"]["add"], 16)) == k["vectors"][5]["m"] + k["vectors"][6]["m"]


OPS_SCALARS = {"mul_scalar_7": 7, "mul_scalar_0": 0, "mul_scalar_neg": -123456789,
               "mul_scalar_i64max": 2**63 - 1, "mul_scalar_i64min": -2**63}


@pytest.mark.parametrize("k", KAT["keys"], ids=lambda k: f"n{8 * k['n_bytes']}")
def test_ops_restatement_matches_gmp_vectors(k):
    """The GMP-computed op vectors (paillier.cc:157-285, :722-733; the signed-scalar route through
    mpz_invert at :201-211) against the Python-int restatement, and what they decrypt to."""
    kp = kp_of(k)
    o = k["ops"]
    c0, c1 = int(k["vectors"][5]["c"], 16), int(k["vectors"][6]["c"], 16)
    m0, m1 = k["vectors"][5]["m"], k["vectors"][6]["m"]
    for name, y in OPS_SCALARS.items():
        assert P.hx(P.mul_scalar(kp, c0, y)) == o[name], name
        want = m0 * y % kp.n
        want = want - kp.n if want > kp.max_ else want
        assert P.decrypt(kp, int(o[name], 16)) == want, name
    assert P.hx(P.mul_scalar_hex(kp, c0, o["mul_scalar_hex_text"])) == o["mul_scalar_hex"]
    for e in (0, 5, 77):
        assert P.hx(P.mul_exp2(kp, c1, e)) == o[f"mul_exp2_{e}"]
    assert P.hx(P.invert(kp, c0)) == o["invert"]
    assert P.decrypt(kp, int(o["invert"], 16)) == -m0
    assert P.add(kp, c0, int(o["invert"], 16)) == 1


@pytest.mark.parametrize("k", KAT["keys"], ids=lambda k: f"n{8 * k['n_bytes']}")
def test_matmul_restatement_matches_gmp_vectors(k):
    """PaillierMatmul (paillier.cc:987-1035) through GMP against the Python restatement, and the
    plaintext it decrypts to: sum_j xm*ym*2^(xe+ye-min)."""
    kp = kp_of(k)
    mm = k["matmul"]
    u, v, w = mm["shape"]
    xm = [[int(k["vectors"][mm["x_vectors"][i * v + j]]["c"], 16) for j in range(v)] for i in range(u)]
    ms = [[k["vectors"][mm["x_vectors"][i * v + j]]["m"] for j in range(v)] for i in range(u)]
    zm, ze = P.matmul(kp, xm, mm["xe"], mm["ym"], mm["ye"])
    assert [[P.hx(c) for c in r] for r in zm] == mm["zm"] and ze == mm["ze"]
    for i in range(u):
        for q in range(w):
            want = sum(ms[i][j] * mm["ym"][j][q] << (mm["xe"][i][j] + mm["ye"][j][q] - ze[i][q]) for j in range(v))
            want %= kp.n
            want = want - kp.n if want > kp.max_ else want
            assert P.decrypt(kp, int(mm["zm"][i][q], 16)) == want


def test_ops_gmp_live():
    """The GMP harness reproduces the committed op and matmul vectors at test time (1024-bit key)."""
    k = KAT["keys"][1]
    n = int(k["n"], 16)
    o = k["ops"]
    c0, c1 = int(k["vectors"][5]["c"], 16), int(k["vectors"][6]["c"], 16)
    assert P.gmp_add(n, c0, c1) == o["add"]
    for name, y in OPS_SCALARS.items():
        assert P.gmp_mul_scalar(n, c0, y) == o[name]
    assert P.gmp_mul_scalar(n, c0, o["mul_scalar_hex_text"]) == o["mul_scalar_hex"]
    assert P.gmp_mul_exp2(n, c1, 77) == o["mul_exp2_77"]
    with pytest.raises(ValueError):
        P.gmp_mul_exp2(n, c1, -1)
    assert P.gmp_invert(n, c0) == o["invert"]
    mm = k["matmul"]
    u, v, w = mm["shape"]
    xm = [[int(k["vectors"][mm["x_vectors"][i * v + j]]["c"], 16) for j in range(v)] for i in range(u)]
    assert P.gmp_matmul(n, xm, mm["xe"], mm["ym"], mm["ye"]) == (mm["zm"], mm["ze"])


def test_fbpowm_gmp_pins_every_key_size():
    """Every KAT's hsa (2048- and 4096-bit keys included) is GMP's mpz_fbpowm through the reference's
    table (gmp_utils.cc:56-144), recomputed live for a sample of each key."""
    for k in KAT["keys"]:
        kp = kp_of(k)
        for v in k["vectors"][:2]:
            assert P.gmp_fbpowm(kp.hs, kp.n2, k["a_bits"], v["g"], int(v["a"], 16)) == int(v["hsa"], 16)


def test_kat_gmp_live():
    k = KAT["keys"][1]
    n, p, q = int(k["n"], 16), int(k["p"], 16), int(k["q"], 16)
    for v in k["vectors"][:8]:
        assert P.gmp_encrypt(n, v["m"], int(v["hsa"], 16)) == v["c"]
        assert P.gmp_decrypt(p, q, int(v["c"], 16)) == v["d"]


def test_keygen_reproduces_kat_keys():
    """GMP keygen with the KAT's MT seed gives the KAT key (paillier.cc:843-896 procedure)."""
    k = KAT["keys"][0]
    n, hs, p, q = P.gmp_keygen(k["n_bytes"], k["mt_seed"])
    assert (P.hx(n), P.hx(hs), P.hx(p), P.hx(q)) == (k["n"], k["hs"], k["p"], k["q"])
    bits = k["n_bytes"] * 4
    for x in (p, q):
        assert x.bit_length() == bits and x & 3 == 3
    import math
    assert math.gcd(p - 1, q - 1) == 2


def test_fbpowm_group_reversal():
    k = KAT["keys"][1]
    kp = kp_of(k)
    rng = random.Random(3)
    for g in (1, 3, 10):
        for _ in range(1 if g == 10 else 4):
            a = rng.getrandbits(rng.randrange(1, 513))
            got = P.gmp_fbpowm(kp.hs, kp.n2, 512, g, a)
            assert got == P.fbpowm(kp.hs, kp.n2, a, g)
            if g == 1:
                assert got == pow(kp.hs, a, kp.n2)
    a = 0b110100110101
    assert P.group_reversed(a, 3) == 0b011001011101   # groups 101,110,100,011 reversed


def test_philox_known_answers():
    assert philox.philox4x32_10((0, 0, 0, 0), (0, 0)) == (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)
    f = 0xFFFFFFFF
    assert philox.philox4x32_10((f, f, f, f), (f, f)) == (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)
    assert philox.philox4x32_10((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0)) == \
        (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)
    a = philox.draw_a(5, 7, 300)
    assert a < 2**300


def test_encrypt_negative_is_inverse_trick():
    """(1+|m|n)^-1 mod n^2 == n^2 + 1 - |m| n  (what the GPU kernel uses instead of an inversion)."""
    kp = kp_of(KAT["keys"][1])
    for m in (1, 5, 2**63, 2**62 + 17):
        assert pow(1 + m * kp.n, -1, kp.n2) == kp.n2 + 1 - m * kp.n
