"""Key generation's host arithmetic (GeneratePaillierKeypairOp, paillier.cc:833-904) in
libefl_hip.so's native host code (csrc/keygen.cpp: efl_host_powm, efl_host_probable_primes) and the
Python search around it (efl.privacy.paillier_cipher.generate_keypair_ints). No GPU needed."""
import math
import random

import pytest

from efl.privacy import paillier_cipher as pc


def test_host_powm_matches_python_pow():
    r = random.Random(5)
    for _ in range(60):
        m = r.getrandbits(r.randrange(2, 4200)) | 1
        b = r.randrange(0, m)
        e = r.getrandbits(r.randrange(0, 1200))
        assert pc.host_powm(b, e, m) == pow(b, e, m)
    assert pc.host_powm(0, 0, 7) == 1 and pc.host_powm(0, 0, 1) == 0 and pc.host_powm(0, 5, 1) == 0
    assert pc.host_powm(2, 10, 2**64 + 13) == 1024


def test_host_powm_rejects_bad_operands():
    from efl import errors
    with pytest.raises(errors.InvalidArgumentError):
        pc.host_powm(3, 5, 10)                # even modulus
    with pytest.raises(errors.InvalidArgumentError):
        pc.host_powm(11, 5, 11)               # base not below the modulus


def test_miller_rabin_known_primes_and_pseudoprimes():
    r = random.Random(1)
    primes = [5, 7, 2**61 - 1, 2**89 - 1, 2**127 - 1, 2**521 - 1, 2**607 - 1, 2**1279 - 1]
    assert pc.probable_primes(primes, 24, r) == [True] * len(primes)
    # Carmichael numbers, strong pseudoprimes to base 2 (2047, 3215031751 strong to 2, 3, 5, 7),
    # semiprimes of large primes, products of small primes
    comp = [561, 1105, 1729, 2047, 3215031751, 3825123056546413051, (2**127 - 1) * (2**61 - 1),
            (2**521 - 1) * (2**89 - 1), 3 * 5 * 7 * 11 * 13 * 17 + 2]
    comp = [c if c & 1 else c + 1 for c in comp]
    assert not any(pc.probable_primes(comp, 24, r))
    # random 512-bit odd numbers: agree with 24 Python Miller-Rabin rounds
    cands = [r.getrandbits(512) | 1 | (1 << 511) for _ in range(300)]

    def py_mr(n):
        d, s = n - 1, 0
        while d % 2 == 0:
            d, s = d // 2, s + 1
        for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
            y = pow(a, d, n)
            if y in (1, n - 1):
                continue
            for _ in range(s - 1):
                y = y * y % n
                if y == n - 1:
                    break
            else:
                return False
        return True
    assert pc.probable_primes(cands, 8, r) == [py_mr(c) for c in cands]


@pytest.mark.parametrize("n_bytes", [64, 128, 256])
def test_generate_keypair_ints_construction(n_bytes):
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    bits = 4 * n_bytes
    assert n == p * q and p != q
    for x in (p, q):
        assert x.bit_length() == bits and x & 3 == 3
    assert math.gcd(p - 1, q - 1) == 2
    assert 0 < hs < n * n and pow(hs, (p - 1) * (q - 1), n * n) == 1      # an n-th residue
    again = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    assert again == (n, hs, p, q)                                          # deterministic given rng


def test_hs_by_crt_equals_direct_power():
    r = random.Random(9)
    _, _, p, q = pc.generate_keypair_ints(128, 24, r)
    n = p * q
    for _ in range(5):
        x = r.randrange(1, n)
        assert pc.hs_of(x, p, q) == pow((-x * x) % n, n, n * n)


def test_host_sqr_chain_matches_repeated_powers():
    """The fixed-base table's row bases (efl_host_sqr_chain): base^(2^(k i)) mod m, as KeyBlock's
    table build takes them, for odd moduli of 1 to 128 words and k = 0, 1, 12."""
    r = random.Random(3)
    for words in (1, 2, 33, 128):
        m = r.getrandbits(32 * words) | 1 | (1 << (32 * words - 1))
        b = r.randrange(m)
        for k in (0, 1, 12):
            rows = pc.host_sqr_chain(b, k, 7, m, words)
            x = b
            for row in rows:
                assert int.from_bytes(row.tobytes(), "little") == x
                x = pow(x, 1 << k, m)
    from efl import errors
    with pytest.raises(errors.InvalidArgumentError):
        pc.host_sqr_chain(5, 1, 2, 10, 1)


def test_keys_below_128_bits_refused_before_the_prime_search():
    """n_bytes < 16 (primes of 16..60 bits): the device kernels need n of 128 bits or more, and the
    sieve would discard every prime of 16 bits or fewer, so the search is refused at once
     instead of looping."""
    import time
    from efl import errors
    t0 = time.perf_counter()
    for nb in (1, 2, 4, 8, 15):
        with pytest.raises(errors.UnimplementedError, match="128 bits"):
            pc.generate_keypair_ints(nb, 4, random.Random(nb))
    assert time.perf_counter() - t0 < 1.0
