"""Generate tests/golden/paillier_kat.json: Paillier known-answer vectors computed by GMP 6.2.1 in
the reference's call order (oracle/paillier_gmp.c; efls-train/cc/efl/math/paillier.cc:103-131,
157-285, 296-312, 722-733, 833-904, 987-1035; gmp_utils.cc:56-144) — encrypt, decrypt and the
fixed-base powm at every key size, and the homomorphic ops and a matmul per key. Keys come from the reference's keygen procedure with an
explicit MT seed instead of time(). Each value is cross-checked against the Python-int
restatement (oracle/paillier.py) before it is written.

Run:  python tests/golden/make_paillier_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import fxp, paillier as P  # noqa: E402

KEYS = [  # (n_bytes, mt seed, group sizes for fbpowm vectors, plaintext count)
    (64, 7, (1, 3), 24),
    (128, 12345, (1, 3, 10), 32),
    (256, 99, (1, 4), 16),
    (512, 2021, (1,), 8),
]


def gmp_ops(kp, n, entries, rng):
    """Homomorphic ops on the KAT ciphertexts, computed by GMP in the reference's call order
    (oracle/paillier_gmp.c: paillier.cc:157-285, :722-733, :987-1035) and cross-checked against the
    Python-int restatement. Scalars: the int32 / int64 / string overloads' values, both signs
    (a negative scalar inverts x first, :201-211), int64's extremes and a 200-bit signed hex text."""
    c0, c1 = int(entries[5]["c"], 16), int(entries[6]["c"], 16)
    big = -rng.getrandbits(200)
    scalars = {"mul_scalar_7": 7, "mul_scalar_0": 0, "mul_scalar_neg": -123456789,
               "mul_scalar_i64max": 2**63 - 1, "mul_scalar_i64min": -2**63,
               "mul_scalar_hex": P.hx(big)}
    ops = {"add": P.gmp_add(n, c0, c1)}
    assert ops["add"] == P.hx(P.add(kp, c0, c1))
    for name, y in scalars.items():
        ops[name] = P.gmp_mul_scalar(n, c0, y)
        assert ops[name] == P.hx(P.mul_scalar_hex(kp, c0, y) if isinstance(y, str) else P.mul_scalar(kp, c0, y))
    ops["mul_scalar_hex_text"] = P.hx(big)
    for e in (5, 0, 77):
        ops[f"mul_exp2_{e}"] = P.gmp_mul_exp2(n, c1, e)
        assert ops[f"mul_exp2_{e}"] == P.hx(P.mul_exp2(kp, c1, e))
    ops["invert"] = P.gmp_invert(n, c0)
    assert ops["invert"] == P.hx(P.invert(kp, c0))
    # PaillierMatmul: x [2, 3] = the first six KAT ciphertexts, mixed-sign y with a zero, spread
    # exponents (the minimum differs per output)
    u, v, w = 2, 3, 2
    xm = [[int(entries[i * v + j]["c"], 16) for j in range(v)] for i in range(u)]
    xe = [[rng.randrange(-30, 10) for _ in range(v)] for _ in range(u)]
    ym = [[rng.randrange(-2**40, 2**40) for _ in range(w)] for _ in range(v)]
    ym[1][0], ym[2][1] = 0, -(2**63 - 1)
    ye = [[rng.randrange(-20, 20) for _ in range(w)] for _ in range(v)]
    zm, ze = P.gmp_matmul(n, xm, xe, ym, ye)
    rm, re_ = P.matmul(kp, xm, xe, ym, ye)
    assert zm == [[P.hx(c) for c in row] for row in rm] and ze == re_
    mm = {"x_vectors": list(range(u * v)), "shape": [u, v, w], "xe": xe, "ym": ym, "ye": ye, "zm": zm, "ze": ze}
    return ops, mm


def main():
    fxp.build()
    rng = random.Random(42)
    out = {"provenance": __doc__.strip().splitlines()[0], "keys": []}
    for n_bytes, seed, groups, count in KEYS:
        n, hs, p, q = P.gmp_keygen(n_bytes, seed)
        a_bits = n_bytes * 4          # a_bytes = n_bytes / 2 (PaillierHook default)
        kp = P.Keypair(n, hs, a_bits // 8, 1, p, q)
        ms = [0, 1, -1, 2**63 - 1, -2**63, 12345, -98765] + \
             [rng.randrange(-2**63, 2**63) for _ in range(count - 7)]
        entries = []
        for i, m in enumerate(ms):
            a = rng.getrandbits(a_bits)
            g = groups[i % len(groups)]
            hsa = P.fbpowm(hs, kp.n2, a, g)
            assert hsa == P.gmp_fbpowm(hs, kp.n2, a_bits, g, a)
            c_hex = P.gmp_encrypt(n, m, hsa)
            assert c_hex == P.hx(P.encrypt(kp, m, hsa))
            d_hex = P.gmp_decrypt(p, q, int(c_hex, 16))
            assert d_hex == P.hx(P.decrypt(kp, int(c_hex, 16))) and int(d_hex, 16) == m
            entries.append({"m": m, "a": P.hx(a), "g": g, "hsa": P.hx(hsa), "c": c_hex, "d": d_hex})
        ops, mm = gmp_ops(kp, n, entries, random.Random(1000 + n_bytes))
        out["keys"].append({"n_bytes": n_bytes, "mt_seed": seed, "n": P.hx(n), "hs": P.hx(hs), "p": P.hx(p),
                            "q": P.hx(q), "a_bits": a_bits, "vectors": entries, "ops": ops, "matmul": mm})
        print(n_bytes, "ok", len(entries))
    with open(os.path.join(HERE, "paillier_kat.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
