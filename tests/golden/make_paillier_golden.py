"""Generate tests/golden/paillier_kat.json: Paillier known-answer vectors computed by GMP 6.2.1 in
the reference's call order (oracle/paillier_gmp.c; efls-train/cc/efl/math/paillier.cc:103-131,
296-312, 833-904; gmp_utils.cc:56-144). Keys come from the reference's keygen procedure with an
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
            if n_bytes <= 128:
                assert hsa == P.gmp_fbpowm(hs, kp.n2, a_bits, g, a)
            c_hex = P.gmp_encrypt(n, m, hsa)
            assert c_hex == P.hx(P.encrypt(kp, m, hsa))
            d_hex = P.gmp_decrypt(p, q, int(c_hex, 16))
            assert d_hex == P.hx(P.decrypt(kp, int(c_hex, 16))) and int(d_hex, 16) == m
            entries.append({"m": m, "a": P.hx(a), "g": g, "hsa": P.hx(hsa), "c": c_hex, "d": d_hex})
        # homomorphic ops on the first ciphertexts (paillier.cc:157-285)
        c0, c1 = int(entries[5]["c"], 16), int(entries[6]["c"], 16)
        ops = {"add": P.hx(P.add(kp, c0, c1)), "mul_scalar_7": P.hx(P.mul_scalar(kp, c0, 7)),
               "mul_exp2_5": P.hx(P.mul_exp2(kp, c1, 5))}
        out["keys"].append({"n_bytes": n_bytes, "mt_seed": seed, "n": P.hx(n), "hs": P.hx(hs), "p": P.hx(p),
                            "q": P.hx(q), "a_bits": a_bits, "vectors": entries, "ops": ops})
        print(n_bytes, "ok", len(entries))
    with open(os.path.join(HERE, "paillier_kat.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
