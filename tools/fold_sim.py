#!/usr/bin/env python3
"""CPU simulation of round 6's folded symmetric Montgomery squaring (csrc/sliced28.h fold_step,
fold_pass, lazy_normalize_folded, normalize_folded; build knob EFL_SQR_FOLD=1), lane by lane, with
Python integers standing in for the 64-bit accumulators. Each accumulator is checked against 2^64.

A square forms 2 a_i a_j once (at step min(i, j)) and a_i^2 once, and a product forms every a_j b_i.
Either way the result must be (x + U m) / R, where U = -x m^-1 mod R and x = a^2 or a b. That is
exactly the blocked CIOS loop's result. Run for the decryption shapes: C = 37 limbs per lane over
G = 2 (2048-bit key, mod p^2) and G = 4 (4096-bit key).

    python tools/fold_sim.py [--trials 20]
"""
import argparse
import random

BITS = 28
MASK = (1 << BITS) - 1


def h1(C):
    return (C + 1) // 2


def pos(C, G, g, j):
    H1, H2 = h1(C), C // 2
    return H1 * g + j if j < H1 else G * H1 + H2 * (G - 1 - g) + (j - H1)


def folded(x, C, G):
    """number -> [lane][slot] 28-bit limbs in the folded layout"""
    return [[(x >> (BITS * pos(C, G, g, j))) & MASK for j in range(C)] for g in range(G)]


def value(lanes, C, G):
    return sum(lanes[g][j] << (BITS * pos(C, G, g, j)) for g in range(G) for j in range(C))


def check(T):
    for row in T:
        for v in row:
            assert 0 <= v < 1 << 64, "accumulator overflow"


def step(T, mul, bi, m, minv, C, G, low):
    H1 = h1(C)
    for g in range(G):
        for j in range(C):
            if j >= H1 or low:
                T[g][j] += mul[g][j] * bi
    check(T)
    u = ((T[0][0] & 0xFFFFFFFF) * minv) & MASK        # lane 0's bottom, broadcast
    for g in range(G):
        for j in range(C):
            T[g][j] += m[g][j] * u
    check(T)
    old = [row[:] for row in T]
    for g in range(G):
        nl = old[g][H1] if g == G - 1 else old[g + 1][0]   # from_next64 of the low bottom
        nh = 0 if g == 0 else old[g - 1][H1]              # from_prev64 of the high bottom
        c0 = old[0][0] >> BITS if g == 0 else 0
        T[g][:H1 - 1] = old[g][1:H1]
        T[g][H1 - 1] = nl
        T[g][H1:C - 1] = old[g][H1 + 1:C]
        T[g][C - 1] = nh
        T[g][0] += c0


def lazy_normalize(T, C, G):
    H1 = h1(C)
    cl, ch = [0] * G, [0] * G
    for g in range(G):
        for j in range(H1):
            v = T[g][j] + cl[g]
            T[g][j], cl[g] = v & MASK, v >> BITS
        for j in range(H1, C):
            v = T[g][j] + ch[g]
            T[g][j], ch[g] = v & MASK, v >> BITS
    for g in range(G):
        inl = 0 if g == 0 else cl[g - 1]
        inh = cl[g] if g == G - 1 else ch[g + 1]
        T[g][0] += inl
        T[g][H1] += inh


def fold_pass(T, mul, bl, m, minv, C, G, sq):
    H1, H2, L = h1(C), C // 2, C * G
    since = 0
    for c in range(G):
        for s in range(H1):
            bi = bl[c * H1 + s]
            if sq:
                mul[c][s] >>= 1
            step(T, mul, bi, m, minv, C, G, True)
            if sq:
                mul[c][s] = 0
        since += H1
        if L > 64 and since + H1 > 64:
            lazy_normalize(T, C, G)
            since = 0
    for c in range(G):
        for s in range(H2):
            bi = bl[G * H1 + c * H2 + s]
            lane = G - 1 - c
            if sq:
                mul[lane][H1 + s] >>= 1
            step(T, mul, bi, m, minv, C, G, not sq)
            if sq:
                mul[lane][H1 + s] = 0
        since += H2
        if L > 64 and since + H2 > 64:
            lazy_normalize(T, C, G)
            since = 0


def normalize(T, C, G):
    """the accumulators' value as one number (normalize_folded's carry ripple, done exactly)"""
    return value(T, C, G)


def fold_mont(a, b, m, C, G):
    """a b R^-1 (b None: a^2 R^-1) through the folded steps; returns the result as a number"""
    L = C * G
    minv = (-pow(m, -1, 1 << BITS)) % (1 << BITS)
    T = [[0] * C for _ in range(G)]
    sq = b is None
    A = folded(a, C, G)
    mul = [[2 * v for v in row] for row in A] if sq else A
    src = a if sq else b
    bl = [(src >> (BITS * i)) & MASK for i in range(L)]
    fold_pass(T, mul, bl, folded(m, C, G), minv, C, G, sq)
    return normalize(T, C, G)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    a = ap.parse_args()
    rng = random.Random(6)
    for G, mbits in ((2, 2048), (4, 4096)):
        C = 37
        L = C * G
        R = 1 << (BITS * L)
        for t in range(a.trials):
            m = rng.getrandbits(mbits) | (1 << (mbits - 1)) | 1
            x = rng.randrange(2 * m) if t else 2 * m - 1       # the walk's values stay below 2m
            y = rng.randrange(2 * m)
            for b in (None, y):
                prod = x * x if b is None else x * b
                U = (-prod * pow(m, -1, R)) % R
                want = (prod + U * m) // R
                got = fold_mont(x, b, m, C, G)
                assert got == want, (G, t, b is None)
                assert got < 2 * m
        print(f"G={G} C={C} ({mbits}-bit modulus): {a.trials} squarings and {a.trials} products "
              f"equal the CIOS result (x + U m) / R, accumulators < 2^64")


if __name__ == "__main__":
    main()
