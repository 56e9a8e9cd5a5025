#!/usr/bin/env python3
"""CPU simulation of the separated-operand-scanning (SOS) Montgomery squaring over G lanes
(csrc/sliced28.h sos_sqr, build knob EFL_SQR_SOS), lane by lane, with Python integers standing in
for the 64-bit accumulators and the 32-bit LDS words (each checked against its width).

Phase 1 (the square into the LDS array T of 2L words, one 28-bit column limb per ds_add):
  lane g: A_g^2 (product scanning, symmetric, at offset 2 g C); the full cross product
  2 A_g A_(g+1 mod G) at offset (2 g + 1) C, or ((g + g+1 mod G) C for the wrap-around pair), its
  partner chunk taken by a lane rotation; and for G = 4 half of the distance-2 pair's rows
  (lane g < 2: rows [0, H) of A_g against A_(g+2); lane g >= 2: rows [H, C) of A_(g-2) against A_g).
  For G = 2 the one cross pair is split by rows between the two lanes the same way.
Phase 2 (reduction): CIOS steps with only the u m products over the lane-sliced window holding the
  low half T_lo, then the high half added: (T + U m) / R = T_hi + (T_lo + U m) / R, U = -T m^-1 mod R
  (U depends on T_lo only).

    python tools/sos_sim.py [--trials 20]
"""
import argparse
import random

BITS = 28
MASK = (1 << BITS) - 1


def limbs(x, n):
    return [(x >> (BITS * i)) & MASK for i in range(n)]


def scan(x, y, cols):
    """product scanning of x (rows) by y: column k = sum x_r y_(k-r); emits `cols` 28-bit limbs
    (the last takes the remaining carry). Returns the limbs; checks the 64-bit accumulator."""
    out, carry = [], 0
    for k in range(cols):
        acc = carry
        for r in range(len(x)):
            j = k - r
            if 0 <= j < len(y):
                acc += x[r] * y[j]
        assert acc < 1 << 64
        if k < cols - 1:
            out.append(acc & MASK)
            carry = acc >> BITS
        else:
            out.append(acc)
            carry = 0
    return out


def square_scan(a, cols):
    out, carry = [], 0
    n = len(a)
    for k in range(cols):
        acc = 0
        for i in range(n):
            j = k - i
            if i < j < n:
                acc += a[i] * a[j]
        acc = 2 * acc + carry
        if k % 2 == 0 and k // 2 < n:
            acc += a[k // 2] ** 2
        assert acc < 1 << 64
        if k < cols - 1:
            out.append(acc & MASK)
            carry = acc >> BITS
        else:
            out.append(acc)
    return out


def sos_sqr(a, m, C, G):
    L = C * G
    H = (C + 1) // 2
    minv = (-pow(m, -1, 1 << BITS)) % (1 << BITS)
    A = [limbs(a >> (BITS * C * g), C) for g in range(G)]
    M = [limbs(m >> (BITS * C * g), C) for g in range(G)]
    T = [0] * (2 * L)

    def add(off, vals):
        for k, v in enumerate(vals):
            if off + k < 2 * L:
                T[off + k] += v
            else:
                assert v == 0, "product beyond 2L limbs"

    for g in range(G):
        add(2 * g * C, square_scan(A[g], 2 * C))
        if G >= 2:
            if G == 2:
                # the one pair (0, 1): lane 0 rows [0, H) of A_0, lane 1 rows [H, C)
                x = A[0][:H] if g == 0 else A[0][H:]
                ro = 0 if g == 0 else H
                add(C + ro, scan(x, [2 * v for v in A[1]], len(x) + C + 1))
            else:
                p = (g + 1) % G
                add((g + p) * C, scan(A[g], [2 * v for v in A[p]], 2 * C + 1))
                if G == 4:
                    if g < 2:
                        x, y, ro = A[g][:H], A[g + 2], 0
                        off = (2 * g + 2) * C
                    else:
                        x, y, ro = A[g - 2][H:], A[g], H
                        off = (2 * (g - 2) + 2) * C
                    add(off + ro, scan(x, [2 * v for v in y], len(x) + C + 1))
    for v in T:
        assert v < 1 << 32, "LDS word overflow"
    assert sum(v << (BITS * i) for i, v in enumerate(T)) == a * a
    # phase 2: reduce the low half alone over the lane-sliced window (T_lo + U m) / R, U from T_lo;
    # then add the high half: (T + U m) / R = T_hi + (T_lo + U m) / R
    W = [[T[g * C + j] for j in range(C)] for g in range(G)]
    for i in range(L):
        u = ((W[0][0] & 0xFFFFFFFF) * minv) & MASK
        for g in range(G):
            for j in range(C):
                W[g][j] += M[g][j] * u
                assert W[g][j] < 1 << 64
        old = [row[:] for row in W]
        for g in range(G):
            inn = 0 if g == G - 1 else old[g + 1][0]
            c0 = old[0][0] >> BITS if g == 0 else 0
            W[g][:C - 1] = old[g][1:]
            W[g][C - 1] = inn
            W[g][0] += c0
        if L > 64 and (i & 63) == 63:
            cs = [0] * G
            for g in range(G):
                c = 0
                for j in range(C):
                    v = W[g][j] + c
                    W[g][j], c = v & MASK, v >> BITS
                cs[g] = c
            assert cs[G - 1] == 0, "window carry out of the top lane"
            for g in range(1, G):
                W[g][0] += cs[g - 1]
    for g in range(G):
        for j in range(C):
            W[g][j] += T[L + g * C + j]
    return sum(W[g][j] << (BITS * (g * C + j)) for g in range(G) for j in range(C))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    a = ap.parse_args()
    rng = random.Random(7)
    for G, mbits in ((2, 2048), (4, 4096)):
        C = 37
        L = C * G
        R = 1 << (BITS * L)
        for t in range(a.trials):
            m = rng.getrandbits(mbits) | (1 << (mbits - 1)) | 1
            x = rng.randrange(2 * m) if t else 2 * m - 1
            U = (-x * x * pow(m, -1, R)) % R
            want = (x * x + U * m) // R
            got = sos_sqr(x, m, C, G)
            assert got == want, (G, t)
            assert got < 2 * m
        print(f"G={G} C={C} ({mbits}-bit modulus): {a.trials} SOS squarings equal the CIOS result "
              f"(x^2 + U m) / R, LDS words < 2^32, accumulators < 2^64")


if __name__ == "__main__":
    main()
