"""ORACLE — test infrastructure only. Philox4x32-10 (Salmon, Moraes, Dror, Shaw: "Parallel random
numbers: as easy as 1, 2, 3", SC'11), the counter-based generator the build uses to draw the
per-element Paillier randomness `a` (counter = element index, key = 64-bit seed). Mirrors
csrc/paillier.hip draw_a()."""
M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0, p1 = M0 * c0, M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return c0, c1, c2, c3


def draw_a(seed: int, counter: int, a_bits: int) -> int:
    words = (a_bits + 31) // 32
    out = []
    for b in range((words + 3) // 4):
        out += philox4x32_10((counter & MASK, (counter >> 32) & MASK, b, 0), (seed & MASK, (seed >> 32) & MASK))
    a = sum(w << (32 * i) for i, w in enumerate(out[:words]))
    return a & ((1 << a_bits) - 1)
