"""ORACLE — test infrastructure only (never imported by the product path).

Python-int restatement of efls-train's Paillier arithmetic (efls-train/cc/efl/math/paillier.cc,
gmp_utils.cc), plus ctypes access to the GMP harness (oracle/paillier_gmp.c) that runs the
reference's call sequence through GMP 6.2.1. Python ints are exact, so the restatement equals GMP
wherever the reference's result is defined (tests/test_paillier_oracle.py checks it).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

from oracle import fxp

CAP = 8192


def _lib():
    L = fxp.lib()
    if not getattr(L, "_pl_ready", False):
        c, i, sz, ul = ctypes.c_char_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_ulong
        L.pl_gmp_keygen.argtypes = [i, i, ul, c, c, c, c, sz]
        L.pl_gmp_encrypt.argtypes = [c, ctypes.c_longlong, c, c, sz]
        L.pl_gmp_decrypt.argtypes = [c, c, c, c, sz]
        L.pl_gmp_fbpowm.argtypes = [c, c, ctypes.c_uint, ctypes.c_uint, c, c, sz]
        L.pl_gmp_fbpowm.restype = i
        L.pl_gmp_powm.argtypes = [c, c, c, c, sz]
        L.pl_gmp_add.argtypes = [c, c, c, c, sz]
        L.pl_gmp_mul_scalar.argtypes = [c, c, c, c, sz]
        L.pl_gmp_mul_scalar.restype = i
        L.pl_gmp_mul_exp2.argtypes = [c, c, ctypes.c_longlong, c, sz]
        L.pl_gmp_mul_exp2.restype = i
        L.pl_gmp_invert.argtypes = [c, c, c, sz]
        L.pl_gmp_invert.restype = i
        vp = ctypes.c_void_p
        L.pl_gmp_matmul.argtypes = [c, vp, vp, vp, vp, i, i, i, vp, sz, vp]
        L.pl_gmp_matmul.restype = i
        L._pl_ready = True
    return L


def hx(v: int) -> str:
    """mpz_get_str(..., 16): lowercase, no prefix, '-' sign (gmp_utils.cc:146-150)."""
    return ("-" + format(-v, "x")) if v < 0 else format(v, "x")


def _buf():
    return ctypes.create_string_buffer(CAP)


# ----------------------------------------------------------------------------- GMP harness

def gmp_keygen(n_bytes: int, seed: int, reps: int = 24):
    bs = [_buf() for _ in range(4)]
    _lib().pl_gmp_keygen(n_bytes, reps, seed, *bs, CAP)
    return tuple(int(b.value, 16) for b in bs)   # n, hs, p, q


def gmp_encrypt(n: int, m: int, hsa: int) -> str:
    b = _buf()
    _lib().pl_gmp_encrypt(hx(n).encode(), m, hx(hsa).encode(), b, CAP)
    return b.value.decode()


def gmp_decrypt(p: int, q: int, c: int) -> str:
    b = _buf()
    _lib().pl_gmp_decrypt(hx(p).encode(), hx(q).encode(), hx(c).encode(), b, CAP)
    return b.value.decode()


def gmp_fbpowm(base: int, mod: int, exp_bits: int, g: int, a: int) -> int:
    b = _buf()
    rc = _lib().pl_gmp_fbpowm(hx(base).encode(), hx(mod).encode(), exp_bits, g, hx(a).encode(), b, CAP)
    if rc != 1:
        raise ValueError("exponent wider than the table")
    return int(b.value, 16)


def gmp_add(n: int, x: int, y: int) -> str:                 # paillier.cc:157-169
    b = _buf()
    _lib().pl_gmp_add(hx(n).encode(), hx(x).encode(), hx(y).encode(), b, CAP)
    return b.value.decode()


def gmp_mul_scalar(n: int, x: int, y) -> str:               # paillier.cc:180-248
    """y: a Python int (int32 / int64 / wider) or the signed hex text the string overload parses."""
    b = _buf()
    ys = y if isinstance(y, str) else hx(y)
    if _lib().pl_gmp_mul_scalar(hx(n).encode(), hx(x).encode(), ys.encode(), b, CAP) != 0:
        raise ValueError("x has no inverse mod n^2")
    return b.value.decode()


def gmp_mul_exp2(n: int, x: int, y: int) -> str:            # paillier.cc:722-733
    b = _buf()
    if _lib().pl_gmp_mul_exp2(hx(n).encode(), hx(x).encode(), y, b, CAP) != 0:
        raise ValueError("y should be a positive tensor.")
    return b.value.decode()


def gmp_invert(n: int, x: int) -> str:                      # paillier.cc:275-285
    b = _buf()
    if _lib().pl_gmp_invert(hx(n).encode(), hx(x).encode(), b, CAP) != 0:
        raise ValueError("x has no inverse mod n^2")
    return b.value.decode()


def gmp_matmul(n: int, xm, xe, ym, ye):                     # paillier.cc:987-1035
    """xm [u][v] ciphertext ints, xe [u][v], ym / ye [v][w] ints -> (zm hex [u][w], ze [u][w])."""
    u, v, w = len(xm), len(xm[0]), len(ym[0])
    strs = [ctypes.create_string_buffer(hx(c).encode()) for row in xm for c in row]
    xs = (ctypes.c_char_p * (u * v))(*[ctypes.cast(s, ctypes.c_char_p) for s in strs])
    arr = ctypes.c_longlong * max(1, u * v)
    xe_c = arr(*[e for row in xe for e in row])
    yarr = ctypes.c_longlong * max(1, v * w)
    ym_c = yarr(*[e for row in ym for e in row])
    ye_c = yarr(*[e for row in ye for e in row])
    out = ctypes.create_string_buffer(CAP * max(1, u * w))
    ze = (ctypes.c_longlong * max(1, u * w))()
    if _lib().pl_gmp_matmul(hx(n).encode(), xs, xe_c, ym_c, ye_c, u, v, w, out, CAP, ze) != 0:
        raise ValueError("an x has no inverse mod n^2")
    zm = [[out.raw[(i * w + k) * CAP:(i * w + k + 1) * CAP].split(b"\0", 1)[0].decode() for k in range(w)]
          for i in range(u)]
    return zm, [[ze[i * w + k] for k in range(w)] for i in range(u)]


# ------------------------------------------------------------------ Python-int restatement

def l_func(x: int, d: int) -> int:                       # paillier.cc:23-26
    assert (x - 1) % d == 0
    return (x - 1) // d


def h_func(n: int, x: int) -> int:                       # paillier.cc:28-37
    return pow(l_func(pow(n + 1, x - 1, x * x), x), -1, x)


@dataclass
class Keypair:
    n: int
    hs: int
    a_bytes: int
    group_size: int = 1
    p: int | None = None
    q: int | None = None
    n2: int = field(init=False)
    max_: int = field(init=False)

    def __post_init__(self):                              # SetPublicKey, paillier.cc:70-86
        self.n2 = self.n * self.n
        self.max_ = -(-(2 * self.n) // 3)                 # mpz_cdiv_q_ui(2n, 3)

    @property
    def has_private(self):
        return self.p is not None

    def private_parts(self):                              # SetPrivateKey, paillier.cc:88-101
        p, q = self.p, self.q
        return dict(p2=p * p, q2=q * q, hp=h_func(self.n, p), hq=h_func(self.n, q), qinvp=pow(q, -1, p))


def encrypt(kp: Keypair, m: int, hsa: int) -> int:       # paillier.cc:103-131, hsa given
    c = 1 + abs(m) * kp.n
    if m < 0:
        c = pow(c, -1, kp.n2)
    return c * hsa % kp.n2


def decrypt(kp: Keypair, c: int) -> int:                 # paillier.cc:296-312
    pp = kp.private_parts()
    mp = l_func(pow(c, kp.p - 1, pp["p2"]), kp.p) * pp["hp"] % kp.p
    mq = l_func(pow(c, kp.q - 1, pp["q2"]), kp.q) * pp["hq"] % kp.q
    m = (mp - mq) * pp["qinvp"] % kp.p * kp.q + mq
    m %= kp.n
    if m > kp.max_:
        m -= kp.n
    return m


def group_reversed(a: int, g: int) -> int:
    """The exponent mpz_fbpowm really applies: every g-bit group of a,
    and the top partial group, bit-reversed in place (gmp_utils.cc:121-125, 133-137)."""
    size = max(1, a.bit_length())
    out = 0
    for s in range(0, size, g):
        w = min(g, size - s)
        grp = (a >> s) & ((1 << w) - 1)
        rev = int(format(grp, f"0{w}b")[::-1], 2)
        out |= rev << s
    return out


def fbpowm(base: int, mod: int, a: int, g: int) -> int:
    return pow(base, group_reversed(a, g), mod)


def add(kp, x, y):                                        # paillier.cc:157-178
    return x * y % kp.n2


def mul_scalar(kp, x, y: int):                            # paillier.cc:180-265
    if y < 0:
        return pow(pow(x, -1, kp.n2), -y, kp.n2)
    return pow(x, y, kp.n2)


def mul_exp2(kp, x, e: int):                              # paillier.cc:683-719
    if e < 0:
        raise ValueError("y should be a positive tensor.")
    return pow(x, 1 << e, kp.n2)


def invert(kp, x):                                        # paillier.cc:267-285
    return pow(x, -1, kp.n2)


def mul_scalar_hex(kp, x, y: str):                        # paillier.cc:239-248 (T = string)
    """mpz_init_set_str(op, y, 16): the scalar text is a signed hex integer."""
    return mul_scalar(kp, x, int(y, 16))


def fixedpoint_add(kp, xm, xe: int, ym, ye: int):         # python/efl/privacy/paillier.py:116-133
    """FixedPointTensor.__add__ of two encrypted mantissas, element-wise: d = xe - ye,
    dl = max(d, 0), dr = |min(d, 0)|; mantissa = (x << dl) + (y << dr) = PaillierAdd of two
    PaillierMulExp2; exponent = min(xe, ye)."""
    d = xe - ye
    return add(kp, mul_exp2(kp, xm, max(d, 0)), mul_exp2(kp, ym, abs(min(d, 0)))), min(xe, ye)


def column_sum(kp, xm, xe):                               # python/efl/privacy/paillier_layer.py:297-310
    """The PaillierPassiveWeight gradient reduction: the rows of an encrypted FixedPointTensor
    ([rows][cols] ciphertexts and exponents) added one at a time, as the reference's
    tf.while_loop does."""
    acc_m, acc_e = list(xm[0]), list(xe[0])
    for r in range(1, len(xm)):
        for c in range(len(acc_m)):
            acc_m[c], acc_e[c] = fixedpoint_add(kp, acc_m[c], acc_e[c], xm[r][c], xe[r][c])
    return acc_m, acc_e


def matmul(kp, xm, xe, ym, ye):
    """PaillierMatmul (paillier.cc:941-1051): xm [u][v] ciphertexts, xe/ym/ye int matrices.
    z[i][k] = prod_j (xm[i][j]^ym[j][k])^(2^(xe+ye - min)) ; z_exp = min_j (xe[i][j] + ye[j][k])."""
    u, v, w = len(xm), len(xm[0]), len(ym[0])
    zm = [[0] * w for _ in range(u)]
    ze = [[0] * w for _ in range(u)]
    for i in range(u):
        for k in range(w):
            exps = [xe[i][j] + ye[j][k] for j in range(v)]
            mn = min(exps)
            acc = None
            for j in range(v):
                y = ym[j][k]
                t = pow(xm[i][j], y, kp.n2) if y >= 0 else pow(pow(xm[i][j], -1, kp.n2), -y, kp.n2)
                t = pow(t, 1 << (exps[j] - mn), kp.n2)
                acc = t if acc is None else t * acc % kp.n2
            zm[i][k], ze[i][k] = acc, mn
    return zm, ze
