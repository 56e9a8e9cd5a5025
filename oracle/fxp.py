"""ORACLE — test infrastructure only (never imported by the product path).

Two independent CPU restatements of efls-train's fixed-point codec
(efls-train/cc/efl/math/fixed_point.cc):

* ``C``   — ctypes binding of oracle/build/liboracle.so (fxp_oracle.c, plain C) plus the GMP-backed
            decode in the reference's call order (fxp_gmp.c) used to pin it.
* ``np_*`` — vectorised numpy restatement written separately from the C one, so the two cross-check
            each other (tests/test_oracle.py).

Rules follow SURVEY.md Appendix A (A1-A6) for encode and GMP mpf_get_d truncation for decode.
Decode defaults to the MXCSR FTZ|DAZ state the reference op runs in inside TensorFlow (its kernels
execute on TF threadpool threads, which set flush-to-zero); ftz=False gives the bare
loop's output (+0.0 -> 2^-127).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.oracle_encode_f32.argtypes = [vp, vp, vp, i64, i32]
        L.oracle_encode_f64.argtypes = [vp, vp, vp, i64, i32]
        L.oracle_encode_int.argtypes = [vp, i32, vp, vp, i64]
        L.oracle_decode_f32.argtypes = [vp, vp, vp, i64, i32]
        L.oracle_decode_f64.argtypes = [vp, vp, vp, i64]
        L.oracle_gmp_get_d_bits.argtypes = [ctypes.c_uint64, i32, i64]
        L.oracle_gmp_get_d_bits.restype = ctypes.c_uint64
        L.oracle_d2f_bits.argtypes = [ctypes.c_uint64, i32]
        L.oracle_d2f_bits.restype = ctypes.c_uint32
        L.oracle_decode_hex_d.argtypes = [ctypes.c_char_p, i64, i64, vp]
        L.oracle_decode_hex_d.restype = i32
        L.gmp_decode_i64.argtypes = [vp, vp, vp, i32, i64, i32]
        L.gmp_decode_hex.argtypes = [vp, vp, vp, vp, i32, i64, i32]
        L.gmp_decode_hex.restype = i64
        L.baseline_encode_f32_mt.argtypes = [vp, vp, vp, i64, i32, i32]
        L.baseline_decode_f32_mt.argtypes = [vp, vp, vp, i64, i32, i32]
        L.baseline_encode_f32_literal.argtypes = [vp, vp, vp, i64, i32]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------------------- C oracle

def encode(x: np.ndarray, decrease_precision: bool = False):
    """ConvertToFixedPoint (fixed_point.cc:24-199) -> (mantissa int64, exponent int64)."""
    x = np.ascontiguousarray(x)
    n = x.size
    M = np.empty(x.shape, np.int64)
    E = np.empty(x.shape, np.int64)
    dp = int(bool(decrease_precision))
    if x.dtype == np.float32:
        lib().oracle_encode_f32(_p(x), _p(M), _p(E), n, dp)
    elif x.dtype == np.float64:
        lib().oracle_encode_f64(_p(x), _p(M), _p(E), n, dp)
    elif x.dtype in (np.int8, np.int16, np.int32, np.int64):
        lib().oracle_encode_int(_p(x), x.dtype.itemsize, _p(M), _p(E), n)
    else:
        raise TypeError(f"unsupported dtype {x.dtype}")
    return M, E


def decode(M: np.ndarray, E: np.ndarray, dtype=np.float32, ftz: bool = True):
    """FixedPointToFloatPoint<int64, dtype> (fixed_point.cc:201-287). ftz (default, as the op runs
    on a TF threadpool thread): float results below the normal range flush to signed zero."""
    M = np.ascontiguousarray(M, np.int64)
    E = np.ascontiguousarray(E, np.int64)
    if M.size != E.size:
        raise ValueError("mantissa and exponent should be the same size.")
    if np.dtype(dtype) == np.float32:
        y = np.empty(M.shape, np.float32)
        lib().oracle_decode_f32(_p(M), _p(E), _p(y), M.size, int(bool(ftz)))
    else:
        y = np.empty(M.shape, np.float64)
        lib().oracle_decode_f64(_p(M), _p(E), _p(y), M.size)
    return y


def pack_hex(strings):
    """list of str/bytes -> (flat uint8 buffer, int64 offsets[n+1])."""
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    offs = np.zeros(len(bs) + 1, np.int64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    buf = np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy()
    return buf, offs


def decode_hex(strings, E: np.ndarray, dtype=np.float32, ftz: bool = True):
    """FixedPointToFloatPoint<string, dtype> restated (top-64-bit truncation)."""
    E = np.ascontiguousarray(E, np.int64).reshape(-1)
    out = np.empty(E.shape, np.float64 if np.dtype(dtype) == np.float64 else np.float32)
    d = ctypes.c_uint64()
    for i, s in enumerate(strings):
        b = s.encode() if isinstance(s, str) else bytes(s)
        if lib().oracle_decode_hex_d(b, len(b), int(E[i]), ctypes.byref(d)):
            raise ValueError(f"malformed hex mantissa {b!r}")
        if out.dtype == np.float64:
            out[i] = np.uint64(d.value).view(np.float64)
        else:
            out[i] = np.uint32(lib().oracle_d2f_bits(d.value, int(bool(ftz)))).view(np.float32)
    return out


# ------------------------------------------------------------------------------ GMP pin

def gmp_decode(M, E, dtype=np.float32, ftz=True):
    """Decode through GMP 6.2.1 mpf in the reference's call order (pinning only)."""
    M = np.ascontiguousarray(M, np.int64)
    E = np.ascontiguousarray(E, np.int64)
    f64 = np.dtype(dtype) == np.float64
    y = np.empty(M.shape, np.float64 if f64 else np.float32)
    lib().gmp_decode_i64(_p(M), _p(E), _p(y), int(f64), M.size, int(bool(ftz)))
    return y


def gmp_decode_hex(strings, E, dtype=np.float32, ftz=True):
    buf, offs = pack_hex(strings)
    E = np.ascontiguousarray(E, np.int64)
    f64 = np.dtype(dtype) == np.float64
    y = np.empty(E.shape, np.float64 if f64 else np.float32)
    bad = lib().gmp_decode_hex(_p(buf), _p(offs), _p(E), _p(y), int(f64), E.size, int(bool(ftz)))
    return y, bad


# ------------------------------------------------------------------------ CPU baseline

def baseline_encode_decode(x: np.ndarray, nthreads: int, decrease_precision=False, ftz=True):
    """Reference op timing stand-in: the literal encode loop + GMP-mpf decode loop, sharded over
    threads (decode under MXCSR FTZ|DAZ when ftz, as on a TF threadpool thread)."""
    x = np.ascontiguousarray(x, np.float32)
    n = x.size
    M = np.empty(n, np.int64)
    E = np.empty(n, np.int64)
    y = np.empty(n, np.float32)
    lib().baseline_encode_f32_mt(_p(x), _p(M), _p(E), n, int(bool(decrease_precision)), nthreads)
    lib().baseline_decode_f32_mt(_p(M), _p(E), _p(y), n, nthreads, int(bool(ftz)))
    return M, E, y


def literal_encode_f32(x: np.ndarray, decrease_precision=False):
    """The reference loop body statement for statement (float-convert ctz), one thread."""
    x = np.ascontiguousarray(x, np.float32)
    M = np.empty(x.shape, np.int64)
    E = np.empty(x.shape, np.int64)
    lib().baseline_encode_f32_literal(_p(x), _p(M), _p(E), x.size, int(bool(decrease_precision)))
    return M, E


# ----------------------------------------------------------------- numpy restatement

def np_encode_f32(x: np.ndarray, decrease_precision=False):
    """Independent numpy restatement of fixed_point.cc:107-137 (A1-A6)."""
    b = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.int64)
    sign = b >> 31
    exp = ((b >> 23) & 0xFF) - 150
    mant = (b & 0x7FFFFF) | np.where(exp != 0, 0x800000, 0)
    if decrease_precision:
        mant = mant >> 13
        exp = exp + 13
    low = mant & -mant                       # lowest set bit (0 when mant == 0)
    safe = np.where(low == 0, 1, low)
    r = np.where(low == 0, -127, np.log2(safe.astype(np.float64)).astype(np.int64))
    mant = np.where(low == 0, 0, mant >> np.where(low == 0, 0, r))
    exp = exp + r
    M = np.where(sign == 1, -mant, mant)
    return M.astype(np.int64), exp.astype(np.int64)


def np_encode_f64(x: np.ndarray, decrease_precision=False):
    b = np.ascontiguousarray(x, np.float64).view(np.uint64)
    sign = (b >> np.uint64(63)).astype(np.int64)
    exp = ((b >> np.uint64(52)) & np.uint64(0x7FF)).astype(np.int64) - 1075
    mant = (b & np.uint64(0xFFFFFFFFFFFFF)).astype(np.int64) | np.where(exp != 0, 1 << 52, 0)
    if decrease_precision:
        mant = mant >> 42
        exp = exp + 42
    low = mant & -mant
    r = np.zeros_like(mant)
    t = low.copy()
    for k in (32, 16, 8, 4, 2, 1):           # integer log2 of a power of two
        big = t >= (1 << k)
        r = r + np.where(big, k, 0)
        t = np.where(big, t >> k, t)
    r = np.where(low == 0, -1023, r)
    mant = np.where(low == 0, 0, mant >> np.where(low == 0, 0, r))
    exp = exp + r
    return np.where(sign == 1, -mant, mant).astype(np.int64), exp.astype(np.int64)


def np_get_d_bits(M: np.ndarray, E: np.ndarray) -> np.ndarray:
    """numpy restatement of GMP mpf_get_d on M*2^E (truncating), returns uint64 bit patterns."""
    M = np.asarray(M, np.int64)
    E = np.asarray(E, np.int64)
    neg = M < 0
    a = np.where(neg, (~M.view(np.uint64)) + np.uint64(1), M.view(np.uint64)).astype(np.uint64)
    p = np.zeros(M.shape, np.int64)
    t = a.copy()
    for k in (32, 16, 8, 4, 2, 1):
        big = t >= (np.uint64(1) << np.uint64(k))
        p = p + np.where(big, k, 0)
        t = np.where(big, t >> np.uint64(k), t)
    Ec = np.clip(E, -9000, 9000)
    L = p + Ec
    sh_r = np.clip(p - 52, 0, 63).astype(np.uint64)
    sh_l = np.clip(52 - p, 0, 63).astype(np.uint64)
    m53 = np.where(p >= 52, a >> sh_r, a << sh_l)
    normal = ((L + 1023).clip(0, 2047).astype(np.uint64) << np.uint64(52)) | (m53 & np.uint64((1 << 52) - 1))
    rs = np.clip(-1022 - L, 0, 63).astype(np.uint64)
    denorm = m53 >> rs
    bits = np.where(L >= -1022, normal, denorm)
    bits = np.where(L >= 1024, np.uint64(0x7FF0000000000000), bits)
    sgn = np.where(neg, np.uint64(1) << np.uint64(63), np.uint64(0))
    bits = bits | sgn
    bits = np.where((L <= -1075) | (a == 0), np.uint64(0), bits)
    bits = np.where((E > 4096) & (a != 0), sgn | np.uint64(0x7FF0000000000000), bits)
    bits = np.where((E < -8192) & (a != 0), np.uint64(0), bits)
    return bits


def np_decode_f32(M, E, ftz=True):
    d = np_get_d_bits(M, E).view(np.float64)
    with np.errstate(over="ignore"):
        f = d.astype(np.float32)
    if ftz:   # x86 FTZ|DAZ: tininess after rounding, unbounded exponent
        tiny = np.abs(d) < float.fromhex("0x1.ffffffp-127")
        sgn = (d.view(np.uint64) >> np.uint64(32)).astype(np.uint32) & np.uint32(0x80000000)
        f = np.where(tiny, sgn, f.view(np.uint32)).astype(np.uint32).view(np.float32)
    return f
