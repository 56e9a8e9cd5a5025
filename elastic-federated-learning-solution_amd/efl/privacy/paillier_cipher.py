"""Paillier keypair, ciphertext tensors and homomorphic ops on the MI355X (Stage P).

Drop-in for efls-train/python/efl/privacy/paillier.py:29-205 (`efl.paillier.Keypair`,
`efl.paillier.Tensor`, FixedPointTensor arithmetic). The per-element arithmetic runs in
libefl_hip.so (csrc/paillier.hip); this module does what the reference's PaillierKeypair resource
does on the host once per key (paillier.cc:50-101, SetPublicKey / SetPrivateKey, the fbpowm table
of gmp_utils.cc:56-89): derive the key constants with exact integer arithmetic, add the Montgomery
constants the kernels need, and upload everything as one device "key block" (include/efl_hip.h,
efl_pl_key).

Ciphertexts stay in HBM as fixed-width limb rows (CipherTensor, [N, 2*ln] uint32); hex text (the
reference's DT_STRING) is produced or parsed on the GPU only when a tensor crosses the wire or is
handed to string-typed callers.
"""
from __future__ import annotations

import ctypes
import hashlib
import math
import os
import secrets

import numpy as np
import torch

from efl import errors, exporter
from efl import lib as _efl_lib
from efl.privacy.hex_tensor import HexTensor

_lib = _efl_lib.raw()
_vp, _i64, _i32, _u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint64


class PlKey(ctypes.Structure):
    """ctypes mirror of efl_pl_key (include/efl_hip.h)."""
    _fields_ = [(n, ctypes.c_int32) for n in ("ln", "a_bits", "group_size", "table_rows", "table_cols",
                                               "has_private", "pm1_bits", "qm1_bits")] + \
               [(n, ctypes.c_uint32) for n in ("n2_minv", "p2_minv", "q2_minv", "p_minv", "q_minv")] + \
               [(n, ctypes.c_int64) for n in ("off_n", "off_n2", "off_n2_r2", "off_n2_one", "off_table", "off_max",
                                               "off_p", "off_q", "off_p2", "off_q2", "off_p2_r3", "off_q2_r3",
                                               "off_pm1", "off_qm1", "off_pinv_w", "off_qinv_w", "off_hp",
                                               "off_hq", "off_qinvp")] + \
               [("p2_28_len", ctypes.c_int32), ("p2_minv28", ctypes.c_uint32), ("q2_minv28", ctypes.c_uint32),
                ("off_p2_28", ctypes.c_int64), ("off_q2_28", ctypes.c_int64),
                ("off_p2_r2_28", ctypes.c_int64 * 6), ("off_q2_r2_28", ctypes.c_int64 * 6),
                ("n2_28_len", ctypes.c_int32), ("table28_log2g", ctypes.c_int32), ("n2_minv28", ctypes.c_uint32),
                ("off_n2_28", ctypes.c_int64), ("off_n2_one28", ctypes.c_int64), ("off_table28", ctypes.c_int64),
                ("off_n2_r2_28", ctypes.c_int64), ("table_window", ctypes.c_int32)]


_PK = ctypes.POINTER(PlKey)
for _name, _args in {
    "efl_pl_encrypt": [_vp, _PK, _vp, _vp, _vp, _i64, _u64, _i64, _vp],
    "efl_pl_fbpowm": [_vp, _PK, _vp, _vp, _i64, _u64, _i64, _vp],
    "efl_pl_crt_join": [_vp, _PK, _vp, _vp, _vp, _vp, _i64, _vp],
    "efl_pl_decrypt": [_vp, _PK, _vp, _vp, _vp, _i64, _vp],
    "efl_pl_add": [_vp, _PK, _vp, _vp, _vp, _i64, _vp],
    "efl_pl_powm": [_vp, _PK, _vp, _vp, _i32, _vp, _i64, _vp],
    "efl_hex_lengths": [_vp, _i32, _vp, _vp, _i64, _vp],
    "efl_hex_write": [_vp, _i32, _vp, _vp, _vp, _i64, _vp],
    "efl_hex_parse": [_vp, _vp, _i32, _vp, _vp, _i64, _vp, _vp],
    "efl_pl_to_int64": [_vp, _i32, _vp, _vp, _i64, _vp],
    "efl_pl_invert": [_vp, _PK, _vp, _vp, _i64, _vp, _vp],
    "efl_pl_matmul": [_vp, _PK, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp],
    "efl_pl_mul_exp2": [_vp, _PK, _vp, _vp, _vp, _i64, _vp, _vp],
    "efl_pl_mul_scalar": [_vp, _PK, _vp, _vp, _vp, _i64, _vp, _vp],
    "efl_pl_mul_scalar_big": [_vp, _PK, _vp, _vp, _i32, _vp, _vp, _i64, _vp, _vp],
    "efl_pl_fxp_add": [_vp, _PK, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp],
    "efl_pl_tune": [_i32, _i32, _i32],
    "efl_host_powm": [_vp, _i32, _vp, _i32, _vp, _i32, _vp],
    "efl_host_sqr_chain": [_vp, _i32, _i32, _i32, _vp, _i32, _vp],
    "efl_host_probable_primes": [_vp, _i32, _i32, _vp, _i32, _i32, _vp],
}.items():
    getattr(_lib, _name).argtypes = _args
    getattr(_lib, _name).restype = _i32


def kernel_slicing(ln: int, decrypt: bool = False) -> int:
    """Kernel family used for keys of `ln` 32-bit limbs: 0 = one lane per element, C = one number
    spread over (2 ln or ln)/C lanes of C limbs (efl_pl_tune)."""
    rc = _lib.efl_pl_tune(ln, int(bool(decrypt)), -1)
    if rc < 0:
        _efl_lib.check(rc)
    return rc


def set_kernel_slicing(ln: int, decrypt: bool, limbs_per_lane: int) -> int:
    """Select the kernel family for keys of `ln` limbs; returns the previous choice."""
    rc = _lib.efl_pl_tune(ln, int(bool(decrypt)), int(limbs_per_lane))
    if rc < 0:
        _efl_lib.check(rc)
    return rc


def reset_kernel_slicing(ln: int, decrypt: bool) -> int:
    """Back to the measured default family (decryption then also sizes it per launch)."""
    rc = _lib.efl_pl_tune(ln, int(bool(decrypt)), -2)
    if rc < 0:
        _efl_lib.check(rc)
    return rc


# kernel families compiled per key size (ln): n^2 ops, decryption
SLICINGS = {16: ([0, 8, 16, 32], [0, 8]), 32: ([0, 8, 16, 32], [0, 8, 16, 32]), 64: ([0, 8, 16, 32], [0, 8, 16, 32]),
            128: ([8, 16, 32], [0, 8, 16, 32]), 256: ([32], [8, 16, 32])}

_LIMB_CLASSES = (16, 32, 64, 128, 256)
MAX_TABLE_BITS = 1 << 40      # gmp_utils.h:20 FBPOWM_MAX_TABLE_MEM, compared against entries x bits
# above this the radix-2^28 copy of the fixed-base table is not built (a table chosen under
# TABLE_MAX_BYTES always has it; an explicit table_window up to 24 may ask for more)
TABLE28_MAX_BYTES = 1 << 36


def _limbs28_rows(vals, L: int, nbytes: int) -> np.ndarray:
    """Many ints -> [len(vals), L] radix-2^28 limbs (vectorised through the little-endian bits)."""
    raw = np.frombuffer(b"".join(v.to_bytes(nbytes, "little") for v in vals), dtype=np.uint8)
    bits = np.unpackbits(raw.reshape(len(vals), nbytes), axis=1, bitorder="little")
    need = 28 * L
    if bits.shape[1] < need:
        bits = np.pad(bits, ((0, 0), (0, need - bits.shape[1])))
    w = (1 << np.arange(28, dtype=np.uint32)).astype(np.uint32)
    return (bits[:, :need].reshape(len(vals), L, 28).astype(np.uint32) * w).sum(axis=2, dtype=np.uint32)


# Device memory the fixed-base table of one key may take, both layouts (round 3; round 2 capped the
# table at 2^18 entries whatever their size). A fresh-randomness encryption costs
# ceil(a_bits / W) (1 - 2^-W) table products, so the widest window that fits is the fastest; the
# lookups of a table larger than the 256 MB Infinity Cache are random HBM reads, and they still pay
# (tools/table_window_probe.py, profiles/r03/table_window_*.jsonl): the examples' 1024-bit key
# 53.9 -> 69.6 M encrypts/s from W = 12 to 16 (1.1 GiB table), the reference default 4096-bit key
# 823 k -> 979 k/s from W = 10 to 12 (1.4 GiB). 1.5 GiB is about half a percent of a 288 GB HBM.
# Round 4: 4 GiB per keypair (profiles/r04/table_window_*.jsonl: the 1024-bit key 65.2 -> 76.2 M
# encrypts/s from W = 16 to 18 (4.0 GiB), 80.8 M/s at W = 20 (14 GiB); the 4096-bit key 0.99 -> 1.07
# -> 1.14 -> 1.22 -> 1.31 M/s from W = 12 to 16 (1.4 -> 17.7 GiB)). A public-key holder spends it on
# its one table; the key owner, whose encryptions go by CRT, on the two CRT sub-tables (half each),
# building its n^2 table only if it is ever walked (KeyBlock.ensure_table). About 1.4 % of a 288 GB
# HBM; EFL_PL_TABLE_MAX_MIB overrides it.
TABLE_MAX_BYTES = 4 << 30
WINDOW_MAX = 24


def table_max_bytes() -> int:
    """The per-keypair table budget: EFL_PL_TABLE_MAX_MIB (MiB) if set, else TABLE_MAX_BYTES."""
    v = os.environ.get("EFL_PL_TABLE_MAX_MIB", "")
    return int(v) << 20 if v else TABLE_MAX_BYTES


def choose_table_window(a_bits: int, entry_bytes: int, max_bytes: int | None = None) -> int:
    """Widest window W <= WINDOW_MAX whose table (ceil(a_bits / W) rows x 2^W - 1 entries of
    entry_bytes: the n^2 words of every layout the key keeps) fits max_bytes (default
    table_max_bytes()). With 4 GiB: 2048-bit a of a 4096-bit n (the reference default) -> W = 13,
    512-bit a of a 1024-bit n (the examples) -> W = 18."""
    if max_bytes is None:
        max_bytes = table_max_bytes()
    best = 1
    for W in range(1, WINDOW_MAX + 1):
        if -(-a_bits // W) * ((1 << W) - 1) * entry_bytes > max_bytes:
            break
        best = W
    return best


def _limbs(x: int, L: int) -> np.ndarray:
    return np.frombuffer(int(x).to_bytes(4 * L, "little"), dtype="<u4").copy()


def _minv32(m: int) -> int:
    return (-pow(m, -1, 1 << 32)) % (1 << 32)


def _limbs28(x: int, L: int) -> np.ndarray:
    """x as L radix-2^28 limbs, one per 32-bit word (csrc/sliced28.h)."""
    return np.array([(x >> (28 * k)) & 0xFFFFFFF for k in range(L)], dtype="<u4")


def table_passes(W: int, cols: int):
    """The table build's doubling passes (KeyBlock._build_table): pass k computes the columns
    (0-based) lo .. lo + cnt - 1, lo = 2^k, as column i times b^(2^k) for i in 0 .. cnt - 1, so column
    c holds b^(c + 1) and every source column was made by an earlier pass."""
    out = []
    for k in range(W):
        lo = 1 << k
        if cols <= lo:
            break
        out.append((lo, min(lo, cols - lo)))
    return out


def limbs28_total(ln: int, G: int) -> int:
    """Limbs of the radix-2^28 form the sliced kernels use for an ln-word modulus over G lanes
    (s28::limbs_per_lane(ln, G) * G: R = 2^(28 L) > 4 m)."""
    return ((32 * ln + 2 + 27) // 28 + G - 1) // G * G


def _hex_of(v) -> str:
    """Scalar hex text from str/bytes/HexTensor/0-d tensor/np array element."""
    if isinstance(v, HexTensor):
        v = v.strings()[0]
    elif isinstance(v, np.ndarray):
        v = v.reshape(-1)[0]
    elif isinstance(v, (list, tuple)):
        v = v[0]
    if isinstance(v, (bytes, bytearray)):
        v = v.decode()
    return str(v)


def _int_of(v) -> int:
    if isinstance(v, torch.Tensor):
        return int(v.reshape(-1)[0].item())
    if isinstance(v, (np.ndarray, list, tuple)):
        return int(np.asarray(v).reshape(-1)[0])
    return int(v)


# ----------------------------------------------------------------------------------------------
# key generation (GeneratePaillierKeypairOp, paillier.cc:833-904), host side, once per session
# ----------------------------------------------------------------------------------------------

_SMALL_PRIMES = [p for p in range(3, 2000) if all(p % d for d in range(2, int(p ** 0.5) + 1))]


def _odd_primes_below(limit: int):
    sieve = bytearray([1]) * limit
    sieve[0:2] = b"\x00\x00"
    for i in range(2, int(limit ** 0.5) + 1):
        if sieve[i]:
            sieve[i * i::i] = bytearray(len(range(i * i, limit, i)))
    return [i for i in range(3, limit) if sieve[i]]


# product of the odd primes below 2^16: one gcd per candidate (after the cheap trial division by
# the primes below 2000) removes 40 % more composites than trial division alone before the
# Miller-Rabin tests (the reference's mpz_probab_prime_p trial-divides first too)
_SIEVE_PRODUCT = math.prod(p for p in _odd_primes_below(1 << 16) if p >= 2000)


def _words(x: int, L: int) -> np.ndarray:
    return np.frombuffer(x.to_bytes(4 * L, "little"), dtype="<u4")


def host_powm(base: int, exp: int, mod: int) -> int:
    """base^exp mod mod (odd mod, 0 <= base < mod) through efl_host_powm (native, host threads)."""
    L = max(1, -(-mod.bit_length() // 32))
    E = max(1, -(-exp.bit_length() // 32))
    b, e, m = _words(base, L), _words(exp, E), _words(mod, L)
    out = np.empty(L, dtype="<u4")
    _efl_lib.check(_lib.efl_host_powm(b.ctypes.data, L, e.ctypes.data, E, m.ctypes.data, L, out.ctypes.data))
    return int.from_bytes(out.tobytes(), "little")


def host_sqr_chain(base: int, k: int, steps: int, mod: int, words: int) -> np.ndarray:
    """[steps, words] little-endian uint32 rows base^(2^(k i)) mod mod (odd mod, base < mod):
    the fixed-base table's row bases, one native call (efl_host_sqr_chain)."""
    b, m = _words(base, words), _words(mod, words)
    out = np.empty((steps, words), dtype="<u4")
    _efl_lib.check(_lib.efl_host_sqr_chain(b.ctypes.data, words, k, steps, m.ctypes.data, words, out.ctypes.data))
    return out


def _sieved(c: int) -> bool:
    for p in _SMALL_PRIMES:
        if c % p == 0:
            return False
    return math.gcd(_SIEVE_PRODUCT % c, c) == 1


def _mr(cands, bases_per, threads=0):
    """efl_host_probable_primes over (candidate, [bases]) pairs; list of bools."""
    L = max(-(-c.bit_length() // 32) for c in cands)
    reps = len(bases_per[0])
    C = np.stack([_words(c, L) for c in cands])
    B = np.stack([np.stack([_words(b, L) for b in bs]) for bs in bases_per])
    out = np.zeros(len(cands), dtype=np.int8)
    _efl_lib.check(_lib.efl_host_probable_primes(C.ctypes.data, L, len(cands), B.ctypes.data, reps, threads,
                                                 out.ctypes.data))
    return [bool(v) for v in out]


def probable_primes(cands, reps: int, rng, threads: int = 0):
    """Miller-Rabin with `reps` random bases each (drawn from rng in candidate order, then round
    order) for odd candidates > 3, on host threads in native code (efl_host_probable_primes): one
    round for every candidate first (almost every composite fails it), then the remaining rounds of
    the survivors side by side, one (candidate, base) per work item. Returns a list of bools."""
    if not cands:
        return []
    bases = [[rng.randrange(2, c - 1) for _ in range(reps)] for c in cands]
    ok = _mr(cands, [b[:1] for b in bases], threads)
    rest = [(i, b) for i, c in enumerate(cands) if ok[i] for b in bases[i][1:]]
    if rest:
        res = _mr([cands[i] for i, _ in rest], [[b] for _, b in rest], threads)
        for (i, _), r in zip(rest, res):
            ok[i] = ok[i] and r
    return ok


def _probable_prime(x: int, reps: int, rng) -> bool:
    if x < 2:
        return False
    for p in _SMALL_PRIMES:
        if x % p == 0:
            return x == p
    return probable_primes([x], reps, rng)[0]


def generate_keypair_ints(n_bytes=512, reps=24, rng=None, batch=None):
    """(n, hs, p, q) with the reference's construction (GeneratePaillierKeypairOp,
    paillier.cc:851-888): primes of n_bytes*4 bits drawn uniformly with bits 0, 1 and the top bit
    set, gcd(p-1, q-1) = 2, hs = (-x^2)^n mod n^2 for a random x in Z_n^*.

    Candidates are drawn `batch` at a time; trial division and one gcd against the product of the
    odd primes below 2^16 discard most composites on the host, a q candidate with
    gcd(p-1, q-1) != 2 is discarded before any primality test (the reference draws both primes
    again instead: the same distribution of accepted pairs, given p), and the survivors of a batch
    get their `reps` Miller-Rabin rounds on host threads in native code (efl_host_probable_primes);
    the first probable prime in draw order is taken. hs is computed by CRT mod p^2 and q^2
    (efl_host_powm) and joined: the same value as the reference's mpz_powm mod n^2."""
    rng = rng or secrets.SystemRandom()
    bits = n_bytes * 4
    if batch is None:
        batch = 64 if bits >= 1024 else 16

    def draw(accept=None):
        while True:
            cs = [rng.getrandbits(bits) | 3 | (1 << (bits - 1)) for _ in range(batch)]
            cs = [c for c in cs if _sieved(c) and (accept is None or accept(c))]
            for c, ok in zip(cs, probable_primes(cs, reps, rng)):
                if ok:
                    return c
    p = draw()
    q = draw(lambda c: c != p and math.gcd(p - 1, c - 1) == 2)
    n = p * q
    while True:
        x = rng.randrange(1, n)
        if math.gcd(x, n) == 1:
            break
    return n, hs_of(x, p, q), p, q


def hs_of(x: int, p: int, q: int) -> int:
    """(-x^2)^n mod n^2 (paillier.cc:884-888) by CRT: the powers mod p^2 and mod q^2 (exponent n
    reduced mod p (p - 1), the order of Z_(p^2)^*) through efl_host_powm, joined by Garner."""
    n = p * q
    h = (-x * x) % n
    p2, q2 = p * p, q * q
    hp = host_powm(h % p2, n % (p * (p - 1)), p2)
    hq = host_powm(h % q2, n % (q * (q - 1)), q2)
    return (hp + p2 * ((hq - hp) * pow(p2, -1, q2) % q2)) % (n * n)


# ----------------------------------------------------------------------------------------------
# device key block
# ----------------------------------------------------------------------------------------------

class KeyBlock:
    """Host derivation + device upload of every constant the kernels read (efl_pl_key)."""

    def __init__(self, n: int, hs: int, a_bits: int, group_size: int, p=None, q=None, device=None,
                 table_window=None, reuse_table=None, walk_start=None, max_bytes=None, defer_table=None):
        """walk_start: the fixed-base walk's accumulator starts from walk_start (mod n^2) instead of 1,
        so efl_pl_fbpowm gives walk_start * hs^(a') mod n^2 (the CRT keys of crt_keys). max_bytes:
        the table's byte budget (default table_max_bytes()). defer_table: build the fixed-base table
        on its first use (ensure_table) instead of now; None = defer exactly when the key owner's
        encryption goes by CRT (crt_capable), which never walks this table."""
        if n.bit_length() < 128:
            raise errors.UnimplementedError("n of fewer than 128 bits is not supported on the GPU")
        if p is not None and q is not None and p == q:
            # q^-1 mod p does not exist: the reference's mpz_invert fails silently there and its
            # decryption is wrong (paillier.cc:88-99); refuse the key instead
            raise errors.InvalidArgumentError("private key: p and q must be distinct")
        if p is not None and q is not None and q >= 2 * p:
            p, q = q, p        # CRT below reduces mq mod p with one subtraction: needs q < 2p
        self.n, self.hs, self.p, self.q = n, hs, p, q
        self.a_bits, self.group_size = a_bits, group_size
        self._window_arg = table_window     # an explicit window also sizes the CRT sub-tables
        self._max_bytes = table_max_bytes() if max_bytes is None else int(max_bytes)
        need = max(n.bit_length(), 2 * max(p or 0, q or 0).bit_length())
        ln = next((c for c in _LIMB_CLASSES if 32 * c >= need), None)
        if ln is None:
            raise errors.UnimplementedError(f"n of {n.bit_length()} bits: at most 8192 supported")
        self.ln, self.lc, self.lh = ln, 2 * ln, ln // 2
        if a_bits <= 0 or a_bits > 8192:
            raise errors.InvalidArgumentError("a_bytes must be in [1, 1024]")
        if group_size < 1 or group_size > 20:
            raise errors.InvalidArgumentError("group_size must be in [1, 20]")
        self.device = device or _efl_lib.require_gpu()
        self.desc = PlKey()
        words = []
        pos = [0]

        def put(x: int, L: int) -> int:
            off = pos[0]
            words.append(_limbs(x, L))
            pos[0] += L
            return off

        d = self.desc
        n2 = n * n
        Rc = 1 << (32 * self.lc)
        d.ln, d.a_bits, d.group_size = ln, a_bits, group_size
        d.off_n = put(n, ln)
        d.off_n2 = put(n2, self.lc)
        d.off_n2_r2 = put(Rc * Rc % n2, self.lc)
        d.off_n2_one = put(Rc % n2, self.lc)
        d.off_max = put(-(-(2 * n) // 3), ln)
        d.n2_minv = _minv32(n2)
        if p is not None and q is not None:
            Rp, Rh = 1 << (32 * ln), 1 << (32 * self.lh)
            d.has_private = 1
            d.off_p, d.off_q = put(p, self.lh), put(q, self.lh)
            d.off_p2, d.off_q2 = put(p * p, ln), put(q * q, ln)
            d.p2_minv, d.q2_minv = _minv32(p * p), _minv32(q * q)
            d.p_minv, d.q_minv = _minv32(p), _minv32(q)
            d.off_p2_r3 = put(pow(Rp, 3, p * p), ln)
            d.off_q2_r3 = put(pow(Rp, 3, q * q), ln)
            d.off_pm1, d.off_qm1 = put(p - 1, self.lh), put(q - 1, self.lh)
            d.pm1_bits, d.qm1_bits = (p - 1).bit_length(), (q - 1).bit_length()
            d.off_pinv_w = put(pow(p, -1, Rh), self.lh)
            d.off_qinv_w = put(pow(q, -1, Rh), self.lh)
            hp = pow((pow(n + 1, p - 1, p * p) - 1) // p, -1, p)      # paillier.cc:28-37
            hq = pow((pow(n + 1, q - 1, q * q) - 1) // q, -1, q)
            d.off_hp = put(hp * Rh % p, self.lh)
            d.off_hq = put(hq * Rh % q, self.lh)
            d.off_qinvp = put(pow(q, -1, p) * Rh % p, self.lh)
            # radix-2^28 constants for the sliced decryption (include/efl_hip.h, csrc/sliced28.h)
            L28s = [limbs28_total(ln, 1 << k) for k in range(6)]
            Lmax = max(L28s)
            d.p2_28_len = Lmax

            def put28(x: int) -> int:
                off = pos[0]
                words.append(_limbs28(x, Lmax))
                pos[0] += Lmax
                return off
            d.off_p2_28, d.off_q2_28 = put28(p * p), put28(q * q)
            d.p2_minv28 = (-pow(p * p, -1, 1 << 28)) % (1 << 28)
            d.q2_minv28 = (-pow(q * q, -1, 1 << 28)) % (1 << 28)
            for k, L28 in enumerate(L28s):
                d.off_p2_r2_28[k] = put28(pow(2, 2 * 28 * L28, p * p))
                d.off_q2_r2_28[k] = put28(pow(2, 2 * 28 * L28, q * q))
        # Fixed-base table (gmp_utils.cc:56-89). The reference builds T[i][j] = hs^((j+1) 2^(g i))
        # with its API group size g and reads it with per-group bit-reversed indices, i.e. it
        # computes hs^(a'), a' = a with every g-bit group reversed. The kernels form a' themselves
        # (pl_common.h regroup_exponent) and walk it in plain windows of THIS table's width W,
        # chosen here for speed: one Montgomery product per non-zero window, so W = 10 cuts the
        # reference default (4096-bit n, g = 1, 2048-bit a) from ~1024 products per encryption
        # to ~205. The reference's size guard still applies to the table it would build.
        g = group_size
        api_rows = a_bits // g + (1 if a_bits % g else 0)
        if api_rows * ((1 << g) - 1) * n2.bit_length() > MAX_TABLE_BITS:
            raise errors.ResourceExhaustedError("Memory usage exceeds a predefined threshold.")
        # radix-2^28 copy of the table for the sliced family the n^2 kernels use (include/efl_hip.h)
        fam = kernel_slicing(ln, False)
        L28 = limbs28_total(2 * ln, 2 * ln // fam) if fam else 0
        W = int(table_window) if table_window else choose_table_window(a_bits, 4 * (self.lc + L28), self._max_bytes)
        if not 1 <= W <= 24:
            raise errors.InvalidArgumentError("table_window must be in [1, 24]")
        cols = (1 << W) - 1
        rows = -(-a_bits // W)
        d.table_rows, d.table_cols, d.table_window = rows, cols, W
        self.table_window = W
        d.off_table28 = -1
        if fam:
            G = 2 * ln // fam
            if rows * cols * L28 * 4 <= TABLE28_MAX_BYTES:
                R28 = 1 << (28 * L28)
                d.n2_28_len, d.table28_log2g = L28, G.bit_length() - 1
                d.n2_minv28 = (-pow(n2, -1, 1 << 28)) % (1 << 28)
                d.off_n2_28 = pos[0]
                words.append(_limbs28(n2, L28))
                pos[0] += L28
                d.off_n2_one28 = pos[0]
                words.append(_limbs28(R28 % n2, L28))
                pos[0] += L28
                d.off_n2_r2_28 = pos[0]
                words.append(_limbs28(R28 * R28 % n2, L28))
                pos[0] += L28
            else:
                L28 = 0
        head = torch.from_numpy(np.concatenate(words).view(np.int32)).to(self.device)
        # the key block without its tables runs the build (n^2 powm / multiply kernels); until a table
        # is attached the descriptor says so (table_rows 0: the encryption entry points refuse)
        self._head = head
        self._tab = (W, rows, cols, L28, d.off_n2_one, walk_start, Rc)
        d.off_table, d.table_rows, d.off_table28 = -1, 0, -1
        self.block, self.ptr = head, head.data_ptr()
        self.has_table = False
        src = reuse_table
        if src is not None and getattr(src, "has_table", False) \
                and (src.n, src.hs, src.a_bits, src.table_window, src.lc) == (n, hs, a_bits, W, self.lc) \
                and torch.device(src.device) == torch.device(self.device) \
                and (src.desc.off_table28 >= 0) == bool(L28) and (not L28 or src.desc.n2_28_len == L28):
            # set_private_key on a key whose public part is unchanged: the tables are the same
            o32, o28 = src.desc.off_table, src.desc.off_table28
            self._attach(src.block[o32:o32 + rows * cols * self.lc],
                         src.block[o28:o28 + rows * cols * L28] if L28 else None)
        elif not (self.crt_capable() if defer_table is None else defer_table):
            self.ensure_table()
        # the key owner's CRT encryption keys (crt_keys), carried over when only the private part
        # was set again
        self._crt = None
        if src is not None and getattr(src, "_crt", None) and (src.p, src.q) == (self.p, self.q) \
                and (src.hs, src.a_bits, src.group_size) == (hs, a_bits, group_size) \
                and torch.device(src.device) == torch.device(self.device):
            self._crt = src._crt
        torch.cuda.current_stream(self.device).synchronize()

    def ensure_table(self):
        """Build and attach the fixed-base table if this key block has none yet (a deferred table:
        the key owner's, whose own encryptions go by CRT). Returns self."""
        if not self.has_table:
            W, rows, cols, L28, r_one, _, _ = self._tab
            t32, t28 = self._build_table(self.hs % (self.n * self.n), self.n * self.n, W, rows, cols, self._head,
                                         r_one, L28)
            self._attach(t32, t28)
            torch.cuda.current_stream(self.device).synchronize()
        return self

    def _attach(self, t32, t28):
        d = self.desc
        head = self._head
        W, rows, cols, L28, _, walk_start, Rc = self._tab
        n2 = self.n * self.n
        parts = [head, t32.reshape(-1)]
        d.table_rows, d.off_table = rows, head.numel()
        if L28:
            d.off_table28 = head.numel() + t32.numel()
            parts.append(t28.reshape(-1))
        self.block = torch.cat(parts)
        if walk_start is not None:   # after the table build, which multiplies by the true R mod n^2
            s0 = walk_start % n2
            self.block[d.off_n2_one:d.off_n2_one + self.lc] = \
                torch.from_numpy(_limbs(s0 * Rc % n2, self.lc).view(np.int32)).to(self.device)
            if L28:
                self.block[d.off_n2_one28:d.off_n2_one28 + L28] = \
                    torch.from_numpy(_limbs28(s0 * (1 << (28 * L28)) % n2, L28).view(np.int32)).to(self.device)
        self.ptr = self.block.data_ptr()
        self.has_table = True

    def crt_capable(self) -> bool:
        """Whether the key owner's encryption goes by CRT (crt_keys): the private key factors n
        (p q = n, p != q), half-length primes of a supported limb class, EFL_PL_CRT_ENCRYPT not 0."""
        if not self.desc.has_private or os.environ.get("EFL_PL_CRT_ENCRYPT", "1") == "0":
            return False
        if self.p == self.q or self.p * self.q != self.n:
            return False
        for x in (self.p, self.q):
            ln_x = next((c for c in _LIMB_CLASSES if 32 * c >= x.bit_length()), None)
            if ln_x is None or 2 * ln_x != self.ln:
                return False
        return True

    def crt_keys(self):
        """The key owner's encryption keys: (KeyBlock of (p, hs mod p^2), KeyBlock of (q, hs mod
        q^2)), built on first use. hs^(a') mod n^2 is then two fixed-base exponentiations on
        half-length moduli (a quarter of the limb products each) and one CRT join
        (efl_pl_crt_join): the same value, bit for bit, as the public-key path. None without the
        private key, with EFL_PL_CRT_ENCRYPT=0, or when p and q are not half-length primes of a
        supported limb class (512-bit n: 256-bit primes). Also None when the private key does not
        factor n (p q != n, or p == q): the reference's Encrypt works mod n^2 only, so such a key
        still encrypts correctly there (paillier.cc:103-131), and the public-key path keeps that."""
        if self._crt is None:
            self._crt = False
            if self.crt_capable():
                subs = []
                p2, q2 = self.p * self.p, self.q * self.q
                R = 1 << (32 * self.lc)   # the n^2 Montgomery radix: the join yields hsa R (efl_pl_crt_join)
                for x, start in ((self.p, R * pow(q2, -1, p2)), (self.q, R * pow(p2, -1, q2))):
                    # the walk mod p^2 yields hs^(a') R (q^2)^-1, mod q^2 hs^(a') R (p^2)^-1: the join
                    # v = q^2 yp + p^2 yq mod n^2 = hs^(a') R then needs no modular product, and
                    # g(m) hs^(a') = mont(g(m), v) is one. The two sub-tables share the keypair's
                    # budget (half each); the key owner's n^2 table is deferred (ensure_table)
                    subs.append(KeyBlock(x, self.hs % (x * x), self.a_bits, self.group_size, device=self.device,
                                         walk_start=start, table_window=self._window_arg,
                                         max_bytes=self._max_bytes // 2, defer_table=False))
                self._crt = tuple(subs)
        return self._crt or None

    def _build_table(self, hs, n2, W, rows, cols, head, r_one, L28, chunk_bytes=64 << 20):
        """T[i][j-1] = hs^(j 2^(W i)) mod n^2 for j in 1..2^W-1, in Montgomery form (x R mod n^2,
        [rows, cols, 2 ln] words) and, with L28, radix-2^28 Montgomery form (x R28 mod n^2,
        [rows, cols, L28] limbs): the table the reference fills with one mpz_mul per entry when a
        keypair is set (gmp_utils.cc:73-88), built here with one GPU product per entry as well.
        One native host call gives every hs^(2^t), t < W rows (efl_host_sqr_chain): P[i][k] =
        b_i^(2^k) for the row base b_i = hs^(2^(W i)). Column 1 is b_i R; pass k then fills columns
        2^k + 1 .. 2^(k+1) of every row at once as column i times P[i][k] (efl_pl_add, which
        multiplies mod n^2: x R * y = x y R), so W passes of independent products replace a chain
        per row. Round 3 ran an efl_pl_powm of b_i^j per entry (about 1.5 W products each). The
        radix-2^28 copy is x R times R28 R^-1 (one more product) cut into 28-bit limbs. Launches
        move at most chunk_bytes of entries."""
        dev, lc = self.device, self.lc
        sh = _stream(dev)
        d = self.desc
        ptr, dp = head.data_ptr(), ctypes.byref(d)

        def mul(dst, a, b, N):
            _efl_lib.check(_lib.efl_pl_add(ptr, dp, a.data_ptr(), b.data_ptr(), dst.data_ptr(), N, sh))

        P = torch.from_numpy(host_sqr_chain(hs, 1, rows * W, n2, lc).view(np.int32)).to(dev).reshape(rows, W, lc)
        t32 = torch.empty((rows, cols, lc), dtype=torch.int32, device=dev)
        ce = max(1, chunk_bytes // (4 * lc))              # entries per launch
        col = torch.empty((rows, lc), dtype=torch.int32, device=dev)
        mul(col, P[:, 0].contiguous(), head[r_one:r_one + lc].expand(rows, lc).contiguous(), rows)
        t32[:, 0] = col
        for k, (lo, cnt) in enumerate(table_passes(W, cols)):
            if cnt >= ce:                                 # long rows: slices of one row, in place
                for r in range(rows):
                    for c0 in range(0, cnt, ce):
                        c1 = min(cnt, c0 + ce)
                        m = P[r, k].expand(c1 - c0, lc).contiguous()
                        mul(t32[r, lo + c0:lo + c1], t32[r, c0:c1], m, c1 - c0)
            else:                                         # short rows: several rows per launch
                rb = max(1, ce // cnt)
                for r0 in range(0, rows, rb):
                    r1 = min(rows, r0 + rb)
                    src = t32[r0:r1, :cnt].contiguous()
                    m = P[r0:r1, k:k + 1].expand(r1 - r0, cnt, lc).contiguous()
                    out = torch.empty_like(src)
                    mul(out, src, m, (r1 - r0) * cnt)
                    t32[r0:r1, lo:lo + cnt] = out
        if not L28:
            return t32, None
        t28 = torch.empty((rows, cols, L28), dtype=torch.int32, device=dev)
        R, R28 = 1 << (32 * lc), 1 << (28 * L28)
        c28 = torch.from_numpy(_limbs(R28 * pow(R, -1, n2) % n2, lc).view(np.int32)).to(dev)
        q, r = divmod(np.arange(L28) * 28, 32)
        qi = torch.from_numpy(q).to(dev)
        rs = torch.from_numpy(r).to(dev)
        pad = int(q.max()) + 2 - lc                       # x R28 mod n^2 < 2^(32 lc): words past lc are 0
        flat32, flat28 = t32.reshape(-1, lc), t28.reshape(-1, L28)
        total = rows * cols
        ce28 = max(1, ce // 4)                            # the int64 staging below is 4x the entries
        for e0 in range(0, total, ce28):
            e1 = min(total, e0 + ce28)
            N = e1 - e0
            X = torch.empty((N, lc), dtype=torch.int32, device=dev)
            mul(X, flat32[e0:e1], c28.expand(N, lc).contiguous(), N)
            w = torch.cat([X.to(torch.int64) & 0xFFFFFFFF,
                           torch.zeros((N, max(1, pad)), dtype=torch.int64, device=dev)], dim=1)
            flat28[e0:e1] = (((w[:, qi] >> rs) | (w[:, qi + 1] << (32 - rs))) & 0xFFFFFFF).to(torch.int32)
        return t32, t28

    def args(self):
        return self.ptr, ctypes.byref(self.desc)


# ----------------------------------------------------------------------------------------------
# ciphertext tensors
# ----------------------------------------------------------------------------------------------

def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def limbs_to_hex(limbs: torch.Tensor, neg: torch.Tensor | None, shape) -> HexTensor:
    """[N, L] uint32 limbs (+ optional sign bytes) -> device HexTensor (mpz_get_str(..., 16))."""
    N, L = limbs.shape[0], limbs.shape[1]
    dev = limbs.device
    lens = torch.empty(N, dtype=torch.int64, device=dev)
    negp = neg.data_ptr() if neg is not None else None
    _efl_lib.check(_lib.efl_hex_lengths(limbs.data_ptr(), L, negp, lens.data_ptr(), N, _stream(dev)))
    offs = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    if N:
        torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item()) if N else 0
    chars = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    _efl_lib.check(_lib.efl_hex_write(limbs.data_ptr(), L, negp, offs.data_ptr(), chars.data_ptr(), N,
                                      _stream(dev)))
    return HexTensor.from_device(chars, offs, shape)


def hex_to_limbs(hx: HexTensor, L: int, device, signed=False):
    """HexTensor -> ([N, L] limbs, sign bytes or None); InvalidArgument on malformed/too wide text."""
    N = hx.numel()
    chars, offs = hx.device_buffers(device)
    limbs = torch.empty((N, L), dtype=torch.int32, device=device)
    neg = torch.empty(N, dtype=torch.int8, device=device) if signed else None
    bad = torch.empty(1, dtype=torch.int64, device=device)
    _efl_lib.check(_lib.efl_hex_parse(chars.data_ptr(), offs.data_ptr(), L, limbs.data_ptr(),
                                      neg.data_ptr() if neg is not None else None, N, bad.data_ptr(),
                                      _stream(device)))
    b = int(bad.item())
    if b >= 0:
        raise errors.InvalidArgumentError(f"element {b} is not a hex integer of at most {32 * L} bits: "
                                          f"{hx.strings()[b][:40]!r}")
    return limbs, neg


class CipherTensor:
    """Paillier ciphertexts in HBM: limbs [N, 2*ln] (int32 storage of uint32 limbs) + shape."""

    def __init__(self, limbs: torch.Tensor, shape, key: KeyBlock):
        self.limbs, self.shape, self.key = limbs, tuple(int(s) for s in shape), key

    def numel(self):
        return self.limbs.shape[0]

    def to_hex(self) -> HexTensor:
        return limbs_to_hex(self.limbs, None, self.shape)

    def reshape(self, shape):
        shape = tuple(int(s) for s in shape)
        if -1 in shape:
            known = int(np.prod([s for s in shape if s != -1])) or 1
            shape = tuple(self.numel() // known if s == -1 else s for s in shape)
        return CipherTensor(self.limbs, shape, self.key)

    def transpose(self):
        r, c = self.shape
        idx = torch.arange(r * c, device=self.limbs.device).reshape(r, c).t().reshape(-1)
        return CipherTensor(self.limbs[idx].contiguous(), (c, r), self.key)

    def __repr__(self):
        return f"CipherTensor(shape={self.shape}, {32 * self.limbs.shape[1]}-bit)"


# ----------------------------------------------------------------------------------------------
# public API (efl.paillier.*)
# ----------------------------------------------------------------------------------------------

@exporter.export("paillier.Tensor")
class PaillierTensor(object):
    """paillier.py:29-50."""

    def __init__(self, keypair, tensor):
        self.keypair = keypair
        self.tensor = tensor

    def __add__(self, another):
        if not isinstance(another, PaillierTensor):
            another = self.keypair.encrypt(another)
        return PaillierTensor(self.keypair, self.keypair.add(self.tensor, another.tensor))

    def __mul__(self, scalar):
        return PaillierTensor(self.keypair, self.keypair.mul_scalar(self.tensor, scalar))

    def decrypt(self, dtype="string"):
        return self.keypair.decrypt(self, dtype)

    def __lshift__(self, exp):
        return PaillierTensor(self.keypair, self.keypair.mul_exp2(self.tensor, exp))

    @property
    def shape(self):
        return self.tensor.shape


def _is_string_dtype(dtype) -> bool:
    return dtype in ("string", str, bytes, "str") or getattr(dtype, "name", None) == "string"


def philox_key(seed: bytes | int | None = None) -> int:
    """64-bit Philox4x32-10 key of a keypair's randomness stream. Bytes (the 32-byte seed rank 0
    broadcasts, efl.distributed) are hashed whole (BLAKE2b-64), so every seed byte matters; an int
    is taken mod 2^64; None draws from os.urandom. Philox is a counter-based generator, not a
    cryptographic PRF; it replaces the reference's time()-seeded MT19937 (paillier.cc:54-57), which
    is weaker still (Randomness)."""
    if seed is None:
        seed = os.urandom(32)
    if isinstance(seed, (bytes, bytearray)):
        return int.from_bytes(hashlib.blake2b(bytes(seed), digest_size=8).digest(), "little")
    return int(seed) & ((1 << 64) - 1)


@exporter.export("paillier.Keypair")
class PaillierKeypair(object):
    """paillier.py:53-104 over the PaillierKeypair resource (paillier.cc:50-331)."""

    # the key owner's fresh-randomness encryption and fbpowm go through CRT (KeyBlock.crt_keys);
    # False (or EFL_PL_CRT_ENCRYPT=0) keeps them on n^2 as the reference does. Same ciphertexts.
    crt_encrypt = True

    def __init__(self, seed: bytes | int | None = None):
        self._key: KeyBlock | None = None
        self._n_bytes = None
        self.seed = philox_key(seed)
        self.counter = 0

    # -- key management ------------------------------------------------------------------
    def initialize(self):
        """CreatePaillierKeypair: the resource exists from construction; kept for the API."""
        return None

    def generate_keypair(self, n_bytes=None, reps=None, a_bytes=None, group_size=None, rng=None):
        """GeneratePaillierKeypair (attr defaults n_bytes=512, a_bytes=256, reps=24, group_size=1).
        Returns (public_key [n, hs], private_key [p, q]) as HexTensors."""
        n_bytes = 512 if n_bytes is None else int(n_bytes)
        a_bytes = 256 if a_bytes is None else int(a_bytes)
        reps = 24 if reps is None else int(reps)
        group_size = 1 if group_size is None else int(group_size)
        n, hs, p, q = generate_keypair_ints(n_bytes, reps, rng)
        self._set(n, n_bytes, hs, a_bytes, group_size, p, q)
        return HexTensor.from_ints([n, hs]), HexTensor.from_ints([p, q])

    def set_public_key(self, n, n_bytes, hs, a_bytes, group_size=None):
        """SetPaillierPublicKey. As in paillier.py:69-70 the group_size argument is not forwarded:
        the table is built with the op's default group size 1."""
        self._set(int(_hex_of(n), 16), _int_of(n_bytes), int(_hex_of(hs), 16), _int_of(a_bytes), 1)

    def set_private_key(self, p, q):
        """SetPaillierPrivateKey (ignored without a public key, paillier.cc:88-91)."""
        if self._key is None:
            return
        k = self._key
        self._set(k.n, self._n_bytes, k.hs, k.a_bits // 8, k.group_size,
                  int(_hex_of(p), 16), int(_hex_of(q), 16))

    def set_keys_ints(self, n, hs, a_bytes, group_size=1, p=None, q=None, n_bytes=None, table_window=None):
        """Host-int variant of set_public_key/set_private_key (tests, key exchange). table_window
        forces the fixed-base table's window (default: choose_table_window; results never change)."""
        self._set(n, n_bytes or (n.bit_length() + 7) // 8, hs, a_bytes, group_size, p, q, table_window)

    def _set(self, n, n_bytes, hs, a_bytes, group_size, p=None, q=None, table_window=None):
        old = self._key
        if old is not None and (old.n, old.hs) != (n, hs):
            # a new public key (a re-key): nothing of the old block can be reused, so the keypair
            # lets go of it, and of the key owner's CRT sub-tables, before the new table is built.
            # Ciphertexts that still reference the old block keep it alive; its sub-tables only
            # ever served this keypair's own encryptions.
            old._crt = None
            self._key = old = None
        self._key = KeyBlock(n, hs, 8 * int(a_bytes), int(group_size), p, q, table_window=table_window,
                             reuse_table=old)
        self._n_bytes = n_bytes

    @property
    def key(self) -> KeyBlock:
        if self._key is None:
            raise errors.AbortedError("No public key.")
        return self._key

    @property
    def public_key(self):
        return self.key.n, self.key.hs

    # -- conversions ---------------------------------------------------------------------
    def _cipher(self, x) -> CipherTensor:
        """PaillierTensor / CipherTensor / HexTensor / strings -> CipherTensor of this key."""
        if isinstance(x, PaillierTensor):
            x = x.tensor
        if isinstance(x, CipherTensor):
            return x
        k = self.key
        hx = x if isinstance(x, HexTensor) else HexTensor.from_strings(x)
        limbs, _ = hex_to_limbs(hx, k.lc, k.device)
        return CipherTensor(limbs, hx.shape, k)

    # -- ops -----------------------------------------------------------------------------
    def _crt_encrypt(self, m, n, counter_base, a_dev=None):
        """The key owner's path (KeyBlock.crt_keys): ciphertexts of the int64 device tensor m ([n, 2 ln]
        limbs) for the Philox draws at counters counter_base + i (or the given exponents a_dev) —
        m = 0 gives hs^(a') itself. None when this keypair cannot take it."""
        k = self.key
        subs = k.crt_keys() if self.crt_encrypt else None
        if subs is None or n == 0:
            return None
        sh = _stream(k.device)
        parts = []
        for sk in subs:
            x = torch.empty((n, sk.lc), dtype=torch.int32, device=k.device)
            _efl_lib.check(_lib.efl_pl_fbpowm(*sk.args(), a_dev.data_ptr() if a_dev is not None else None,
                                              x.data_ptr(), n, self.seed, counter_base, sh))
            parts.append(x)
        z = torch.empty((n, k.lc), dtype=torch.int32, device=k.device)
        _efl_lib.check(_lib.efl_pl_crt_join(*k.args(), parts[0].data_ptr(), parts[1].data_ptr(), m.data_ptr(),
                                            z.data_ptr(), n, sh))
        return z

    def encrypt(self, plaintext, hsa=None, counter_base=None):
        """PaillierEncrypt (paillier.cc:443-503). hsa None (or all "0") draws a fresh a per element
        from Philox(seed, counter); counter_base defaults to a running per-keypair counter."""
        k = self.key
        m = _efl_lib.as_tensor(plaintext)
        if m.dtype != torch.int64:
            m = m.to(torch.int64)
        shape = tuple(m.shape)
        m = m.reshape(-1).contiguous().to(k.device)
        N = m.numel()
        out = torch.empty((N, k.lc), dtype=torch.int32, device=k.device)
        hsa_limbs = None
        if hsa is not None:
            hx = hsa if isinstance(hsa, HexTensor) else HexTensor.from_strings(hsa)
            if hx.numel() != N:
                raise errors.InvalidArgumentError("plaintext and hsa should be the same size.")
            strs_zero = np.array([s in ("0", "-0", "") for s in hx.strings()]) if N else np.zeros(0, bool)
            if not strs_zero.all():
                hsa_limbs, _ = hex_to_limbs(hx, k.lc, k.device)
            zero_idx = np.nonzero(strs_zero)[0] if hsa_limbs is not None else None
        # element i draws its a from Philox counter ctr + i: the call owns [ctr, ctr + N) and the
        # running counter moves past it, so no two elements of any two calls share an a (a shared
        # a gives equal hs^a factors, and the quotient of the two ciphertexts reveals m1 - m2)
        ctr = self.counter if counter_base is None else int(counter_base)
        if counter_base is None:
            self.counter += N
        crt = self._crt_encrypt(m, N, ctr) if hsa_limbs is None else None   # the key owner: by CRT, same bits
        if crt is not None:
            out = crt
        else:
            if hsa_limbs is None:
                k.ensure_table()          # fresh randomness walks the n^2 table
            _efl_lib.check(_lib.efl_pl_encrypt(*k.args(), m.data_ptr(),
                                               hsa_limbs.data_ptr() if hsa_limbs is not None else None,
                                               out.data_ptr(), N, self.seed, ctr, _stream(k.device)))
        if hsa_limbs is not None and zero_idx is not None and zero_idx.size:
            # the rows whose hsa is "0" draw a fresh a at their own index's counter (ctr + idx),
            # inside this call's range: rows with a given hsa consume no counter
            idx = torch.from_numpy(zero_idx).to(k.device)
            sub = torch.empty((idx.numel(), k.lc), dtype=torch.int32, device=k.device)
            msub = m[idx].contiguous()
            for j0, j1, c0 in _counter_runs(zero_idx):
                h = self._crt_encrypt(msub[j0:j1], j1 - j0, ctr + c0)
                if h is not None:
                    sub[j0:j1] = h
                    continue
                k.ensure_table()
                _efl_lib.check(_lib.efl_pl_encrypt(*k.args(), msub[j0:j1].data_ptr(), None, sub[j0:j1].data_ptr(),
                                                   j1 - j0, self.seed, ctr + c0, _stream(k.device)))
            out[idx] = sub
        return PaillierTensor(self, CipherTensor(out, shape, k))

    def fbpowm(self, a=None, n=None, counter_base=None):
        """hs^(a') mod n^2 for given exponents (Python ints) or the Philox draw (FixedBasePowm).
        A Philox draw takes its counters from the running counter (like encrypt) unless
        counter_base is given, so it never repeats an a an encryption used."""
        k = self.key
        if a is None:
            if counter_base is None:
                counter_base = self.counter
                self.counter += int(n)
        else:
            counter_base = 0
        words = (k.a_bits + 31) // 32
        if a is not None:
            a = list(a)
            n = len(a)
            if any(v < 0 or v.bit_length() > k.a_bits for v in a):
                raise errors.InvalidArgumentError("exponent wider than the fixed-base table")
            arr = np.stack([_limbs(v, words) for v in a]) if n else np.zeros((0, words), "<u4")
            a_dev = torch.from_numpy(arr.view(np.int32)).to(k.device)
        zeros = torch.zeros(n, dtype=torch.int64, device=k.device)   # g(0) = 1: the join gives hs^(a')
        out = self._crt_encrypt(zeros, n, counter_base, a_dev if a is not None else None)
        if out is None:
            out = torch.empty((n, k.lc), dtype=torch.int32, device=k.device)
            k.ensure_table()
            _efl_lib.check(_lib.efl_pl_fbpowm(*k.args(), a_dev.data_ptr() if a is not None else None,
                                              out.data_ptr(), n, self.seed, counter_base, _stream(k.device)))
        return CipherTensor(out, (n,), k)

    def decrypt(self, paillier_tensor, dtype="string"):
        """PaillierDecrypt (paillier.cc:505-561): HexTensor of the signed plaintext (default) or
        int64 (mpz_get_sll semantics)."""
        k = self.key
        if not k.desc.has_private:
            raise errors.AbortedError("No private key.")
        c = self._cipher(paillier_tensor)
        N = c.numel()
        mag = torch.empty((N, k.ln), dtype=torch.int32, device=k.device)
        neg = torch.empty(N, dtype=torch.int8, device=k.device)
        _efl_lib.check(_lib.efl_pl_decrypt(*k.args(), c.limbs.data_ptr(), mag.data_ptr(), neg.data_ptr(), N,
                                           _stream(k.device)))
        if _is_string_dtype(dtype):
            return limbs_to_hex(mag, neg, c.shape)
        if _efl_lib.to_torch_dtype(dtype) != torch.int64:
            raise errors.InvalidArgumentError("PaillierDecrypt: dtype must be string or int64")
        out = torch.empty(N, dtype=torch.int64, device=k.device)
        _efl_lib.check(_lib.efl_pl_to_int64(mag.data_ptr(), k.ln, neg.data_ptr(), out.data_ptr(), N,
                                            _stream(k.device)))
        return out.reshape(c.shape)

    def add(self, x, y):
        """PaillierAdd: z = x * y mod n^2 (paillier.py:75-79 broadcasts first)."""
        k = self.key
        x, y = self._cipher(x), self._cipher(y)
        x, y = _broadcast_pair(x, y)
        out = torch.empty_like(x.limbs)
        _efl_lib.check(_lib.efl_pl_add(*k.args(), x.limbs.data_ptr(), y.limbs.data_ptr(), out.data_ptr(),
                                       x.numel(), _stream(k.device)))
        return CipherTensor(out, x.shape, k)

    def invert(self, x):
        """PaillierInvert: x^-1 mod n^2 (paillier.cc:267-285, 721-797)."""
        k = self.key
        x = self._cipher(x)
        out = torch.empty_like(x.limbs)
        bad = torch.empty(1, dtype=torch.int64, device=k.device)
        _efl_lib.check(_lib.efl_pl_invert(*k.args(), x.limbs.data_ptr(), out.data_ptr(), x.numel(),
                                          bad.data_ptr(), _stream(k.device)))
        b = int(bad.item())
        if b >= 0:
            raise errors.InvalidArgumentError(f"element {b} has no inverse mod n^2")
        return CipherTensor(out, x.shape, k)

    def mul_scalar(self, x, scalar):
        """PaillierMulScalar (paillier.cc:180-265, :616-678): z = x^y mod n^2. T = int32/int64
        (torch/numpy integers, Python ints of int64 range): efl_pl_mul_scalar, which computes
        x^|y| and inverts it where y < 0 — the element the reference forms as (x^-1)^|y|. T = string
        (str / bytes / HexTensor, or Python ints wider than int64): signed hex big integers parsed
        on the GPU as mpz_init_set_str(op, y, 16) does (:239-248), then efl_pl_mul_scalar_big.
        x and y broadcast against each other first (paillier.py:81-85)."""
        k = self.key
        x = self._cipher(x)
        y = _scalar_operand(scalar, k.device)
        shape = _broadcast_shape(x.shape, y.shape)
        x = _expand(x, shape)
        N = x.numel()
        out = torch.empty_like(x.limbs)
        bad = torch.empty(1, dtype=torch.int64, device=k.device)
        if isinstance(y, HexTensor):
            y = _expand_hex(y, shape)
            L = max(1, _hex_words(y))
            mag, neg = hex_to_limbs(y, L, k.device, signed=True)
            _efl_lib.check(_lib.efl_pl_mul_scalar_big(*k.args(), x.limbs.data_ptr(), mag.data_ptr(), L, neg.data_ptr(),
                                                      out.data_ptr(), N, bad.data_ptr(), _stream(k.device)))
        else:
            y = y.expand(shape).reshape(-1).contiguous()
            _efl_lib.check(_lib.efl_pl_mul_scalar(*k.args(), x.limbs.data_ptr(), y.data_ptr(), out.data_ptr(), N,
                                                  bad.data_ptr(), _stream(k.device)))
        b = int(bad.item())
        if b >= 0:
            raise errors.InvalidArgumentError(f"element {b} has no inverse mod n^2 (a negative scalar needs x^-1)")
        return CipherTensor(out, shape, k)

    def matmul(self, xm, xe, ym, ye):
        """PaillierMatmul (paillier.cc:915-1053): ciphertext [u, v] x plaintext fixed-point [v, w]
        -> (ciphertext mantissa [u, w], exponent [u, w])."""
        k = self.key
        x = self._cipher(xm)
        xe = _efl_lib.as_tensor(xe).to(k.device, torch.int64).contiguous()
        ym = _efl_lib.as_tensor(ym).to(k.device, torch.int64).contiguous()
        ye = _efl_lib.as_tensor(ye).to(k.device, torch.int64).contiguous()
        if len(x.shape) != 2:
            raise errors.InvalidArgumentError("the rank of x should be two.")
        if ym.dim() != 2:
            raise errors.InvalidArgumentError("the rank of y should be two.")
        if tuple(xe.shape) != x.shape:
            raise errors.InvalidArgumentError("x_mantissa and x_exponent should be the same size.")
        if ym.shape != ye.shape:
            raise errors.InvalidArgumentError("y_mantissa and y_exponent should be the same size.")
        u, v = x.shape
        if ym.shape[0] != v:
            raise errors.InvalidArgumentError("the size of x's 1st dim should be equal to the size of y's 2nd dim.")
        w = ym.shape[1]
        if u and v and w:
            rx = torch.stack([xe.max() - xe.min(), ye.max() - ye.min()]).tolist()
            if rx[0] + rx[1] > MATMUL_MAX_SPREAD:
                return self._matmul_composed(x, xe, ym, ye)
        zpos = torch.empty((u * w, k.lc), dtype=torch.int32, device=k.device)
        zneg = torch.empty_like(zpos)
        ze = torch.empty((u, w), dtype=torch.int64, device=k.device)
        _efl_lib.check(_lib.efl_pl_matmul(*k.args(), x.limbs.data_ptr(), xe.data_ptr(), ym.data_ptr(), ye.data_ptr(),
                                          zpos.data_ptr(), zneg.data_ptr(), ze.data_ptr(), u, v, w,
                                          _stream(k.device)))
        if bool((ym < 0).any()):
            inv = self.invert(CipherTensor(zneg, (u * w,), k))
            z = self.add(CipherTensor(zpos, (u * w,), k), inv)
            return CipherTensor(z.limbs, (u, w), k), ze
        return CipherTensor(zpos, (u, w), k), ze

    def _matmul_composed(self, x, xe, ym, ye):
        """PaillierMatmul term by term, as the reference forms it (paillier.cc:1008-1034): term (i, j, k)
        = x_ij^y_jk (PaillierMulScalar; x^-1 for y < 0) shifted by 2^(xe_ij + ye_jk - m_ik), m_ik the
        minimum over j, and the terms of an output multiplied mod n^2. Used when the exponents spread
        past MATMUL_MAX_SPREAD: the shifts then run through _exp2_chunked's bounded launches. The
        product is exact, so the ciphertexts equal efl_pl_matmul's; rows go in chunks of about
        _COMPOSED_CHUNK_BYTES (256 MiB) of terms."""
        k = self.key
        u, v = x.shape
        w = ym.shape[1]
        rows = max(1, _COMPOSED_CHUNK_BYTES // (v * w * k.lc * 4))
        zs, ms = [], []
        for i0 in range(0, u, rows):
            i1 = min(u, i0 + rows)
            r = i1 - i0
            xr = CipherTensor(x.limbs[i0 * v:i1 * v], (r, v, 1), k)
            t = self.mul_scalar(xr, ym.reshape(1, v, w))                          # [r, v, w]
            s = xe[i0:i1].reshape(r, v, 1) + ye.reshape(1, v, w)
            m = s.amin(dim=1)                                                      # [r, w]
            t = self._exp2_chunked(t.limbs, (s - m.reshape(r, 1, w)).reshape(-1).contiguous())
            t = t.view(r, v, w, k.lc)
            while t.shape[1] > 1:                                                  # product over j
                h = t.shape[1] // 2
                a = t[:, :h].contiguous()
                b = t[:, h:2 * h].contiguous()
                p = torch.empty_like(a)
                _efl_lib.check(_lib.efl_pl_add(*k.args(), a.data_ptr(), b.data_ptr(), p.data_ptr(),
                                               r * h * w, _stream(k.device)))
                t = torch.cat([p, t[:, 2 * h:]], dim=1) if t.shape[1] % 2 else p
            zs.append(t.reshape(r * w, k.lc))
            ms.append(m)
        return CipherTensor(torch.cat(zs).contiguous(), (u, w), k), torch.cat(ms)

    def mul_exp2(self, x, exp):
        """PaillierMulExp2 (paillier.cc:680-751): z = x^(2^y) mod n^2, y int32/int64 >= 0, y
        squarings per element on the GPU (efl_pl_mul_exp2). x and y broadcast first (paillier.py:87-91).
        A launch squares at most MAX_SHIFT times per element; longer shifts are cut into launches of
        at most that many (_exp2_chunked), so any y >= 0 is computed as the reference computes it."""
        k = self.key
        x = self._cipher(x)
        y = _scalar_operand(exp, k.device)
        if isinstance(y, HexTensor):
            raise errors.InvalidArgumentError("PaillierMulExp2: y must be int32 or int64")
        shape = _broadcast_shape(x.shape, y.shape)
        x = _expand(x, shape)
        y = y.expand(shape).reshape(-1).contiguous()
        out, b = self._exp2_launch(x.limbs, y)
        if b >= 0:
            if int(y[b].item()) < 0:
                raise errors.InvalidArgumentError("y should be a positive tensor.")
            out = self._exp2_chunked(x.limbs, y)
        return CipherTensor(out, shape, k)

    def _exp2_launch(self, limbs, y):
        """One efl_pl_mul_exp2 launch: (out, index of the first element with y < 0 or y > MAX_SHIFT,
        or -1)."""
        k = self.key
        out = torch.empty_like(limbs)
        bad = torch.empty(1, dtype=torch.int64, device=k.device)
        _efl_lib.check(_lib.efl_pl_mul_exp2(*k.args(), limbs.data_ptr(), y.data_ptr(), out.data_ptr(),
                                            limbs.shape[0], bad.data_ptr(), _stream(k.device)))
        return out, int(bad.item())

    def _exp2_chunked(self, limbs, y):
        """x^(2^y) for shifts past one launch's MAX_SHIFT squarings: x^(2^(a + b)) = (x^(2^a))^(2^b),
        so each launch squares every element min(remaining, MAX_SHIFT) times (0 = the element passes
        through) until no element has squarings left. Like the reference's y squarings
        (paillier.cc:728-731) the work grows with y; each launch stays bounded."""
        if bool((y < 0).any()):
            raise errors.InvalidArgumentError("y should be a positive tensor.")
        rem = y.clone()
        cur = limbs
        while True:
            step = torch.clamp(rem, max=_SHIFT_CHUNK)
            cur, b = self._exp2_launch(cur, step)
            if b >= 0:   # cannot happen: every step is within [0, MAX_SHIFT]
                raise errors.InternalError(f"shift chunk of element {b} refused")
            rem -= step
            if not bool((rem > 0).any()):
                return cur

    def shift_add(self, x, x_exponent, y, y_exponent):
        """The ciphertext half of FixedPointTensor.__add__ (paillier.py:119-132):
        (x << dl) + (y << dr) = x^(2^(xe - m)) * y^(2^(ye - m)) mod n^2, m = min(xe, ye), as ONE
        launch (efl_pl_fxp_add) instead of two PaillierMulExp2 and a PaillierAdd; the same ciphertext
        bits. Everything broadcasts to one shape. Returns (CipherTensor, m)."""
        k = self.key
        x, y = self._cipher(x), self._cipher(y)
        xe = _efl_lib.as_tensor(x_exponent).to(k.device, torch.int64)
        ye = _efl_lib.as_tensor(y_exponent).to(k.device, torch.int64)
        shape = _broadcast_shape(_broadcast_shape(x.shape, y.shape), _broadcast_shape(tuple(xe.shape), tuple(ye.shape)))
        x, y = _expand(x, shape), _expand(y, shape)
        xe = xe.expand(shape).reshape(-1).contiguous()
        ye = ye.expand(shape).reshape(-1).contiguous()
        out = torch.empty_like(x.limbs)
        bad = torch.empty(1, dtype=torch.int64, device=k.device)
        _efl_lib.check(_lib.efl_pl_fxp_add(*k.args(), x.limbs.data_ptr(), xe.data_ptr(), y.limbs.data_ptr(),
                                           ye.data_ptr(), out.data_ptr(), x.numel(), bad.data_ptr(), _stream(k.device)))
        b = int(bad.item())
        m = torch.minimum(xe, ye)
        if b >= 0:
            # a shift past one launch's squarings: the reference's own composition (two
            # PaillierMulExp2, one PaillierAdd), the shifts cut into bounded launches
            xs = self._exp2_chunked(x.limbs, xe - m)
            ys = self._exp2_chunked(y.limbs, ye - m)
            out = torch.empty_like(xs)
            _efl_lib.check(_lib.efl_pl_add(*k.args(), xs.data_ptr(), ys.data_ptr(), out.data_ptr(), x.numel(),
                                           _stream(k.device)))
        return CipherTensor(out, shape, k), m.reshape(shape)


MAX_SHIFT = 1 << 16   # pl_common.h kMaxShift: squarings per element in one launch
_SHIFT_CHUNK = MAX_SHIFT   # squarings per launch of _exp2_chunked (tests lower it; never above MAX_SHIFT)
# PaillierMatmul: an exponent spread (max - min of x_exponent plus that of y_exponent) past this
# runs as the reference's per-term composition (_matmul_composed) instead of one efl_pl_matmul,
# whose bit-level loop would spend that many squarings per output in one launch
MATMUL_MAX_SPREAD = MAX_SHIFT
_COMPOSED_CHUNK_BYTES = 256 << 20   # terms of _matmul_composed per row chunk



def _scalar_operand(s, device):
    """The y operand of PaillierMulScalar / PaillierMulExp2 (TF T = int32/int64/string): an int64
    tensor on `device`, or a HexTensor of signed hex integers for the string variant (and for Python
    ints beyond int64, which only the string variant can carry)."""
    if isinstance(s, HexTensor):
        return s
    if isinstance(s, torch.Tensor):
        if s.dtype.is_floating_point or s.dtype.is_complex or s.dtype == torch.bool:
            raise errors.InvalidArgumentError(f"scalar dtype must be int32, int64 or string, got {s.dtype}")
        return s.to(device, torch.int64)
    if isinstance(s, (str, bytes, bytearray)):
        return HexTensor.from_strings([s], shape=())
    a = np.asarray(s) if not isinstance(s, np.ndarray) else s
    if a.dtype.kind in "iu":
        if a.dtype == np.uint64 and a.size and int(a.max()) >= 1 << 63:
            return HexTensor.from_ints([int(v) for v in a.reshape(-1)], a.shape)
        return torch.from_numpy(np.ascontiguousarray(a, np.int64)).to(device)
    if a.dtype.kind in "USO":
        flat = a.reshape(-1).tolist()
        if all(isinstance(v, (int, np.integer)) and not isinstance(v, bool) for v in flat):
            if all(-(1 << 63) <= int(v) < (1 << 63) for v in flat):
                return torch.tensor([int(v) for v in flat], dtype=torch.int64).reshape(a.shape).to(device)
            return HexTensor.from_ints([int(v) for v in flat], a.shape)
        if all(isinstance(v, (str, bytes, bytearray, np.str_, np.bytes_)) for v in flat):
            return HexTensor.from_strings(np.array(flat, dtype=object).reshape(a.shape))
    raise errors.InvalidArgumentError(f"scalar must be int32, int64 or string, got {a.dtype}")


def _hex_words(hx: HexTensor) -> int:
    """32-bit words that hold the widest text's magnitude (8 hex digits per word)."""
    offs = hx.offs
    if hx.numel() == 0:
        return 1
    return int(((offs[1:] - offs[:-1]).max() + 7) // 8)


def _expand_hex(hx: HexTensor, shape) -> HexTensor:
    if hx.shape == tuple(shape):
        return hx
    idx = np.broadcast_to(np.arange(hx.numel()).reshape(hx.shape), shape).reshape(-1)
    return hx.take(idx, shape)


def _counter_runs(idx: np.ndarray):
    """Sorted element indices -> (j0, j1, first index) runs of consecutive indices, so each run
    is one launch whose element t draws counter (first index + t)."""
    runs = []
    j0 = 0
    for j in range(1, idx.size + 1):
        if j == idx.size or idx[j] != idx[j - 1] + 1:
            runs.append((j0, j, int(idx[j0])))
            j0 = j
    return runs


def _broadcast_shape(a, b):
    return tuple(np.broadcast_shapes(tuple(a), tuple(b)))


def _broadcast_pair(x: CipherTensor, y: CipherTensor):
    shape = _broadcast_shape(x.shape, y.shape)
    return _expand(x, shape), _expand(y, shape)


def _expand(x: CipherTensor, shape) -> CipherTensor:
    if x.shape == shape:
        return x
    idx = torch.arange(x.numel(), device=x.limbs.device).reshape(x.shape).expand(shape).reshape(-1)
    return CipherTensor(x.limbs[idx].contiguous(), shape, x.key)


# ----------------------------------------------------------------------------------------------
# FixedPointTensor arithmetic with encrypted mantissas (paillier.py:116-145)
# ----------------------------------------------------------------------------------------------

def _fp_encode(v):
    from efl.privacy.paillier import FixedPointTensor, fixedpoint_encode
    return v if isinstance(v, FixedPointTensor) else fixedpoint_encode(v)


def fixedpoint_add(self, another):
    """FixedPointTensor.__add__ (paillier.py:116-133): align exponents with mul_exp2 shifts, then
    add in ciphertext space; a plaintext side is encrypted with the other side's keypair. The shifts
    and the add run as one launch (PaillierKeypair.shift_add): bit-identical to
    (self_m << dl) + (another_m << dr)."""
    from efl.privacy.paillier import FixedPointTensor
    another = _fp_encode(another)
    se, ae = _efl_lib.as_tensor(self.exponent), _efl_lib.as_tensor(another.exponent)
    if not isinstance(self.mantissa, PaillierTensor):
        self_m = another.mantissa.keypair.encrypt(self.mantissa)
        another_m = another.mantissa
    elif not isinstance(another.mantissa, PaillierTensor):
        self_m = self.mantissa
        another_m = self.mantissa.keypair.encrypt(another.mantissa)
    else:
        self_m, another_m = self.mantissa, another.mantissa
    kp = self_m.keypair
    mantissa, exponent = kp.shift_add(self_m.tensor, se, another_m.tensor, ae)
    return FixedPointTensor(PaillierTensor(kp, mantissa), exponent)


def fixedpoint_mul(self, another):
    """FixedPointTensor.__mul__ (paillier.py:135-138): ciphertext ^ plaintext mantissa."""
    from efl.privacy.paillier import FixedPointTensor
    another = _fp_encode(another)
    ex = _efl_lib.as_tensor(self.exponent)
    ey = _efl_lib.as_tensor(another.exponent).to(ex.device)
    return FixedPointTensor(self.mantissa * another.mantissa, ex + ey)


def fixedpoint_matmul(self, another):
    """FixedPointTensor.__matmul__ (paillier.py:140-145) -> PaillierMatmul."""
    from efl.privacy.paillier import FixedPointTensor
    another = _fp_encode(another)
    keypair = self.mantissa.keypair
    mantissa, exponent = keypair.matmul(self.mantissa.tensor, self.exponent, another.mantissa, another.exponent)
    return FixedPointTensor(PaillierTensor(keypair, mantissa), exponent)


@exporter.export("paillier.Hook")
class PaillierHook(object):
    """Key exchange (paillier.py:158-205): the SENDER generates the keypair and sends the public
    key [n, hs] and n_bytes; the RECEIVER installs it (group size 1, as paillier.py:69-70).
    `after_create_session()` runs the exchange; `before_run/after_run` refresh every
    `update_step_interval` steps."""

    def __init__(self, keypair, communicator, role, prefix, update_step_interval=None, n_bytes=None,
                 a_bytes=None, reps=None, group_size=None):
        from efl.privacy.encryptor_utils import Role
        self._kp, self._comm, self._role, self._prefix = keypair, communicator, role, prefix
        self._interval = update_step_interval
        self._local_step = 0
        self._n_bytes = 512 if n_bytes is None else n_bytes
        self._a_bytes = self._n_bytes // 2 if a_bytes is None else a_bytes
        self._reps, self._group = reps, group_size
        if role not in (Role.SENDER, Role.RECEIVER):
            raise ValueError(str(role) + ": No such role.")
        self._sender = role == Role.SENDER

    def _update(self):
        if self._sender:
            public_key, _ = self._kp.generate_keypair(n_bytes=self._n_bytes, a_bytes=self._a_bytes, reps=self._reps,
                                                      group_size=self._group)
            return [self._comm.send(self._prefix + "_public_key", public_key),
                    self._comm.send(self._prefix + "_bytes", torch.tensor([self._n_bytes], dtype=torch.int32))]
        pk = self._comm.recv(self._prefix + "_public_key", shape=(2,), dtype="string")
        nb = self._comm.recv(self._prefix + "_bytes", dtype=torch.int32)
        s = pk.strings()
        self._kp.set_public_key(s[0], nb, s[1], self._a_bytes, group_size=self._group)
        return []

    def after_create_session(self, sess=None, coord=None):
        self._kp.initialize()
        if self._interval is None:
            for h in self._update():
                h.result()

    def before_run(self, run_context=None):
        if self._interval is not None and self._local_step % self._interval == 0:
            self._local_step = 0
            for h in self._update():
                h.result()

    def after_run(self, run_context=None, run_values=None):
        if self._interval is not None:
            self._local_step += 1

    def end(self, sess=None):
        pass
