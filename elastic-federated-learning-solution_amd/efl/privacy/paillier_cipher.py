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
import weakref

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
                ("off_n2_r2_28", ctypes.c_int64), ("table_window", ctypes.c_int32),
                ("off_gn28", ctypes.c_int64), ("off_gstart28", ctypes.c_int64)]


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

# Device memory the fixed-base tables may take (csrc/keyset.hip sizes them; round 3 measured why the
# widest window that fits is the fastest: a fresh-randomness encryption costs ceil(a_bits / W)
# (1 - 2^-W) table products, and lookups past the 256 MB Infinity Cache still pay:
# profiles/r03/table_window_*.jsonl, profiles/r04/table_window_*.jsonl: the 1024-bit key 65.2 -> 76.2
# M encrypts/s from W = 16 to 18 (4.0 GiB), the 4096-bit key 0.99 -> 1.07 M/s from W = 12 to 13).
# Two bounds (round 5): a cap per keypair, TABLE_MAX_BYTES (EFL_PL_TABLE_MAX_MIB), and one
# PROCESS-WIDE budget shared by every live keypair (table_budget(); EFL_PL_TABLE_BUDGET_MIB, default
# 4 GiB): a key's window is the widest whose table fits the smaller of its cap and what the budget has
# left. A public-key holder spends it on its one table; the key owner, whose encryptions go by CRT, on
# the two CRT sub-tables (half each), building its n^2 table from what the budget has left only if
# it is ever walked.
TABLE_MAX_BYTES = 4 << 30
WINDOW_MAX = 24


def table_max_bytes() -> int:
    """The per-keypair table cap: EFL_PL_TABLE_MAX_MIB (MiB) if set, else TABLE_MAX_BYTES."""
    v = os.environ.get("EFL_PL_TABLE_MAX_MIB", "")
    return int(v) << 20 if v else TABLE_MAX_BYTES


def choose_table_window(a_bits: int, entry_bytes: int, max_bytes: int | None = None) -> int:
    """Widest window W <= WINDOW_MAX whose table (ceil(a_bits / W) rows x 2^W - 1 entries of
    entry_bytes: the n^2 words of every layout the key keeps) fits max_bytes (default
    table_max_bytes()); the library's own rule (efl_pl_choose_window), 1 when none fits. With 4 GiB:
    2048-bit a of a 4096-bit n (the reference default) -> W = 13, 512-bit a of a 1024-bit n (the
    examples) -> W = 18."""
    if max_bytes is None:
        max_bytes = table_max_bytes()
    return max(1, _lib.efl_pl_choose_window(int(a_bits), int(entry_bytes), int(max_bytes)))


def _limbs(x: int, L: int) -> np.ndarray:
    return np.frombuffer(int(x).to_bytes(4 * L, "little"), dtype="<u4").copy()


def table_passes(W: int, cols: int):
    """The table build's doubling passes (csrc/keyset.hip build_table): pass k computes the columns
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
    if n_bytes < 16:
        # the device kernels need n of at least 128 bits (KeyBlock refuses smaller keys), and the
        # sieve below discards every prime of 16 bits or fewer: refuse before the prime search
        raise errors.UnimplementedError("n of fewer than 128 bits is not supported on the GPU")
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

class PlCtxInfo(ctypes.Structure):
    """ctypes mirror of efl_pl_ctx_info (include/efl_hip.h)."""
    _fields_ = [(n, ctypes.c_int32) for n in ("has_public", "has_private", "n_bytes", "ln", "a_bits", "group_size",
                                               "table_window", "has_table", "crt_capable", "crt")] + \
               [("crt_table_window", ctypes.c_int32 * 2)] + \
               [(n, ctypes.c_int64) for n in ("block_bytes", "table_bytes", "table_max_bytes")] + \
               [("crt_block_bytes", ctypes.c_int64 * 2), ("crt_table_bytes", ctypes.c_int64 * 2),
                ("generation", ctypes.c_uint64)]


_cp = ctypes.c_char_p
for _name, _args, _res in (
        ("efl_pl_ctx_create", [ctypes.POINTER(_vp)], _i32),
        ("efl_pl_ctx_destroy", [_vp], _i32),
        ("efl_pl_ctx_options", [_vp, _i64, _i32, _i32], _i32),
        ("efl_pl_set_public", [_vp, _cp, _i32, _cp, _i32, _i32, _vp], _i32),
        ("efl_pl_set_private", [_vp, _cp, _cp, _vp], _i32),
        ("efl_pl_set_keypair", [_vp, _cp, _i32, _cp, _i32, _i32, _cp, _cp, _vp], _i32),
        ("efl_pl_ctx_key", [_vp, _i32, ctypes.POINTER(_vp), _PK], _i32),
        ("efl_pl_ctx_prepare", [_vp, _i32, _vp], _i32),
        ("efl_pl_ctx_query", [_vp, ctypes.POINTER(PlCtxInfo)], _i32),
        ("efl_pl_ctx_copy", [_vp, _i32, _i64, _i64, _vp, _vp], _i32),
        ("efl_pl_ctx_encrypt", [_vp, _vp, _vp, _vp, _i64, _u64, _i64, _i32, _vp], _i32),
        ("efl_pl_ctx_fbpowm", [_vp, _vp, _vp, _i64, _u64, _i64, _i32, _vp], _i32),
        ("efl_pl_ctx_decrypt", [_vp, _vp, _vp, _vp, _i64, _vp], _i32),
        ("efl_pl_table_budget", [_i64, ctypes.POINTER(_i64)], _i64),
        ("efl_pl_choose_window", [_i32, _i64, _i64], _i32),
        ("efl_pl_key_derive", [_cp, _cp, _i32, _i32, _cp, _cp, _cp, _i32, _i64, _vp, ctypes.POINTER(_i64), _PK],
         _i32)):
    getattr(_lib, _name).argtypes = _args
    getattr(_lib, _name).restype = _res

PREPARE_TABLE, PREPARE_CRT, PUBLIC_PATH = 1, 2, 1


def _hx(x: int) -> bytes:
    return format(int(x), "x").encode()


def table_budget(nbytes: int | None = None):
    """The process-wide device-memory budget of the fixed-base tables (efl_pl_table_budget):
    returns (budget, bytes in use) after setting it to `nbytes` if given."""
    used = _i64(0)
    prev = _lib.efl_pl_table_budget(-1 if nbytes is None else int(nbytes), ctypes.byref(used))
    cur = prev if nbytes is None else int(nbytes)
    return cur, used.value


class _KeyView:
    """One key block of a context (which 0 = the key, 1 / 2 = the CRT sub-keys): what the efl_pl_*
    ops take, fetched from the library on every use (a key set again moves the block)."""

    def __init__(self, owner: "KeyBlock", which: int, n: int, ln: int):
        # a weak reference: the key's views must not keep it (and its device memory) alive in a cycle
        self._ref, self.which, self.n, self.ln = weakref.ref(owner), which, n, ln
        self.lc, self.lh = 2 * ln, ln // 2
        self.device = owner.device
        self._desc = PlKey()

    def args(self):
        ptr = _vp()
        _efl_lib.check(_lib.efl_pl_ctx_key(self._owner.ctx, self.which, ctypes.byref(ptr), ctypes.byref(self._desc)))
        return ptr.value, ctypes.byref(self._desc)

    @property
    def _owner(self) -> "KeyBlock":
        o = self._ref()
        if o is None or not o.ctx:
            raise errors.AbortedError("the key this view belongs to was released")
        return o

    @property
    def desc(self) -> PlKey:
        self.args()
        return self._desc

    @property
    def table_window(self) -> int:
        return self.desc.table_window

    @property
    def block_bytes(self) -> int:
        i = self._owner.info()
        return i.block_bytes if self.which == 0 else i.crt_block_bytes[self.which - 1]

    def read_words(self, off: int, count: int) -> np.ndarray:
        """count 32-bit words of this key block from word `off` (efl_pl_ctx_copy), as uint32."""
        out = np.empty(count, dtype="<u4")
        with torch.cuda.device(self.device):
            _efl_lib.check(_lib.efl_pl_ctx_copy(self._owner.ctx, self.which, off, count, out.ctypes.data, None))
            torch.cuda.synchronize(self.device)
        return out


class KeyBlock:
    """A Paillier key in device memory: the library's key context (efl_pl_ctx, csrc/keyset.hip),
    which derives every constant the kernels read from the key's hex text, builds the fixed-base
    table on the device, and keeps the key owner's CRT sub-keys. This class is the thin Python
    handle: the reference's PaillierKeypair resource (paillier.cc:50-101) on the host side of the
    C ABI (include/efl_hip.h, "Key context")."""

    def __init__(self, n: int, hs: int, a_bits: int, group_size: int, p=None, q=None, device=None,
                 table_window=None, max_bytes=None, n_bytes=None):
        """Set (n, hs) and, with p and q, the private key, in one call (efl_pl_set_keypair, or
        efl_pl_set_public). max_bytes: the context's table cap (default EFL_PL_TABLE_MAX_MIB or 4
        GiB); the process-wide budget (table_budget) bounds it further. table_window forces the
        window (1..24; results never depend on it)."""
        KeyBlock.check(n, hs, a_bits, group_size, p, q, table_window)     # refusals before the device
        self.device = device or _efl_lib.require_gpu()
        ctx = _vp()
        _efl_lib.check(_lib.efl_pl_ctx_create(ctypes.byref(ctx)))
        self.ctx = ctx.value
        self._views = {}
        self._crt_views = None
        try:
            _efl_lib.check(_lib.efl_pl_ctx_options(self.ctx, -1 if max_bytes is None else int(max_bytes),
                                                   int(table_window or 0), -1))
            self.set(n, hs, a_bits, group_size, p, q, n_bytes)
        except Exception:
            self.close()
            raise

    @staticmethod
    def check(n: int, hs: int, a_bits: int, group_size: int, p=None, q=None, table_window=None):
        """Everything setting this key could refuse on the host (arguments, sizes, the reference's
        table guard), without the device (efl_pl_key_derive); raises the error setting it would."""
        if a_bits % 8:
            raise errors.InvalidArgumentError("a_bits must be a whole number of bytes")
        words = _i64(0)
        d = PlKey()
        priv = p is not None and q is not None
        _efl_lib.check(_lib.efl_pl_key_derive(_hx(n), _hx(hs), int(a_bits) // 8, int(group_size),
                                              _hx(p) if priv else None, _hx(q) if priv else None, None,
                                              int(table_window or 0), 1 << 62, None, ctypes.byref(words),
                                              ctypes.byref(d)))

    def set(self, n: int, hs: int, a_bits: int, group_size: int, p=None, q=None, n_bytes=None):
        """SetPaillierPublicKey (+ SetPaillierPrivateKey) on this context, in place. A refused key
        (bad argument, unsupported size, the table budget) leaves the previous key in place."""
        nb = int(n_bytes) if n_bytes is not None else (int(n).bit_length() + 7) // 8
        with torch.cuda.device(self.device):
            sh = _stream(self.device)
            if p is not None and q is not None:
                rc = _lib.efl_pl_set_keypair(self.ctx, _hx(n), nb, _hx(hs), int(a_bits) // 8, int(group_size),
                                             _hx(p), _hx(q), sh)
            else:
                rc = _lib.efl_pl_set_public(self.ctx, _hx(n), nb, _hx(hs), int(a_bits) // 8, int(group_size), sh)
            _efl_lib.check(rc)
        self._refresh(n, hs, a_bits, group_size, p, q)

    def set_private(self, p: int, q: int):
        """SetPaillierPrivateKey in place (the public part and its table stay)."""
        with torch.cuda.device(self.device):
            _efl_lib.check(_lib.efl_pl_set_private(self.ctx, _hx(p), _hx(q), _stream(self.device)))
        self._refresh(self.n, self.hs, self.a_bits, self.group_size, p, q)

    def _refresh(self, n, hs, a_bits, group_size, p, q):
        self.n, self.hs, self.a_bits, self.group_size = int(n), int(hs), int(a_bits), int(group_size)
        if p is not None and q is not None:
            p, q = int(p), int(q)
            if q >= 2 * p:
                p, q = q, p              # as the key block orders them (the CRT reduces mq mod p once)
        self.p, self.q = p, q
        i = self.info()
        self.ln, self.lc, self.lh = i.ln, 2 * i.ln, i.ln // 2
        self._main = _KeyView(self, 0, self.n, self.ln)

    def close(self):
        ctx, self.ctx = getattr(self, "ctx", None), None
        if ctx:
            _lib.efl_pl_ctx_destroy(ctx)

    def __del__(self):
        try:
            self.close()
        except Exception:       # noqa: BLE001 - interpreter shutdown
            pass

    # -- the key the ops take ------------------------------------------------------------------
    def args(self):
        return self._main.args()

    @property
    def desc(self) -> PlKey:
        return self._main.desc

    def info(self) -> PlCtxInfo:
        i = PlCtxInfo()
        _efl_lib.check(_lib.efl_pl_ctx_query(self.ctx, ctypes.byref(i)))
        return i

    @property
    def table_window(self) -> int:
        return self.info().table_window

    @property
    def has_table(self) -> bool:
        return bool(self.info().has_table)

    @property
    def block_bytes(self) -> int:
        return self.info().block_bytes

    @property
    def table_bytes(self) -> int:
        return self.info().table_bytes

    def read_words(self, off: int, count: int) -> np.ndarray:
        return self._main.read_words(off, count)

    def crt_capable(self) -> bool:
        """Whether the key owner's encryption goes by CRT (crt_keys): the private key factors n
        (p q = n, p != q), half-length primes of a supported limb class, EFL_PL_CRT_ENCRYPT not 0."""
        return bool(self.info().crt_capable)

    def ensure_table(self):
        """Build the n^2 fixed-base table if this key has none yet (the key owner's is deferred:
        its encryptions go by CRT). Returns self."""
        with torch.cuda.device(self.device):
            _efl_lib.check(min(0, _lib.efl_pl_ctx_prepare(self.ctx, PREPARE_TABLE, _stream(self.device))))
        return self

    def crt_keys(self):
        """The key owner's encryption keys ((p, hs mod p^2) and (q, hs mod q^2), walks starting from
        R (q^2)^-1 and R (p^2)^-1) as key views, built on first use; None when this key cannot take
        them (no private key, p q != n, p == q, primes not of a half-length limb class, CRT off, or
        no room in the table budget). The reference's Encrypt works mod n^2 only
        (paillier.cc:103-131); the join gives its ciphertexts bit for bit."""
        with torch.cuda.device(self.device):
            rc = _lib.efl_pl_ctx_prepare(self.ctx, PREPARE_CRT, _stream(self.device))
        _efl_lib.check(min(0, rc))
        if rc != 1:
            return None
        gen = self.info().generation
        if self._crt_views is None or self._crt_views[0] != gen:
            self._crt_views = (gen, (_KeyView(self, 1, self.p, self.lh), _KeyView(self, 2, self.q, self.lh)))
        return self._crt_views[1]


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
        """SetPaillierPrivateKey (ignored without a public key, paillier.cc:88-91): in place, the
        public key and its table stay (efl_pl_set_private)."""
        if self._key is None:
            return
        self._key.set_private(int(_hex_of(p), 16), int(_hex_of(q), 16))

    def set_keys_ints(self, n, hs, a_bytes, group_size=1, p=None, q=None, n_bytes=None, table_window=None):
        """Host-int variant of set_public_key/set_private_key (tests, key exchange). table_window
        forces the fixed-base table's window (default: chosen against the table budget; results
        never change)."""
        self._set(n, n_bytes or (n.bit_length() + 7) // 8, hs, a_bytes, group_size, p, q, table_window)

    def _set(self, n, n_bytes, hs, a_bytes, group_size, p=None, q=None, table_window=None):
        old = self._key
        a_bits = 8 * int(a_bytes)
        if old is not None and p is not None and q is not None and table_window is None \
                and (old.n, old.hs, old.a_bits, old.group_size) == (n, hs, a_bits, int(group_size)):
            old.set_private(p, q)        # the same public key: its table stays
            self._n_bytes = n_bytes
            return
        if old is not None:
            # a re-key: the new key is checked on the host first, so a refused key (bad argument,
            # unsupported size, the reference's table guard) leaves the old one in place; then the
            # old key's device memory is let go of before the new tables are sized against the
            # process-wide budget. Ciphertexts made under the old key keep their limbs; their key
            # handle is closed (every op takes the keypair's current key, as the reference's do).
            KeyBlock.check(n, hs, a_bits, int(group_size), p, q, table_window)
            self._key = None
            old.close()
        self._key = KeyBlock(n, hs, a_bits, int(group_size), p, q, table_window=table_window, n_bytes=n_bytes)
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
    def _path_flags(self) -> int:
        """efl_pl_ctx_encrypt / _fbpowm flags: the key owner's CRT path unless crt_encrypt is off."""
        return 0 if self.crt_encrypt else PUBLIC_PATH

    def encrypt(self, plaintext, hsa=None, counter_base=None):
        """PaillierEncrypt (paillier.cc:443-503). hsa None (or all "0") draws a fresh a per element
        from Philox(seed, counter); counter_base defaults to a running per-keypair counter. The key
        context routes it (efl_pl_ctx_encrypt): the key owner by CRT, a public-key holder through
        the n^2 table, a given hsa straight to the product; the same ciphertexts on every path."""
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
        sh, fl = _stream(k.device), self._path_flags()
        _efl_lib.check(_lib.efl_pl_ctx_encrypt(k.ctx, m.data_ptr(),
                                               hsa_limbs.data_ptr() if hsa_limbs is not None else None,
                                               out.data_ptr(), N, self.seed, ctr, fl, sh))
        if hsa_limbs is not None and zero_idx is not None and zero_idx.size:
            # the rows whose hsa is "0" draw a fresh a at their own index's counter (ctr + idx),
            # inside this call's range: rows with a given hsa consume no counter
            idx = torch.from_numpy(zero_idx).to(k.device)
            sub = torch.empty((idx.numel(), k.lc), dtype=torch.int32, device=k.device)
            msub = m[idx].contiguous()
            for j0, j1, c0 in _counter_runs(zero_idx):
                _efl_lib.check(_lib.efl_pl_ctx_encrypt(k.ctx, msub[j0:j1].data_ptr(), None, sub[j0:j1].data_ptr(),
                                                       j1 - j0, self.seed, ctr + c0, fl, sh))
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
        a_dev = None
        if a is not None:
            a = list(a)
            n = len(a)
            if any(v < 0 or v.bit_length() > k.a_bits for v in a):
                raise errors.InvalidArgumentError("exponent wider than the fixed-base table")
            arr = np.stack([_limbs(v, words) for v in a]) if n else np.zeros((0, words), "<u4")
            a_dev = torch.from_numpy(arr.view(np.int32)).to(k.device)
        out = torch.empty((n, k.lc), dtype=torch.int32, device=k.device)
        _efl_lib.check(_lib.efl_pl_ctx_fbpowm(k.ctx, a_dev.data_ptr() if a_dev is not None else None, out.data_ptr(),
                                              n, self.seed, counter_base, self._path_flags(), _stream(k.device)))
        return CipherTensor(out, (n,), k)

    def decrypt(self, paillier_tensor, dtype="string"):
        """PaillierDecrypt (paillier.cc:505-561): HexTensor of the signed plaintext (default) or
        int64 (mpz_get_sll semantics)."""
        k = self.key
        if k.p is None:
            raise errors.AbortedError("No private key.")
        c = self._cipher(paillier_tensor)
        N = c.numel()
        mag = torch.empty((N, k.ln), dtype=torch.int32, device=k.device)
        neg = torch.empty(N, dtype=torch.int8, device=k.device)
        _efl_lib.check(_lib.efl_pl_ctx_decrypt(k.ctx, c.limbs.data_ptr(), mag.data_ptr(), neg.data_ptr(), N,
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
        product is exact, so the ciphertexts equal efl_pl_matmul's. Blocks of rows i and output
        columns k hold at most about _COMPOSED_CHUNK_BYTES (256 MiB) of terms each (a whole
        column of v terms at least), so peak memory stays a small multiple of that for any shape."""
        k = self.key
        u, v = x.shape
        w = ym.shape[1]
        term_bytes = v * k.lc * 4                       # one output's terms
        wc = max(1, min(w, _COMPOSED_CHUNK_BYTES // term_bytes))
        rows = max(1, min(u, _COMPOSED_CHUNK_BYTES // (term_bytes * wc)))
        z = torch.empty((u, w, k.lc), dtype=torch.int32, device=k.device)
        mins = torch.empty((u, w), dtype=torch.int64, device=k.device)
        for i0 in range(0, u, rows):
            i1 = min(u, i0 + rows)
            r = i1 - i0
            xr = CipherTensor(x.limbs[i0 * v:i1 * v], (r, v, 1), k)
            for k0 in range(0, w, wc):
                k1 = min(w, k0 + wc)
                c = k1 - k0
                yb, yeb = ym[:, k0:k1], ye[:, k0:k1]
                t = self.mul_scalar(xr, yb.reshape(1, v, c))                      # [r, v, c]
                s = xe[i0:i1].reshape(r, v, 1) + yeb.reshape(1, v, c)
                m = s.amin(dim=1)                                                  # [r, c]
                t = self._exp2_chunked(t.limbs, (s - m.reshape(r, 1, c)).reshape(-1).contiguous())
                t = t.view(r, v, c, k.lc)
                while t.shape[1] > 1:                                              # product over j
                    h = t.shape[1] // 2
                    a = t[:, :h].contiguous()
                    b = t[:, h:2 * h].contiguous()
                    p = torch.empty_like(a)
                    _efl_lib.check(_lib.efl_pl_add(*k.args(), a.data_ptr(), b.data_ptr(), p.data_ptr(),
                                                   r * h * c, _stream(k.device)))
                    t = torch.cat([p, t[:, 2 * h:]], dim=1) if t.shape[1] % 2 else p
                z[i0:i1, k0:k1] = t.reshape(r, c, k.lc)
                mins[i0:i1, k0:k1] = m
        return CipherTensor(z.reshape(u * w, k.lc), (u, w), k), mins

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
