"""CPU: the key context's host derivation (csrc/keyset.hip via efl_pl_key_derive, no device) gives
every constant the kernels read, checked field by field against a Python-int restatement of the
reference's key setup (paillier.cc:70-101 SetPublicKey / SetPrivateKey: n^2, ceil(2n/3), p^2, q^2,
hp = h(p), hq = h(q), q^-1 mod p, and the h-function of :28-37) plus this build's own constants
(Montgomery radices and -m^-1, radix-2^28 forms, exact-division inverses, the table plan), for
every known-answer key and the CRT sub-keys. Also the refusals the reference's ops make."""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)


@pytest.fixture(scope="module")
def pc():
    import efl  # noqa: F401
    from efl.privacy import paillier_cipher as _pc
    return _pc


def ids(k):
    return f"n{8 * k['n_bytes']}"


def derive(pc, n, hs, a_bytes, g, p=None, q=None, walk=None, window=0, allowance=1 << 62):
    lib = pc._lib
    words = ctypes.c_int64(0)
    d = pc.PlKey()
    hx = (lambda v: format(v, "x").encode() if v is not None else None)
    rc = lib.efl_pl_key_derive(hx(n), hx(hs), a_bytes, g, hx(p), hx(q), hx(walk), window, allowance, None,
                               ctypes.byref(words), ctypes.byref(d))
    pc._efl_lib.check(rc)
    head = np.zeros(words.value, dtype="<u4")
    rc = lib.efl_pl_key_derive(hx(n), hx(hs), a_bytes, g, hx(p), hx(q), hx(walk), window, allowance,
                               head.ctypes.data, ctypes.byref(words), ctypes.byref(d))
    pc._efl_lib.check(rc)
    return head, d


def val(head, off, L, bits=32):
    w = head[off:off + L]
    return sum(int(v) << (bits * t) for t, v in enumerate(w))


def limbs28_total(ln, G):
    return ((32 * ln + 2 + 27) // 28 + G - 1) // G * G


def check_public(pc, head, d, n, hs, a_bits, g, W, walk=None):
    """The public constants (paillier.cc:70-80 plus the n^2 Montgomery constants)."""
    ln = next(c for c in (16, 32, 64, 128, 256) if 32 * c >= n.bit_length())
    lc = 2 * ln
    n2 = n * n
    Rc = 1 << (32 * lc)
    s0 = 1 if walk is None else walk % n2
    assert d.ln == ln and d.a_bits == a_bits and d.group_size == g
    assert val(head, d.off_n, ln) == n
    assert val(head, d.off_n2, lc) == n2
    assert val(head, d.off_n2_r2, lc) == Rc * Rc % n2
    assert val(head, d.off_n2_one, lc) == s0 * Rc % n2
    assert val(head, d.off_max, ln) == -(-(2 * n) // 3)                  # mpz_cdiv_q_ui(2n, 3)
    assert d.n2_minv == (-pow(n2, -1, 1 << 32)) % (1 << 32)
    assert d.table_window == W and d.table_cols == (1 << W) - 1 and d.table_rows == -(-a_bits // W)
    assert d.off_table == -1 and d.off_table28 == -1                   # no table attached yet
    fam = pc.kernel_slicing(ln, False)
    if fam:
        L28 = limbs28_total(2 * ln, 2 * ln // fam)
        assert d.n2_28_len == L28 and (1 << d.table28_log2g) == 2 * ln // fam
        R28 = 1 << (28 * L28)
        assert val(head, d.off_n2_28, L28, 28) == n2
        assert val(head, d.off_n2_one28, L28, 28) == s0 * R28 % n2
        assert val(head, d.off_n2_r2_28, L28, 28) == R28 * R28 % n2
        assert d.n2_minv28 == (-pow(n2, -1, 1 << 28)) % (1 << 28)
        assert all(int(v) < (1 << 28) for v in head[d.off_n2_28:d.off_n2_28 + L28])
    return ln


def check_private(head, d, n, p, q, ln):
    """The private constants (paillier.cc:88-99) and this build's CRT-decryption constants."""
    if q >= 2 * p:
        p, q = q, p
    lh = ln // 2
    Rp, Rh = 1 << (32 * ln), 1 << (32 * lh)
    assert d.has_private == 1
    assert val(head, d.off_p, lh) == p and val(head, d.off_q, lh) == q
    assert val(head, d.off_p2, ln) == p * p and val(head, d.off_q2, ln) == q * q
    assert d.p2_minv == (-pow(p * p, -1, 1 << 32)) % (1 << 32)
    assert d.q2_minv == (-pow(q * q, -1, 1 << 32)) % (1 << 32)
    assert d.p_minv == (-pow(p, -1, 1 << 32)) % (1 << 32) and d.q_minv == (-pow(q, -1, 1 << 32)) % (1 << 32)
    assert val(head, d.off_p2_r3, ln) == pow(Rp, 3, p * p) and val(head, d.off_q2_r3, ln) == pow(Rp, 3, q * q)
    assert val(head, d.off_pm1, lh) == p - 1 and val(head, d.off_qm1, lh) == q - 1
    assert d.pm1_bits == (p - 1).bit_length() and d.qm1_bits == (q - 1).bit_length()
    assert val(head, d.off_pinv_w, lh) == pow(p, -1, Rh) and val(head, d.off_qinv_w, lh) == pow(q, -1, Rh)
    # h-function of paillier.cc:28-37 with g = n + 1, computed here with a real powm
    hp = pow((pow(n + 1, p - 1, p * p) - 1) // p, -1, p)
    hq = pow((pow(n + 1, q - 1, q * q) - 1) // q, -1, q)
    assert val(head, d.off_hp, lh) == hp * Rh % p and val(head, d.off_hq, lh) == hq * Rh % q
    assert val(head, d.off_qinvp, lh) == pow(q, -1, p) * Rh % p
    L28s = [limbs28_total(ln, 1 << k) for k in range(6)]
    Lmax = max(L28s)
    assert d.p2_28_len == Lmax
    assert val(head, d.off_p2_28, Lmax, 28) == p * p and val(head, d.off_q2_28, Lmax, 28) == q * q
    assert d.p2_minv28 == (-pow(p * p, -1, 1 << 28)) % (1 << 28)
    assert d.q2_minv28 == (-pow(q * q, -1, 1 << 28)) % (1 << 28)
    for k, L28 in enumerate(L28s):
        assert val(head, d.off_p2_r2_28[k], Lmax, 28) == pow(2, 2 * 28 * L28, p * p)
        assert val(head, d.off_q2_r2_28[k], Lmax, 28) == pow(2, 2 * 28 * L28, q * q)


@pytest.mark.parametrize("k", KAT["keys"], ids=ids)
@pytest.mark.parametrize("g", [1, 10])
def test_public_constants(pc, k, g):
    n, hs = int(k["n"], 16), int(k["hs"], 16)
    head, d = derive(pc, n, hs, k["a_bits"] // 8, g, window=7)
    check_public(pc, head, d, n, hs, k["a_bits"], g, 7)
    assert d.has_private == 0


@pytest.mark.parametrize("k", KAT["keys"], ids=ids)
def test_private_constants(pc, k):
    n, hs, p, q = (int(k[f], 16) for f in ("n", "hs", "p", "q"))
    for pp, qq in ((p, q), (q, p)):
        head, d = derive(pc, n, hs, k["a_bits"] // 8, 1, pp, qq, window=5)
        ln = check_public(pc, head, d, n, hs, k["a_bits"], 1, 5)
        check_private(head, d, n, pp, qq, ln)


@pytest.mark.parametrize("k", [k for k in KAT["keys"] if k["n_bytes"] >= 128], ids=ids)
def test_crt_sub_key_constants(pc, k):
    """The key owner's sub-keys: (p, hs mod p^2) whose walk starts from R (q^2)^-1 mod p^2, R the
    n^2 Montgomery radix, and likewise for q (efl_pl_crt_join then needs no modular product)."""
    n, hs, p, q = (int(k[f], 16) for f in ("n", "hs", "p", "q"))
    if q >= 2 * p:
        p, q = q, p
    ln = next(c for c in (16, 32, 64, 128, 256) if 32 * c >= n.bit_length())
    R = 1 << (32 * 2 * ln)
    for x, y in ((p, q), (q, p)):
        start = R * pow(y * y, -1, x * x)
        head, d = derive(pc, x, hs % (x * x), k["a_bits"] // 8, 1, walk=start, window=6)
        check_public(pc, head, d, x, hs % (x * x), k["a_bits"], 1, 6, walk=start)


def test_window_against_allowance(pc):
    """The window is the widest whose table (both layouts) fits the allowance; none fits ->
    RESOURCE_EXHAUSTED with the reference's message."""
    from efl import errors
    k = KAT["keys"][1]
    n, hs = int(k["n"], 16), int(k["hs"], 16)
    ln = 32
    fam = pc.kernel_slicing(ln, False)
    eb = 4 * (2 * ln + (limbs28_total(2 * ln, 2 * ln // fam) if fam else 0))
    for budget in (1 << 20, 64 << 20, 1 << 30, 4 << 30):
        _, d = derive(pc, n, hs, k["a_bits"] // 8, 1, allowance=budget)
        W = d.table_window
        assert W == pc.choose_table_window(k["a_bits"], eb, budget)
        assert -(-k["a_bits"] // W) * ((1 << W) - 1) * eb <= budget
        assert W == 24 or -(-k["a_bits"] // (W + 1)) * ((1 << (W + 1)) - 1) * eb > budget
    with pytest.raises(errors.ResourceExhaustedError, match="Memory usage exceeds a predefined threshold"):
        derive(pc, n, hs, k["a_bits"] // 8, 1, allowance=eb * k["a_bits"] - 1)      # W = 1 needs a_bits entries
    assert pc._lib.efl_pl_choose_window(512, eb, eb * 512 - 1) == 0


def test_reference_table_guard(pc):
    """paillier.cc:399-401 / gmp_utils.h:20: the table the reference would build with its group
    size (ceil(a / g) rows x (2^g - 1) entries of |n^2| bits) past 2^40 bits is refused."""
    from efl import errors
    k = KAT["keys"][3]                 # 4096-bit n: n^2 of 8192 bits
    n, hs = int(k["n"], 16), int(k["hs"], 16)
    derive(pc, n, hs, 256, 16, window=4)                    # 128 x 65535 x 8192 bits < 2^40
    with pytest.raises(errors.ResourceExhaustedError, match="Memory usage exceeds a predefined threshold"):
        derive(pc, n, hs, 512, 20, window=4)               # 205 x (2^20 - 1) x 8192 bits > 2^40


def test_refusals(pc):
    from efl import errors
    k = KAT["keys"][1]
    n, hs, p, q = (int(k[f], 16) for f in ("n", "hs", "p", "q"))
    with pytest.raises(errors.InvalidArgumentError, match="distinct"):
        derive(pc, n, hs, 64, 1, p, p)
    with pytest.raises(errors.InvalidArgumentError, match="a_bytes"):
        derive(pc, n, hs, 0, 1)
    with pytest.raises(errors.InvalidArgumentError, match="group_size"):
        derive(pc, n, hs, 64, 21)
    with pytest.raises(errors.InvalidArgumentError, match="table_window"):
        derive(pc, n, hs, 64, 1, window=25)
    with pytest.raises(errors.UnimplementedError, match="128 bits"):
        derive(pc, (1 << 100) + 1, 5, 8, 1)
    with pytest.raises(errors.UnimplementedError, match="at most 8192"):
        derive(pc, (1 << 8200) + 1, 5, 8, 1)
    lib = pc._lib
    w = ctypes.c_int64(0)
    d = pc.PlKey()
    assert lib.efl_pl_key_derive(b"12g4", b"5", 8, 1, None, None, None, 0, 1 << 40, None, ctypes.byref(w),
                                 ctypes.byref(d)) == -3
    assert "hex" in lib.efl_last_error().decode()
    # white space is ignored, as mpz_set_str ignores it; upper case digits are digits
    a = derive(pc, n, hs, 64, 1, window=3)
    hx = format(n, "X")
    spaced = (hx[:10] + " \n" + hx[10:]).encode()
    h2 = np.zeros(a[0].size, dtype="<u4")
    assert lib.efl_pl_key_derive(spaced, format(hs, "x").encode(), 64, 1, None, None, None, 3, 1 << 62,
                                 h2.ctypes.data, ctypes.byref(ctypes.c_int64(h2.size)), ctypes.byref(d)) == 0
    assert np.array_equal(h2, a[0])


def test_ctx_without_device_refuses_cleanly(pc):
    """A context with no key: every op is ABORTED "No public key." (no device touched)."""
    lib = pc._lib
    ctx = ctypes.c_void_p()
    assert lib.efl_pl_ctx_create(ctypes.byref(ctx)) == 0
    try:
        assert lib.efl_pl_ctx_encrypt(ctx, None, None, None, 4, 0, 0, 0, None) == -10
        assert "No public key" in lib.efl_last_error().decode()
        assert lib.efl_pl_ctx_decrypt(ctx, None, None, None, 4, None) == -10
        assert lib.efl_pl_set_private(ctx, b"5", b"7", None) == 0          # ignored without a public key
        info = pc.PlCtxInfo()
        assert lib.efl_pl_ctx_query(ctx, ctypes.byref(info)) == 0 and info.has_public == 0
        assert lib.efl_pl_ctx_options(ctx, -2, 25, -2) == -3
        assert lib.efl_pl_set_public(ctx, b"xyz", 16, b"5", 8, 1, None) == -3   # refused on the host
    finally:
        assert lib.efl_pl_ctx_destroy(ctx) == 0


def test_budget_query_and_set(pc):
    lib = pc._lib
    used = ctypes.c_int64(-1)
    prev = lib.efl_pl_table_budget(-1, ctypes.byref(used))
    assert prev > 0 and used.value == 0
    try:
        assert lib.efl_pl_table_budget(123 << 20, None) == prev
        assert pc.table_budget() == (123 << 20, 0)
    finally:
        lib.efl_pl_table_budget(prev, None)


def test_ctx_info_struct_matches_ctypes_mirror(tmp_path):
    """efl_pl_ctx_info and its ctypes mirror agree on size and every offset (gcc from the header)."""
    import subprocess
    from conftest import ROOT
    import efl  # noqa: F401
    from efl.privacy.paillier_cipher import PlCtxInfo
    names = [f[0] for f in PlCtxInfo._fields_]
    src = tmp_path / "info.c"
    src.write_text("#include <stddef.h>\n#include <stdio.h>\n#include \"efl_hip.h\"\nint main(void) {\n"
                   "  printf(\"%zu\\n\", sizeof(efl_pl_ctx_info));\n"
                   + "".join(f"  printf(\"%zu\\n\", offsetof(efl_pl_ctx_info, {n}));\n" for n in names)
                   + "  return 0;\n}\n")
    exe = tmp_path / "info"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(s) for s in subprocess.check_output([str(exe)]).split()]
    assert got[0] == ctypes.sizeof(PlCtxInfo)
    assert got[1:] == [getattr(PlCtxInfo, n).offset for n in names]
