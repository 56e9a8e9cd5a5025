"""GPU: Paillier keys set through the raw C ABI only — ctypes on libefl_hip.so, torch for device
buffers, and neither the efl Python package nor the oracle. This is what a TensorFlow C++ shim
binding CreatePaillierKeypair / SetPaillierPublicKey / SetPaillierPrivateKey
(paillier.cc:337-441) does: hex text in, an opaque context out, the key block and its
descriptor fetched from the library. The known answers are GMP 6.2.1's (tests/golden/paillier_kat.json).
Also the process-wide table budget (gmp_utils.h:20 / paillier.cc:399-401's ResourceExhausted)."""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, PKG

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)
KEYS = [k for k in KAT["keys"] if k["n_bytes"] in (128, 512)]        # 1024- and 4096-bit n

vp, i32, i64, u64, cp = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_char_p
DESC_BYTES = 1024                      # room for efl_pl_key: the test treats it as opaque


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = ctypes.CDLL(os.path.join(PKG, "efl", "libefl_hip.so"))
    sig = {
        "efl_pl_ctx_create": [ctypes.POINTER(vp)], "efl_pl_ctx_destroy": [vp],
        "efl_pl_set_public": [vp, cp, i32, cp, i32, i32, vp], "efl_pl_set_private": [vp, cp, cp, vp],
        "efl_pl_ctx_key": [vp, i32, ctypes.POINTER(vp), vp], "efl_pl_ctx_prepare": [vp, i32, vp],
        "efl_pl_ctx_encrypt": [vp, vp, vp, vp, i64, u64, i64, i32, vp],
        "efl_pl_ctx_fbpowm": [vp, vp, vp, i64, u64, i64, i32, vp],
        "efl_pl_ctx_decrypt": [vp, vp, vp, vp, i64, vp],
        "efl_pl_encrypt": [vp, vp, vp, vp, vp, i64, u64, i64, vp],
        "efl_pl_decrypt": [vp, vp, vp, vp, vp, i64, vp],
        "efl_pl_ctx_options": [vp, i64, i32, i32], "efl_pl_ctx_query": [vp, vp],
    }
    for name, args in sig.items():
        getattr(L, name).argtypes = args
        getattr(L, name).restype = i32
    L.efl_pl_table_budget.argtypes = [i64, ctypes.POINTER(i64)]
    L.efl_pl_table_budget.restype = i64
    L.efl_last_error.restype = cp
    return L


def ok(L, rc):
    assert rc == 0, (rc, L.efl_last_error().decode())


def limbs(vals, L):
    a = np.stack([np.frombuffer(int(v).to_bytes(4 * L, "little"), "<u4") for v in vals])
    return torch.from_numpy(a.view(np.int32)).cuda()


def ints(t):
    a = t.cpu().numpy().view("<u4")
    return [int.from_bytes(r.tobytes(), "little") for r in a]


class Ctx:
    def __init__(self, L):
        self.L = L
        h = vp()
        ok(L, L.efl_pl_ctx_create(ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            ok(self.L, self.L.efl_pl_ctx_destroy(self.h))
            self.h = None


def stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("k", KEYS, ids=lambda k: f"n{8 * k['n_bytes']}")
def test_kat_through_the_context(lib, k):
    """set_public (hex) + set_private (hex); encryption with the vectors' hsa, decryption, fixed-base
    exponentiation of the vectors' a: all bit-equal to GMP. The context's key block also drives the
    stateless entry points (efl_pl_encrypt / efl_pl_decrypt) with the same results."""
    ln = k["n_bytes"] // 4
    n_hex, hs_hex = k["n"].encode(), k["hs"].encode()
    for g in sorted({v["g"] for v in k["vectors"]}):
        vs = [v for v in k["vectors"] if v["g"] == g]
        c = Ctx(lib)
        try:
            ok(lib, lib.efl_pl_set_public(c.h, n_hex, k["n_bytes"], hs_hex, k["a_bits"] // 8, g, stream()))
            N = len(vs)
            m = torch.tensor([v["m"] for v in vs], dtype=torch.int64, device="cuda")
            hsa = limbs([int(v["hsa"], 16) for v in vs], 2 * ln)
            ct = torch.empty((N, 2 * ln), dtype=torch.int32, device="cuda")
            ok(lib, lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), hsa.data_ptr(), ct.data_ptr(), N, 0, 0, 0, stream()))
            assert ints(ct) == [int(v["c"], 16) for v in vs]
            # FixedBasePowm of the given exponents through the n^2 table the public key built
            aw = (k["a_bits"] + 31) // 32
            a = limbs([int(v["a"], 16) for v in vs], aw)
            hs_out = torch.empty_like(ct)
            ok(lib, lib.efl_pl_ctx_fbpowm(c.h, a.data_ptr(), hs_out.data_ptr(), N, 0, 0, 0, stream()))
            assert ints(hs_out) == [int(v["hsa"], 16) for v in vs]
            # no private key yet: ABORTED, as the reference's decrypt op
            mag = torch.empty((N, ln), dtype=torch.int32, device="cuda")
            neg = torch.empty(N, dtype=torch.int8, device="cuda")
            assert lib.efl_pl_ctx_decrypt(c.h, ct.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, stream()) == -10
            ok(lib, lib.efl_pl_set_private(c.h, k["p"].encode(), k["q"].encode(), stream()))
            ok(lib, lib.efl_pl_ctx_decrypt(c.h, ct.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, stream()))
            got = [(-x if s else x) for x, s in zip(ints(mag), neg.cpu().tolist())]
            assert got == [v["m"] for v in vs]
            assert [format(abs(x), "x") if x >= 0 else "-" + format(-x, "x") for x in got] == [v["d"] for v in vs]
            # the stateless ops on the context's block and descriptor
            blk, desc = vp(), ctypes.create_string_buffer(DESC_BYTES)
            ok(lib, lib.efl_pl_ctx_key(c.h, 0, ctypes.byref(blk), desc))
            ct2 = torch.empty_like(ct)
            ok(lib, lib.efl_pl_encrypt(blk, desc, m.data_ptr(), hsa.data_ptr(), ct2.data_ptr(), N, 0, 0, stream()))
            assert torch.equal(ct2, ct)
            mag2 = torch.empty_like(mag)
            ok(lib, lib.efl_pl_decrypt(blk, desc, ct.data_ptr(), mag2.data_ptr(), neg.data_ptr(), N, stream()))
            assert torch.equal(mag2, mag)
        finally:
            c.close()


@pytest.mark.parametrize("k", KEYS, ids=lambda k: f"n{8 * k['n_bytes']}")
def test_fresh_randomness_paths_agree(lib, k):
    """The key owner's encryption (set together: CRT sub-keys, n^2 table deferred) and the public
    path (EFL_PL_PUBLIC_PATH: the n^2 table, built on first use) give the same ciphertexts, which
    decrypt to the plaintext."""
    ln = k["n_bytes"] // 4
    c = Ctx(lib)
    try:
        lib.efl_pl_set_keypair.argtypes = [vp, cp, i32, cp, i32, i32, cp, cp, vp]
        ok(lib, lib.efl_pl_set_keypair(c.h, k["n"].encode(), k["n_bytes"], k["hs"].encode(), k["a_bits"] // 8, 1,
                                       k["p"].encode(), k["q"].encode(), stream()))
        N = 300
        m = torch.randint(-2**62, 2**62, (N,), dtype=torch.int64, device="cuda")
        m[:3] = torch.tensor([0, -1, 2**63 - 1])
        a = torch.empty((N, 2 * ln), dtype=torch.int32, device="cuda")
        b = torch.empty_like(a)
        ok(lib, lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), None, a.data_ptr(), N, 99, 1000, 0, stream()))
        assert lib.efl_pl_ctx_prepare(c.h, 2, stream()) == 1                   # CRT sub-keys in use
        ok(lib, lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), None, b.data_ptr(), N, 99, 1000, 1, stream()))
        assert torch.equal(a, b)
        mag = torch.empty((N, ln), dtype=torch.int32, device="cuda")
        neg = torch.empty(N, dtype=torch.int8, device="cuda")
        ok(lib, lib.efl_pl_ctx_decrypt(c.h, a.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, stream()))
        got = [(-x if s else x) for x, s in zip(ints(mag), neg.cpu().tolist())]
        assert got == m.cpu().tolist()
    finally:
        c.close()


def test_process_wide_table_budget(lib):
    """Three live keypairs under one 768 MiB process budget: every table is sized against what the
    budget has left, the bytes in use never pass it, every key still gives the known answers, and
    a key whose smallest table cannot fit is refused with RESOURCE_EXHAUSTED (the old key stays)."""
    k = KEYS[0]                                   # 1024-bit n, 512-bit a
    ln = k["n_bytes"] // 4
    vs = [v for v in k["vectors"] if v["g"] == 1]
    N = len(vs)
    m = torch.tensor([v["m"] for v in vs], dtype=torch.int64, device="cuda")
    hsa = limbs([int(v["hsa"], 16) for v in vs], 2 * ln)
    aw = (k["a_bits"] + 31) // 32
    a = limbs([int(v["a"], 16) for v in vs], aw)
    used0 = i64(0)
    prev = lib.efl_pl_table_budget(-1, ctypes.byref(used0))
    budget = 768 << 20
    ctxs = []
    try:
        assert lib.efl_pl_table_budget(used0.value + budget, None) == prev
        windows = []
        for i in range(3):
            c = Ctx(lib)
            ctxs.append(c)
            ok(lib, lib.efl_pl_ctx_options(c.h, 1 << 40, 0, -2))      # no per-context cap: the budget binds
            ok(lib, lib.efl_pl_set_public(c.h, k["n"].encode(), k["n_bytes"], k["hs"].encode(), k["a_bits"] // 8, 1,
                                          stream()))
            used = i64(0)
            lib.efl_pl_table_budget(-1, ctypes.byref(used))
            assert used.value - used0.value <= budget
            info = (ctypes.c_char * 256)()
            ok(lib, lib.efl_pl_ctx_query(c.h, info))
            windows.append(int.from_bytes(bytes(info[24:28]), "little", signed=True))   # table_window
        assert windows[0] > windows[1] > windows[2] >= 1, windows    # each fits what the others left
        for c in ctxs:
            ct = torch.empty((N, 2 * ln), dtype=torch.int32, device="cuda")
            ok(lib, lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), hsa.data_ptr(), ct.data_ptr(), N, 0, 0, 0, stream()))
            assert ints(ct) == [int(v["c"], 16) for v in vs]
            ok(lib, lib.efl_pl_ctx_fbpowm(c.h, a.data_ptr(), ct.data_ptr(), N, 0, 0, 0, stream()))
            assert ints(ct) == [int(v["hsa"], 16) for v in vs]
        # the budget now full: a fourth key's W = 1 table (512 entries x 552 B) still fits or not
        lib.efl_pl_table_budget(-1, ctypes.byref(used0))
        lib.efl_pl_table_budget(used0.value + 1000, None)          # 1000 bytes left: nothing fits
        c = Ctx(lib)
        ctxs.append(c)
        rc = lib.efl_pl_set_public(c.h, k["n"].encode(), k["n_bytes"], k["hs"].encode(), k["a_bits"] // 8, 1,
                                   stream())
        assert rc == -8 and b"Memory usage exceeds a predefined threshold" in lib.efl_last_error()
        # re-keying a live context within the budget releases its old table first, and a refused
        # re-key keeps the old key working
        rc = lib.efl_pl_set_public(ctxs[0].h, b"zz", 128, b"5", 64, 1, stream())
        assert rc == -3
        ct = torch.empty((N, 2 * ln), dtype=torch.int32, device="cuda")
        ok(lib, lib.efl_pl_ctx_fbpowm(ctxs[0].h, a.data_ptr(), ct.data_ptr(), N, 0, 0, 0, stream()))
        assert ints(ct) == [int(v["hsa"], 16) for v in vs]
    finally:
        for c in ctxs:
            c.close()
        lib.efl_pl_table_budget(prev, None)


def _info(lib, c):
    info = (ctypes.c_char * 256)()
    ok(lib, lib.efl_pl_ctx_query(c.h, info))
    b = bytes(info)

    def i32_at(o):
        return int.from_bytes(b[o:o + 4], "little", signed=True)

    def i64_at(o):
        return int.from_bytes(b[o:o + 8], "little", signed=True)
    return {"table_window": i32_at(24), "has_table": i32_at(28), "crt": i32_at(36),
            "crt_table_window": [i32_at(40), i32_at(44)], "table_bytes": i64_at(56), "generation": i64_at(104)}


def test_failed_table_build_leaves_a_live_key(lib, monkeypatch):
    """a deferred n^2 table build that fails after the block was re-uploaded must
    not leave the context with a freed key block. With the build forced to fail
    (EFL_PL_FAIL_TABLE_BUILD=1), the public-path encryption returns RESOURCE_EXHAUSTED; then
    decryption, the CRT encryption and, once the build succeeds, the public path all give the right
    answers. The stateless ops refuse a null key block instead of faulting."""
    k = KEYS[0]
    ln = k["n_bytes"] // 4
    c = Ctx(lib)
    try:
        lib.efl_pl_set_keypair.argtypes = [vp, cp, i32, cp, i32, i32, cp, cp, vp]
        ok(lib, lib.efl_pl_set_keypair(c.h, k["n"].encode(), k["n_bytes"], k["hs"].encode(), k["a_bits"] // 8, 1,
                                       k["p"].encode(), k["q"].encode(), stream()))
        assert _info(lib, c)["has_table"] == 0                     # the owner's n^2 table is deferred
        N = 64
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device="cuda")
        ct = torch.empty((N, 2 * ln), dtype=torch.int32, device="cuda")
        monkeypatch.setenv("EFL_PL_FAIL_TABLE_BUILD", "1")
        rc = lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), None, ct.data_ptr(), N, 5, 0, 1, stream())
        assert rc == -8 and b"fault injection" in lib.efl_last_error()
        assert lib.efl_pl_ctx_prepare(c.h, 1, stream()) == -8
        assert _info(lib, c)["has_table"] == 0
        mag = torch.empty((N, ln), dtype=torch.int32, device="cuda")
        neg = torch.empty(N, dtype=torch.int8, device="cuda")
        # the CRT sub-tables' build fails too (the injection covers every table build): the owner's
        # route reports it, and the key block stays live for decryption
        rc = lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), None, ct.data_ptr(), N, 5, 0, 0, stream())
        assert rc == -8
        hsa = torch.zeros((N, 2 * ln), dtype=torch.int32, device="cuda")
        hsa[:, 0] = 1                                              # hsa = 1: the ciphertext is g(m)
        ok(lib, lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), hsa.data_ptr(), ct.data_ptr(), N, 5, 0, 0, stream()))
        ok(lib, lib.efl_pl_ctx_decrypt(c.h, ct.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, stream()))
        assert [(-x if s else x) for x, s in zip(ints(mag), neg.cpu().tolist())] == m.cpu().tolist()
        monkeypatch.delenv("EFL_PL_FAIL_TABLE_BUILD")
        # the CRT route once the builds succeed, and its ciphertexts decrypt
        ok(lib, lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), None, ct.data_ptr(), N, 5, 0, 0, stream()))
        ok(lib, lib.efl_pl_ctx_decrypt(c.h, ct.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, stream()))
        assert [(-x if s else x) for x, s in zip(ints(mag), neg.cpu().tolist())] == m.cpu().tolist()
        ct2 = torch.empty_like(ct)
        ok(lib, lib.efl_pl_ctx_encrypt(c.h, m.data_ptr(), None, ct2.data_ptr(), N, 5, 0, 1, stream()))
        assert torch.equal(ct2, ct) and _info(lib, c)["has_table"] == 1
        # a null key block is refused by every stateless entry point
        blk, desc = vp(), ctypes.create_string_buffer(DESC_BYTES)
        ok(lib, lib.efl_pl_ctx_key(c.h, 0, ctypes.byref(blk), desc))
        assert lib.efl_pl_decrypt(None, desc, ct.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, stream()) == -3
        assert b"null key block" in lib.efl_last_error()
        assert lib.efl_pl_encrypt(None, desc, m.data_ptr(), None, ct.data_ptr(), N, 0, 0, stream()) == -3
    finally:
        c.close()


def test_public_then_private_gives_crt_the_whole_budget(lib):
    """the reference's usual order (SetPaillierPublicKey, then SetPaillierPrivateKey). The
    public step builds the n^2 table; when keeping it would narrow the CRT sub-tables' window (a
    binding process budget), the owner's first encryption releases it and the sub-tables get the
    windows efl_pl_set_keypair gives them; with room for both (a budget that does not bind) the
    table stays. Either way the ciphertexts are the public path's."""
    k = KEYS[0]
    ln = k["n_bytes"] // 4
    used0 = i64(0)
    prev = lib.efl_pl_table_budget(-1, ctypes.byref(used0))
    N = 128
    m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device="cuda")
    lib.efl_pl_set_keypair.argtypes = [vp, cp, i32, cp, i32, i32, cp, cp, vp]
    try:
        for budget, released in ((2 << 30, True), (64 << 30, False)):
            lib.efl_pl_table_budget(used0.value + budget, None)
            a, b = Ctx(lib), Ctx(lib)
            try:
                ok(lib, lib.efl_pl_set_keypair(a.h, k["n"].encode(), k["n_bytes"], k["hs"].encode(), k["a_bits"] // 8,
                                               1, k["p"].encode(), k["q"].encode(), stream()))
                assert lib.efl_pl_ctx_prepare(a.h, 2, stream()) == 1
                want = _info(lib, a)["crt_table_window"]
                a.close()
                ok(lib, lib.efl_pl_set_public(b.h, k["n"].encode(), k["n_bytes"], k["hs"].encode(), k["a_bits"] // 8,
                                              1, stream()))
                assert _info(lib, b)["has_table"] == 1
                ok(lib, lib.efl_pl_set_private(b.h, k["p"].encode(), k["q"].encode(), stream()))
                c1 = torch.empty((N, 2 * ln), dtype=torch.int32, device="cuda")
                c2 = torch.empty_like(c1)
                ok(lib, lib.efl_pl_ctx_encrypt(b.h, m.data_ptr(), None, c1.data_ptr(), N, 9, 3, 0, stream()))
                inf = _info(lib, b)
                assert inf["crt"] == 1 and inf["has_table"] == (0 if released else 1), (budget, inf)
                if released:
                    assert inf["table_bytes"] == 0 and inf["crt_table_window"] == want, (inf, want)
                ok(lib, lib.efl_pl_ctx_encrypt(b.h, m.data_ptr(), None, c2.data_ptr(), N, 9, 3, 1, stream()))
                assert torch.equal(c1, c2)
            finally:
                a.close()
                b.close()
    finally:
        lib.efl_pl_table_budget(prev, None)
