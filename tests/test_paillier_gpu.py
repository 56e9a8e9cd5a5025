"""GPU parity of Stage P (libefl_hip.so csrc/paillier.hip, csrc/paillier_sliced.hip) against
GMP-made known answers and the Python-int oracle. Bar: bit-exact ciphertext hex given hsa; exact
decryption; exact fbpowm. Every kernel family (one lane per element, sliced over 16- or 32-limb
lanes) is run on every key size it is compiled for."""
import contextlib
import json
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import paillier as P
from oracle import philox

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)
ENC_KEYS = [k for k in KAT["keys"] if k["n_bytes"] <= 128]
ALL = KAT["keys"]
# kernel families per ln (mirrors paillier_cipher.SLICINGS): (n^2 ops, decryption)
SLICINGS = {16: ([0, 8, 16, 32], [0, 8]), 32: ([0, 8, 16, 32], [0, 8, 16, 32]), 64: ([0, 8, 16, 32], [0, 8, 16, 32]),
            128: ([8, 16, 32], [0, 8, 16, 32]), 256: ([32], [8, 16, 32])}


def fams(keys, decrypt=False):
    return [pytest.param(k, c, id=f"n{8 * k['n_bytes']}-C{c}")
            for k in keys for c in SLICINGS[k["n_bytes"] // 4][1 if decrypt else 0]]


@contextlib.contextmanager
def family(ln, decrypt, c):
    from efl.privacy import paillier_cipher as pc
    prev = pc.set_kernel_slicing(ln, decrypt, c)
    try:
        yield
    finally:
        pc.set_kernel_slicing(ln, decrypt, prev)


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


def keypair(efl, k, private=True, g=1, seed=1234):
    kp = efl.paillier.Keypair(seed=seed)
    kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, g,
                     int(k["p"], 16) if private else None, int(k["q"], 16) if private else None)
    return kp


def ids(k):
    return f"n{8 * k['n_bytes']}"


@pytest.mark.parametrize("k,c", fams(ALL))
def test_encrypt_given_hsa_kat(efl, k, c):
    kp = keypair(efl, k)
    vs = k["vectors"]
    m = torch.tensor([v["m"] for v in vs], dtype=torch.int64, device="cuda")
    with family(k["n_bytes"] // 4, False, c):
        ct = kp.encrypt(m, hsa=[v["hsa"] for v in vs])
    assert ct.tensor.to_hex().strings() == [v["c"] for v in vs]


@pytest.mark.parametrize("k,c", fams(ALL, decrypt=True))
def test_decrypt_kat(efl, k, c):
    kp = keypair(efl, k)
    vs = k["vectors"]
    hx = efl.HexTensor.from_strings([v["c"] for v in vs])
    with family(k["n_bytes"] // 4, True, c):
        assert kp.decrypt(hx).strings() == [v["d"] for v in vs]
        got = kp.decrypt(hx, dtype=torch.int64).cpu().tolist()
    assert got == [v["m"] for v in vs]


@pytest.mark.parametrize("k,c", [p for p in fams(ALL, decrypt=True) if p.values[1]])
def test_decrypt_kat_binary_method(efl, k, c):
    """The sliced decryption's two exponentiation methods (efl_pl_tune(ln, 2, .)): sliding 5-bit
    windows over per-element odd powers (default) and binary square-and-multiply agree with GMP."""
    lib = efl.lib.raw()
    ln = k["n_bytes"] // 4
    kp = keypair(efl, k)
    vs = k["vectors"]
    hx = efl.HexTensor.from_strings([v["c"] for v in vs])
    assert lib.efl_pl_tune(ln, 2, -1) == 1
    prev = lib.efl_pl_tune(ln, 2, 0)
    try:
        with family(ln, True, c):
            got = kp.decrypt(hx, dtype=torch.int64).cpu().tolist()
    finally:
        lib.efl_pl_tune(ln, 2, prev)
    assert got == [v["m"] for v in vs]


@pytest.mark.parametrize("k,c", fams(ALL))
def test_fbpowm_kat(efl, k, c):
    for g in sorted({v["g"] for v in k["vectors"]}):
        kp = keypair(efl, k, g=g)
        vs = [v for v in k["vectors"] if v["g"] == g]
        with family(k["n_bytes"] // 4, False, c):
            out = kp.fbpowm(a=[int(v["a"], 16) for v in vs])
        assert out.to_hex().strings() == [v["hsa"] for v in vs]


@pytest.mark.parametrize("W", [1, 3, 7, 12])
@pytest.mark.parametrize("k,c", fams(ENC_KEYS))
def test_fbpowm_kat_any_table_window(efl, k, c, W):
    """The table's own window W is a build choice: the kernels reverse a's API-group bits
    (a -> a', as mpz_fbpowm's lookup does) and walk a' in W-bit windows. Every (g, W) pair gives
    the reference's hs^(a') bit for bit, and so does fresh-randomness encryption."""
    for g in sorted({v["g"] for v in k["vectors"]}):
        kp = efl.paillier.Keypair(seed=77)
        kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, g, table_window=W)
        assert kp.key.desc.table_window == W and kp.key.desc.table_cols == (1 << W) - 1
        vs = [v for v in k["vectors"] if v["g"] == g]
        with family(k["n_bytes"] // 4, False, c):
            out = kp.fbpowm(a=[int(v["a"], 16) for v in vs])
            ct = kp.encrypt(torch.tensor([3, -5]), counter_base=40)
        assert out.to_hex().strings() == [v["hsa"] for v in vs]
        okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, g)
        want = [P.hx(P.encrypt(okp, m, P.fbpowm(okp.hs, okp.n2, philox.draw_a(77, 40 + i, k["a_bits"]), g)))
                for i, m in enumerate([3, -5])]
        assert ct.tensor.to_hex().strings() == want


def _host_table(hs, n2, W, rows, cols, R):
    """[rows][cols] of hs^(j 2^(W i)) R mod n^2 with Python ints."""
    out = []
    for i in range(rows):
        b = pow(hs, 1 << (W * i), n2)
        x, row = 1, []
        for _ in range(cols):
            x = x * b % n2
            row.append(x * R % n2)
        out.append(row)
    return out


def _as_ints(words, width, bits):
    w = np.asarray(words, dtype=np.uint32).reshape(-1, width)
    return [sum(int(v) << (bits * t) for t, v in enumerate(r)) for r in w]


@pytest.mark.parametrize("W", [1, 2, 5, 7])
def test_table_built_on_gpu_matches_host(efl, W, monkeypatch):
    """The fixed-base table the key context builds on the GPU (csrc/keyset.hip: every hs^(2^t) on
    the host, then column 1 = b R and W passes of one efl_pl_add product per entry, then x R28 by one
    more) equals hs^(j 2^(W i)) R mod n^2 computed with Python ints, every entry of both layouts; and
    so does a build whose launches take 8 entries each (EFL_PL_TABLE_CHUNK_BYTES)."""
    from efl.privacy import paillier_cipher as pc
    k = ENC_KEYS[1]
    n, hs = int(k["n"], 16), int(k["hs"], 16)
    n2 = n * n
    for chunk in (None, 8 * 4 * 64):
        if chunk:
            monkeypatch.setenv("EFL_PL_TABLE_CHUNK_BYTES", str(chunk))
        kb = pc.KeyBlock(n, hs, k["a_bits"], 1, table_window=W)
        d = kb.desc
        rows, cols, lc = d.table_rows, d.table_cols, kb.lc
        assert lc == 64
        want = [v for row in _host_table(hs, n2, W, rows, cols, 1 << (32 * lc)) for v in row]
        assert _as_ints(kb.read_words(d.off_table, rows * cols * lc), lc, 32) == want
        L28 = d.n2_28_len if d.off_table28 >= 0 else 0
        assert L28
        inv = pow(1 << (32 * lc), -1, n2) * (1 << (28 * L28))
        want28 = [v * inv % n2 for v in want]
        assert _as_ints(kb.read_words(d.off_table28, rows * cols * L28), L28, 28) == want28
        assert kb.table_bytes == rows * cols * (lc + L28) * 4
        kb.close()


@pytest.mark.parametrize("k", ALL, ids=ids)
def test_default_table_window_keeps_the_radix28_table(efl, k, monkeypatch):
    """The default window (the widest whose table, both layouts, fits the 4 GiB cap) keeps the
    radix-2^28 copy the n^2 kernels walk (profiles/r04/table_window_*)."""
    from efl.privacy import paillier_cipher as pc
    monkeypatch.delenv("EFL_PL_TABLE_MAX_MIB", raising=False)     # the production cap
    n, hs = int(k["n"], 16), int(k["hs"], 16)
    budget, used = pc.table_budget()
    assert budget - used >= pc.TABLE_MAX_BYTES                    # the session's budget leaves the cap binding
    kb = pc.KeyBlock(n, hs, k["a_bits"], 1)
    assert kb.has_table
    want = {512: 20, 1024: 18, 2048: 15, 4096: 13}[8 * k["n_bytes"]]
    assert kb.table_window == want
    if pc.kernel_slicing(kb.ln, False):
        assert kb.desc.off_table28 >= 0
    assert kb.table_bytes <= pc.table_max_bytes()
    assert kb.block_bytes <= pc.table_max_bytes() + (1 << 20)   # the table plus the key's constants
    kb.close()


@pytest.mark.parametrize("k,c", fams(ALL))
def test_homomorphic_ops_kat(efl, k, c):
    kp = keypair(efl, k)
    c0 = efl.HexTensor.from_strings([k["vectors"][5]["c"]])
    c1 = efl.HexTensor.from_strings([k["vectors"][6]["c"]])
    with family(k["n_bytes"] // 4, False, c):
        assert kp.add(c0, c1).to_hex().strings() == [k["ops"]["add"]]
        assert kp.mul_scalar(c0, 7).to_hex().strings() == [k["ops"]["mul_scalar_7"]]
        assert kp.mul_exp2(c1, 5).to_hex().strings() == [k["ops"]["mul_exp2_5"]]
        # every GMP-made op vector (oracle/paillier_gmp.c, paillier.cc:157-285, :722-733): both
        # scalar signs (negative: the route through x^-1, :201-211), int64's extremes, the string
        # overload's signed hex text, shifts 0 and 77, and the inverse
        o = k["ops"]
        for name, y in (("mul_scalar_0", 0), ("mul_scalar_neg", -123456789), ("mul_scalar_i64max", 2**63 - 1),
                        ("mul_scalar_i64min", -2**63)):
            assert kp.mul_scalar(c0, torch.tensor([y], dtype=torch.int64)).to_hex().strings() == [o[name]], name
        assert kp.mul_scalar(c0, o["mul_scalar_hex_text"]).to_hex().strings() == [o["mul_scalar_hex"]]
        for e in (0, 77):
            assert kp.mul_exp2(c1, e).to_hex().strings() == [o[f"mul_exp2_{e}"]]
        assert kp.invert(c0).to_hex().strings() == [o["invert"]]


@pytest.mark.parametrize("k,c", fams(ALL))
def test_matmul_gmp_kat(efl, k, c):
    """PaillierMatmul against GMP's PaillierMatmulOp::Compute (paillier.cc:987-1035) on the KAT
    ciphertexts: mixed-sign y with a zero and -(2^63 - 1), per-output minimum exponents."""
    kp = keypair(efl, k)
    mm = k["matmul"]
    u, v, w = mm["shape"]
    xct = efl.HexTensor.from_strings([k["vectors"][i]["c"] for i in mm["x_vectors"]], shape=(u, v))
    xe = torch.tensor(mm["xe"], dtype=torch.int64)
    ym = torch.tensor(mm["ym"], dtype=torch.int64)
    ye = torch.tensor(mm["ye"], dtype=torch.int64)
    with family(k["n_bytes"] // 4, False, c):
        zm, ze = kp.matmul(xct, xe, ym, ye)
    assert zm.to_hex().strings() == [h for row in mm["zm"] for h in row]
    assert ze.cpu().tolist() == mm["ze"]


@pytest.mark.parametrize("c", [16, 32])
def test_round_trip_4096_fresh_randomness(efl, c):
    """The reference's default key size (n of 4096 bits): fresh-randomness encryption through the
    fixed-base table (sliced kernels) and CRT decryption, across many elements and both signs;
    the ciphertexts equal the oracle's for the same Philox draws."""
    k = ALL[3]
    kp = keypair(efl, k, seed=99)
    rng = np.random.default_rng(c)
    m = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, 300, dtype=np.int64))
    m[:3] = torch.tensor([0, -1, 2**63 - 1])
    with family(128, False, c), family(128, True, c):
        ct = kp.encrypt(m, counter_base=5)
        assert torch.equal(kp.decrypt(ct, dtype=torch.int64).cpu(), m)
    okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))
    got = ct.tensor.to_hex().strings()
    for i in (0, 1, 2, 77, 299):
        a = philox.draw_a(99, 5 + i, k["a_bits"])
        assert got[i] == P.hx(P.encrypt(okp, int(m[i]), P.fbpowm(okp.hs, okp.n2, a, 1))), i


@pytest.mark.parametrize("c", [0, 16])
@pytest.mark.parametrize("g", [1, 3])
def test_encrypt_random_a_is_philox_stream(efl, g, c):
    """hsa == 0 path: a = Philox(seed, counter_base + i); c == oracle encrypt with hs^(a')."""
    k = ENC_KEYS[0]
    kp = keypair(efl, k, g=g, seed=0xC0FFEE)
    okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, g, int(k["p"], 16), int(k["q"], 16))
    rng = random.Random(g)
    ms = [rng.randrange(-2**63, 2**63) for _ in range(70)]
    with family(16, False, c):
        ct = kp.encrypt(torch.tensor(ms), counter_base=1000)
    got = ct.tensor.to_hex().strings()
    for i, m in enumerate(ms):
        a = philox.draw_a(0xC0FFEE, 1000 + i, k["a_bits"])
        want = P.encrypt(okp, m, P.fbpowm(okp.hs, okp.n2, a, g))
        assert got[i] == P.hx(want), i
    assert kp.decrypt(ct, dtype=torch.int64).cpu().tolist() == ms


def test_round_trip_and_counter_advance(efl):
    k = ENC_KEYS[1]
    kp = keypair(efl, k)
    m = torch.randint(-2**62, 2**62, (33, 7), dtype=torch.int64)
    a = kp.encrypt(m)
    b = kp.encrypt(m)                        # fresh randomness: different ciphertexts
    assert kp.counter == 2 * m.numel()
    assert a.tensor.to_hex().strings() != b.tensor.to_hex().strings()
    assert torch.equal(kp.decrypt(a, dtype=torch.int64).cpu(), m)
    assert torch.equal(kp.decrypt(b, dtype="int64").cpu(), m)
    d = kp.decrypt(a)                        # default: hex strings
    assert d.shape == (33, 7) and [int(s, 16) for s in d.strings()] == m.reshape(-1).tolist()


def test_mixed_hsa_never_reuses_a(efl):
    """encrypt with some hsa given and some "0", then default encrypts and a Philox
    fbpowm: every freshly drawn hs^a is distinct (m = 0 makes the ciphertext equal hs^a), and the
    zero-hsa rows draw the counter of their own index."""
    k = ENC_KEYS[0]
    kp = keypair(efl, k, seed=4321)
    N = 40
    zero_rows = [0, 1, 2, 7, 20, 21, 39]
    given = kp.fbpowm(a=[12345 + i for i in range(N)]).to_hex().strings()
    hsa = ["0" if i in zero_rows else given[i] for i in range(N)]
    c1 = kp.encrypt(torch.zeros(N, dtype=torch.int64), hsa=hsa).tensor.to_hex().strings()
    for i in range(N):
        if i not in zero_rows:
            assert c1[i] == given[i]
    okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1)
    for i in zero_rows:   # row i of the call took counter 0 + i
        assert c1[i] == P.hx(P.fbpowm(okp.hs, okp.n2, philox.draw_a(kp.seed, i, k["a_bits"]), 1))
    c2 = kp.encrypt(torch.zeros(N, dtype=torch.int64)).tensor.to_hex().strings()
    c3 = kp.fbpowm(n=N).to_hex().strings()
    fresh = [c1[i] for i in zero_rows] + c2 + c3
    assert len(set(fresh)) == len(fresh)
    assert kp.counter == 3 * N


def test_errors(efl):
    k = ENC_KEYS[0]
    pub = keypair(efl, k, private=False)
    ct = pub.encrypt(torch.tensor([1, 2, 3]))
    with pytest.raises(efl.errors.AbortedError, match="No private key"):
        pub.decrypt(ct)
    with pytest.raises(efl.errors.AbortedError, match="No public key"):
        efl.paillier.Keypair().encrypt(torch.tensor([1]))
    with pytest.raises(efl.errors.InvalidArgumentError, match="same size"):
        pub.encrypt(torch.tensor([1, 2]), hsa=["1"])
    with pytest.raises(efl.errors.InvalidArgumentError, match="hex"):
        pub.add(efl.HexTensor.from_strings(["12", "zz"]), efl.HexTensor.from_strings(["1", "1"]))
    with pytest.raises(efl.errors.InvalidArgumentError, match="positive"):
        pub.mul_exp2(ct, torch.tensor([1, -1, 2]))


def test_fixed_point_encrypt_decrypt_like_reference_test(efl):
    """efls-train/test/paillier_test.py:20-31 (encode -> encrypt -> decrypt -> decode), 1024-bit."""
    kp = efl.paillier.Keypair()
    kp.generate_keypair(n_bytes=128)
    a = torch.randn(100, 100, generator=torch.Generator().manual_seed(0)).cuda()
    b = efl.paillier.fixedpoint.encode(a)
    b.mantissa = kp.encrypt(b.mantissa)
    b.mantissa = b.mantissa.decrypt()
    y = efl.paillier.fixedpoint.decode(b)
    assert torch.equal(y[a != 0], a[a != 0])           # exact, stronger than the reference allclose


def test_fixed_point_add_like_reference_test(efl):
    """paillier_test.py:33-47: encrypted a + plaintext b (mul_exp2 alignment + PaillierAdd)."""
    kp = efl.paillier.Keypair()
    kp.generate_keypair(n_bytes=128)
    g = torch.Generator().manual_seed(1)
    a = torch.randn(40, 30, generator=g).cuda()
    b = torch.randn(40, 30, generator=g).cuda()
    fa = efl.paillier.fixedpoint.encode(a)
    fa.mantissa = kp.encrypt(fa.mantissa)
    c2 = fa + b
    c2.mantissa = c2.mantissa.decrypt()
    c2 = efl.paillier.fixedpoint.decode(c2)
    c1 = (a.double() + b.double()).float()
    assert torch.allclose(c1, c2)
    # bit-exact: the exact integer sum (mantissas aligned like paillier.py:119-132) through the
    # GMP-pinned hex decode of the oracle
    from oracle import fxp
    Ma, Ea = fxp.encode(a.cpu().numpy())
    Mb, Eb = fxp.encode(b.cpu().numpy())
    E = np.minimum(Ea, Eb).reshape(-1)
    sums = [int(ma) * 2 ** int(ea - e) + int(mb) * 2 ** int(eb - e)
            for ma, ea, mb, eb, e in zip(Ma.reshape(-1), Ea.reshape(-1), Mb.reshape(-1), Eb.reshape(-1), E)]
    want = fxp.decode_hex([P.hx(v) for v in sums], E)
    assert np.array_equal(c2.cpu().numpy().reshape(-1).view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("c", [0, 16, 32])
def test_invert_and_negative_scalars(efl, c):
    k = ENC_KEYS[1]
    kp = keypair(efl, k)
    with family(32, False, c):
        _invert_and_negative_scalars(efl, k, kp)


@pytest.mark.parametrize("k", ALL, ids=ids)
@pytest.mark.parametrize("n", [1, 100, 5000, 40000])
def test_decrypt_default_family_sized_per_launch(efl, k, n):
    """With the default family, small decryptions take more lanes per element (decrypt_family);
    results stay exact at every size."""
    from efl.privacy import paillier_cipher as pc
    ln = k["n_bytes"] // 4
    prev = pc.reset_kernel_slicing(ln, True)
    try:
        kp = keypair(efl, k)
        gen = torch.Generator(device="cuda").manual_seed(n)
        m = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda", generator=gen)
        got = kp.decrypt(kp.encrypt(m), dtype=torch.int64)
        assert torch.equal(got, m)
    finally:
        pc.set_kernel_slicing(ln, True, prev)


@pytest.mark.parametrize("k", ALL, ids=ids)
def test_invert_random_and_edges(efl, k):
    """Batched binary GCD (k_invert) against exact Python inverses mod n^2 for every key size: 512
    random units, 1, n^2 - 1, 2, small and top-heavy values; non-units (a multiple of p, 0) give
    the 'no inverse' error."""
    kp = keypair(efl, k, private=False)
    n = int(k["n"], 16)
    n2 = n * n
    rng = random.Random(k["n_bytes"])
    xs = [rng.randrange(1, n2) for _ in range(512)]
    xs += [1, n2 - 1, 2, 3, (1 << 64) + 1, n2 - 2, n2 >> 1, (n2 >> 1) + 1]
    want = []
    for x in xs:
        try:
            want.append(pow(x, -1, n2))
        except ValueError:
            want.append(None)
    units = [x for x, w in zip(xs, want) if w is not None]
    got = kp.invert(efl.HexTensor.from_ints(units)).to_hex().to_ints()
    assert got == [w for w in want if w is not None]
    p = int(k["p"], 16)
    with pytest.raises(efl.errors.InvalidArgumentError, match="no inverse"):
        kp.invert(efl.HexTensor.from_ints([units[0], p * 12345, 0]))


def _invert_and_negative_scalars(efl, k, kp):
    okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))
    cs = [int(v["c"], 16) for v in k["vectors"][:12]]
    hx = efl.HexTensor.from_ints(cs)
    assert kp.invert(hx).to_hex().to_ints() == [P.invert(okp, c) for c in cs]
    ys = [3, -1, 0, -7, 2**40 + 1, -(2**62), 5, -2, 1, -1, 9, -2**63]
    got = kp.mul_scalar(hx, torch.tensor(ys)).to_hex().to_ints()
    assert got == [P.mul_scalar(okp, c, y) for c, y in zip(cs, ys)]
    with pytest.raises(efl.errors.InvalidArgumentError, match="no inverse"):
        kp.invert(efl.HexTensor.from_ints([okp.n]))         # gcd(n, n^2) != 1


@pytest.mark.parametrize("k,c", fams(ALL))
def test_matmul_vs_oracle(efl, k, c):
    """PaillierMatmul against the oracle bit for bit at every key size and n^2 kernel family (the
    2048- and 4096-bit keys run k_matmul28 / k_mmevents at G = 2 / 4 lanes per number)."""
    with family(k["n_bytes"] // 4, False, c):
        _matmul_vs_oracle(efl, k)


def _matmul_vs_oracle(efl, k=None):
    k = k or ENC_KEYS[0]
    kp = keypair(efl, k)
    okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))
    rng = np.random.default_rng(5)
    u, v, w = 3, 5, 4
    xm_plain = rng.integers(-2**20, 2**20, (u, v))
    ct = kp.encrypt(torch.from_numpy(xm_plain))
    xe = rng.integers(-30, -10, (u, v))
    ym = rng.integers(-2**20, 2**20, (v, w))
    ym[0, 0] = 0
    ye = rng.integers(-25, -12, (v, w))
    zm, ze = kp.matmul(ct.tensor, torch.from_numpy(xe), torch.from_numpy(ym), torch.from_numpy(ye))
    xs = [[int(s, 16) for s in row] for row in np.array(ct.tensor.to_hex().strings()).reshape(u, v)]
    om, oe = _oracle_matmul(okp, xs, xe, ym, ye)
    assert np.array_equal(ze.cpu().numpy(), np.array(oe))
    assert zm.to_hex().to_ints() == [c for row in om for c in row]
    # and the plaintext meaning: sum_j xm*ym*2^(xe+ye-min)
    dec = kp.decrypt(zm, dtype="string").to_ints()
    want = [sum(int(xm_plain[i, j]) * int(ym[j, q]) * 2 ** int(xe[i, j] + ye[j, q] - oe[i][q]) for j in range(v))
            for i in range(u) for q in range(w)]
    assert dec == want


_ORACLE_MM = {}


def _oracle_matmul(okp, xs, xe, ym, ye):
    """oracle.paillier.matmul, memoised on its inputs: the result does not depend on the kernel
    family, and a 4096-bit case costs the Python oracle up to ~10 s."""
    key = (okp.n, str(xs), xe.tobytes(), ym.tobytes(), ye.tobytes())
    if key not in _ORACLE_MM:
        _ORACLE_MM[key] = P.matmul(okp, xs, xe.tolist(), ym.tolist(), ye.tolist())
    return _ORACLE_MM[key]


def _matmul_case(efl, xe, ym, ye, seed, k=None):
    k = k or ENC_KEYS[0]
    kp = keypair(efl, k)
    okp = P.Keypair(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))
    u, v = xe.shape
    xm_plain = np.random.default_rng(seed).integers(-2**20, 2**20, (u, v))
    ct = kp.encrypt(torch.from_numpy(xm_plain))
    zm, ze = kp.matmul(ct.tensor, torch.from_numpy(xe), torch.from_numpy(ym), torch.from_numpy(ye))
    xs = [[int(s, 16) for s in row] for row in np.array(ct.tensor.to_hex().strings()).reshape(u, v)]
    om, oe = _oracle_matmul(okp, xs, xe, ym, ye)
    assert np.array_equal(ze.cpu().numpy(), np.array(oe))
    assert zm.to_hex().to_ints() == [c for row in om for c in row]


def _schedule_case(case):
    rng = np.random.default_rng(21)
    u, v, w = 3, 5, 4
    xe = rng.integers(-30, -10, (u, v))
    ye = rng.integers(-25, -12, (v, w))
    ym = rng.integers(-2**11, 2**11, (v, w))
    if case == "level_scan":
        xe[:, 0] -= 300
    elif case == "over_capacity":
        ym = rng.integers(-2**60, 2**60, (v, w))
    elif case == "deep":
        xe[:, 1] -= 1100
    elif case == "mixed":
        xe[1, 2] -= 1100
        ym[:, 1] = rng.integers(-2**60, 2**60, v)
    return xe, ym, ye


@pytest.mark.parametrize("case", ["sorted", "level_scan", "over_capacity", "deep", "mixed"])
@pytest.mark.parametrize("splits", [0, 1])
@pytest.mark.parametrize("c", [16, 32])
def test_matmul_schedule_paths(efl, case, splits, c):
    """Every path of the multiply schedules (k_mmevents / k_matmul28) equals the oracle: the LDS
    counting sort (levels < 128), the builder's level-major scan (levels 128..1023), and the
    in-kernel scan for lists that do not fit — more than 5 windows per term (60-bit weights) or a
    level past 1023 — alone and next to listed outputs in the same wave ("mixed": one row's
    exponents spread past 1023)."""
    xe, ym, ye = _schedule_case(case)
    lib = efl.lib.raw()
    ln = ENC_KEYS[0]["n_bytes"] // 4
    prev = lib.efl_pl_tune(ln, 3, splits)
    try:
        with family(ln, False, c):
            _matmul_case(efl, xe, ym, ye, 3)
    finally:
        lib.efl_pl_tune(ln, 3, prev)


@pytest.mark.parametrize("case", ["sorted", "level_scan", "over_capacity", "deep", "mixed"])
@pytest.mark.parametrize("k,c", fams(ALL[1:]))
def test_matmul_schedule_paths_every_key(efl, k, c, case):
    """The same schedule paths at the 1024-, 2048- and 4096-bit keys, every n^2 family, default
    term splits: bit-identical to the oracle."""
    xe, ym, ye = _schedule_case(case)
    with family(k["n_bytes"] // 4, False, c):
        _matmul_case(efl, xe, ym, ye, 3, k)


@pytest.mark.parametrize("splits", [1, 2, 3, 4, 16])
def test_matmul_term_splits(efl, splits):
    """efl_pl_tune(ln, 3, S) fixes k_matmul28's term splits (rounded down to a power of two, at
    most v; S = 1 writes the outputs directly, S > 1 goes through k_matcomb28): the same ciphertexts
    as the oracle for each."""
    lib = efl.lib.raw()
    ln = ENC_KEYS[0]["n_bytes"] // 4
    prev = lib.efl_pl_tune(ln, 3, splits)
    try:
        assert lib.efl_pl_tune(ln, 3, -1) == splits
        _matmul_vs_oracle(efl)
    finally:
        lib.efl_pl_tune(ln, 3, prev)
    assert lib.efl_pl_tune(ln, 3, 17) < 0
    assert lib.efl_pl_tune(ln, 3, -1) == prev


def test_matmul_many_outputs_plaintext(efl):
    """Many outputs, each output's terms in one group (S = 1, set through efl_pl_tune; the small
    oracle cases above take the split + combine path by default): exact plaintexts of sampled
    outputs, both signs, zeros and exponent spreads."""
    k = ENC_KEYS[0]
    kp = keypair(efl, k)
    lib = efl.lib.raw()
    prev = lib.efl_pl_tune(k["n_bytes"] // 4, 3, 1)
    try:
        _many_outputs(kp)
    finally:
        lib.efl_pl_tune(k["n_bytes"] // 4, 3, prev)


def _many_outputs(kp):
    rng = np.random.default_rng(11)
    u, v, w = 512, 3, 256
    xm = rng.integers(-2**30, 2**30, (u, v))
    xe = rng.integers(-40, -5, (u, v))
    ym = rng.integers(-2**11, 2**11, (v, w))
    ym[1, ::7] = 0
    ye = rng.integers(-30, -3, (v, w))
    ct = kp.encrypt(torch.from_numpy(xm))
    zm, ze = kp.matmul(ct.tensor, torch.from_numpy(xe), torch.from_numpy(ym), torch.from_numpy(ye))
    ze = ze.cpu().numpy()
    ex = xe[:, :, None] + ye[None, :, :]
    assert np.array_equal(ze, ex.min(axis=1))
    pick = rng.choice(u * w, 200, replace=False)
    from efl.privacy import paillier_cipher as pc
    sub = pc.CipherTensor(zm.limbs[torch.from_numpy(pick).to(zm.limbs.device)], (len(pick),), kp.key)
    dec = kp.decrypt(sub, dtype="string").to_ints()
    for o, got in zip(pick.tolist(), dec):
        i, q = divmod(o, w)
        assert got == sum(int(xm[i, j]) * int(ym[j, q]) << int(ex[i, j, q] - ze[i, q]) for j in range(v)), o


def test_fixed_point_matmul_and_mul_like_reference_test(efl):
    """paillier_test.py:49-79 (mul_scalar, matmul) with a 512-bit key; exact plaintext check."""
    kp = efl.paillier.Keypair()
    kp.generate_keypair(n_bytes=64)
    g = torch.Generator().manual_seed(2)
    a = torch.randn(6, 5, generator=g).cuda()
    b = torch.randn(6, 5, generator=g).cuda()
    fa = efl.paillier.fixedpoint.encode(a)
    fa.mantissa = kp.encrypt(fa.mantissa)
    c2 = fa * b
    c2.mantissa = c2.mantissa.decrypt()
    c2 = efl.paillier.fixedpoint.decode(c2)
    assert torch.allclose(a * b, c2)
    bm = torch.randn(5, 3, generator=g).cuda()
    fa = efl.paillier.fixedpoint.encode(a)
    fa.mantissa = kp.encrypt(fa.mantissa)
    c3 = fa @ bm
    c3.mantissa = c3.mantissa.decrypt()
    c3 = efl.paillier.fixedpoint.decode(c3)
    assert torch.allclose(a @ bm, c3, 1e-5, 1e-4)


def test_refused_rekey_keeps_the_old_key(efl):
    """A re-key the library refuses on the host (an even n, a_bytes out of range, n past 8192 bits)
    leaves the keypair's previous key working (the old key used to be dropped first)."""
    from efl import errors
    k = ENC_KEYS[1]
    kp = keypair(efl, k)
    vs = k["vectors"][:4]
    hsa = [v["hsa"] for v in vs]
    m = torch.tensor([v["m"] for v in vs], dtype=torch.int64)
    before = kp.key
    for bad in (dict(n=int(k["n"], 16) + 1, a=64), dict(n=int(k["n"], 16), a=0), dict(n=(1 << 8200) + 1, a=64)):
        with pytest.raises((errors.InvalidArgumentError, errors.UnimplementedError)):
            kp.set_keys_ints(bad["n"], int(k["hs"], 16), bad["a"], 1)
        assert kp.key is before
        assert kp.encrypt(m, hsa=hsa).tensor.to_hex().strings() == [v["c"] for v in vs]
        assert kp.decrypt(efl.HexTensor.from_strings([v["c"] for v in vs]), dtype=torch.int64).cpu().tolist() == \
            [v["m"] for v in vs]
