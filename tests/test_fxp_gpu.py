"""GPU parity: libefl_hip.so's Stage-F kernels vs the oracle and the golden fixtures.

Bar: bit-exact (integer work on IEEE bit patterns; the decode reproduces GMP's truncating
mpf_get_d). All calls go through the C ABI via the `efl` package.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import fxp

pytestmark = pytest.mark.gpu

G = np.load(os.path.join(GOLDEN, "fxp_golden.npz"))
H = np.load(os.path.join(GOLDEN, "fxp_hex_golden.npz"))


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.cpu().numpy()


def bits32(t):
    return host(t).view(np.uint32)


def bits64(t):
    return host(t).view(np.uint64)


# ------------------------------------------------------------------------------ golden sets

@pytest.mark.parametrize("dp", [0, 1])
def test_encode_f32_golden(efl, dp):
    x = dev(G["f32_bits"].view(np.float32))
    fp = efl.paillier.fixedpoint.encode(x, decrease_precision=bool(dp))
    assert np.array_equal(host(fp.mantissa), G[f"f32_M_dp{dp}"])
    assert np.array_equal(host(fp.exponent), G[f"f32_E_dp{dp}"])


@pytest.mark.parametrize("dp", [0, 1])
@pytest.mark.parametrize("ftz", [0, 1])
def test_round_trip_f32_golden(efl, dp, ftz):
    M, E = dev(G[f"f32_M_dp{dp}"]), dev(G[f"f32_E_dp{dp}"])
    y = efl.lib.ops.fixed_point_to_float_point(M, E, torch.float32, flush_denormal=bool(ftz))
    assert np.array_equal(bits32(y), G[f"f32_rt_dp{dp}_ftz{ftz}"])


@pytest.mark.parametrize("dp", [0, 1])
def test_f64_golden(efl, dp):
    x = dev(G["f64_bits"].view(np.float64))
    fp = efl.paillier.fixedpoint.encode(x, decrease_precision=bool(dp))
    assert np.array_equal(host(fp.mantissa), G[f"f64_M_dp{dp}"])
    assert np.array_equal(host(fp.exponent), G[f"f64_E_dp{dp}"])
    y = efl.paillier.fixedpoint.decode(fp, dtype=torch.float64)
    assert np.array_equal(bits64(y), G[f"f64_rt_dp{dp}"])


@pytest.mark.parametrize("name", ["int8", "int16", "int32", "int64"])
def test_encode_int_golden(efl, name):
    fp = efl.paillier.fixedpoint.encode(dev(G[name]))
    assert np.array_equal(host(fp.mantissa), G[name].astype(np.int64))
    assert not host(fp.exponent).any()


@pytest.mark.parametrize("ftz", [0, 1])
def test_decode_i64_golden(efl, ftz):
    y = efl.lib.ops.fixed_point_to_float_point(dev(G["dec_M"]), dev(G["dec_E"]), "float32",
                                               flush_denormal=bool(ftz))
    assert np.array_equal(bits32(y), G[f"dec_f32_ftz{ftz}"])


def test_decode_i64_f64_golden(efl):
    y = efl.lib.ops.fixed_point_to_float_point(dev(G["dec_M"]), dev(G["dec_E"]), torch.float64)
    assert np.array_equal(bits64(y), G["dec_f64"])


def test_decode_fast_path_boundaries(efl):
    """The decode kernels take an exact ldexp path for |M| < 2^53 and E >= -1022 and GMP's
    bit-by-bit truncation otherwise: every pair straddling that boundary, in every vector lane
    position (odd-sized batches reach the scalar tail too), against the GMP-pinned oracle."""
    ms = [0, 1, -1, 3, (1 << 53) - 1, -((1 << 53) - 1), 1 << 53, -(1 << 53), (1 << 53) + 1,
          -((1 << 53) + 1), (1 << 62) + 12345, -(1 << 63), (1 << 63) - 1, 0x00FFFFFF, -0x00FFFFFF]
    es = [-1023, -1022, -1021, -1074, -1075, -1200, -150, -149, 0, 971, 972, 1000, 4096, 4097,
          1 << 40, -(1 << 40), (1 << 62), -(1 << 62)]
    M = np.array([m for m in ms for _ in es], np.int64)
    E = np.array([e for _ in ms for e in es], np.int64)
    for sl in (slice(None), slice(1, None), slice(0, -3)):
        m, e = M[sl], E[sl]
        for ftz in (0, 1):
            y = efl.lib.ops.fixed_point_to_float_point(dev(m), dev(e), "float32", flush_denormal=bool(ftz))
            assert np.array_equal(bits32(y), fxp.gmp_decode(m, e, np.float32, bool(ftz)).view(np.uint32))
        y = efl.lib.ops.fixed_point_to_float_point(dev(m), dev(e), torch.float64)
        assert np.array_equal(bits64(y), fxp.gmp_decode(m, e, np.float64).view(np.uint64))


def _hex():
    b, o = H["buf"].tobytes(), H["offs"]
    return [b[o[i]:o[i + 1]] for i in range(o.size - 1)]


@pytest.mark.parametrize("ftz", [0, 1])
def test_decode_hex_golden(efl, ftz):
    hx = efl.HexTensor.from_strings(np.array(_hex(), dtype=object))
    y = efl.lib.ops.fixed_point_to_float_point(hx, dev(H["E"]), torch.float32, flush_denormal=bool(ftz))
    assert np.array_equal(bits32(y), H[f"f32_ftz{ftz}"])
    y64 = efl.lib.ops.fixed_point_to_float_point(hx, dev(H["E"]), torch.float64)
    assert np.array_equal(bits64(y64), H["f64"])


def test_decode_hex_malformed(efl):
    hx = efl.HexTensor.from_strings(["1f", "xyz", "-3"])
    with pytest.raises(efl.errors.InvalidArgumentError, match=r"mantissa\[1\]"):
        efl.lib.ops.fixed_point_to_float_point(hx, dev(np.zeros(3, np.int64)))


@pytest.mark.parametrize("ftz", [None, 0, 1])
def test_relu_zeros_and_denormals_both_modes(efl, ftz):
    """ReLU-style activations (half exact zeros), +-0.0 and every denormal class,
    round-tripped through the GPU codec and compared with GMP run in the same MXCSR mode. The
    default (ftz=None) is the op as TF runs it (FTZ|DAZ): zeros come back as signed zeros."""
    rng = np.random.default_rng(21)
    x = np.maximum(rng.standard_normal(1 << 16).astype(np.float32), 0)     # ReLU
    x[:8] = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-40, -1e-39, 1.1754942e-38, -1.1754942e-38], np.float32)
    x[8:40] = (np.arange(1, 33, dtype=np.uint32) << np.uint32(18)).view(np.float32)   # denormals
    fp = efl.paillier.fixedpoint.encode(dev(x))
    Mo, Eo = fxp.encode(x)
    assert np.array_equal(host(fp.mantissa), Mo) and np.array_equal(host(fp.exponent), Eo)
    mode = True if ftz is None else bool(ftz)
    y = efl.lib.ops.fixed_point_to_float_point(fp.mantissa, fp.exponent, flush_denormal=None if ftz is None else mode)
    want = fxp.gmp_decode(Mo, Eo, np.float32, mode).view(np.uint32)
    assert np.array_equal(bits32(y), want)
    if mode:      # FTZ: zeros keep their sign, denormal inputs flush to signed zero
        assert bits32(y)[0] == 0 and bits32(y)[1] == 0x80000000
        assert (bits32(y)[(x == 0)] & 0x7FFFFFFF == 0).all()
        normal = np.abs(x) >= np.float32(1.1754944e-38)
        assert np.array_equal(bits32(y)[normal], x[normal].view(np.uint32))
    else:         # bare loop: +-0.0 -> +-2^-127
        assert bits32(y)[0] == 0x00400000 and bits32(y)[1] == 0x80400000
    # the batched decode honours the same mode
    ys = efl.lib.ops.fixed_point_to_float_point_batched([fp.mantissa[:1000], fp.mantissa],
                                                        [fp.exponent[:1000], fp.exponent],
                                                        flush_denormal=None if ftz is None else mode)
    assert np.array_equal(bits32(ys[1]), want) and np.array_equal(bits32(ys[0]), want[:1000])


def test_batched_decode_validates_pairs(efl):
    M = torch.zeros(8, dtype=torch.int64, device="cuda")
    E = torch.zeros(8, dtype=torch.int64, device="cuda")
    with pytest.raises(efl.errors.InvalidArgumentError, match="same size"):
        efl.lib.ops.fixed_point_to_float_point_batched([M], [E[:7]])
    with pytest.raises(efl.errors.InvalidArgumentError, match="int64"):
        efl.lib.ops.fixed_point_to_float_point_batched([M.int()], [E])
    with pytest.raises(efl.errors.InvalidArgumentError, match="as many"):
        efl.lib.ops.fixed_point_to_float_point_batched([M, M], [E])
    # a strided view decodes its own elements
    Mb = torch.arange(16, dtype=torch.int64, device="cuda") + 1
    Eb = torch.zeros(16, dtype=torch.int64, device="cuda")
    (y,) = efl.lib.ops.fixed_point_to_float_point_batched([Mb[::2]], [Eb[::2]])
    assert torch.equal(y.cpu(), torch.arange(1, 17, 2, dtype=torch.float32))


# ---------------------------------------------------------------- seeded inputs vs oracle

SIZES = [0, 1, 2, 3, 5, 127, 255, 256, 1023, 4097, 65537, (1 << 20) + 3]


def rand_bits(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    x[: n // 3] = rng.standard_normal(n // 3).astype(np.float32).view(np.uint32)
    return x


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dp", [0, 1])
def test_f32_vs_oracle(efl, n, dp):
    xb = rand_bits(n, n + 17 * dp)
    x = xb.view(np.float32)
    fp = efl.paillier.fixedpoint.encode(dev(x), decrease_precision=bool(dp))
    Mo, Eo = fxp.encode(x, dp)
    assert np.array_equal(host(fp.mantissa), Mo) and np.array_equal(host(fp.exponent), Eo)
    y = efl.paillier.fixedpoint.decode(fp)
    assert np.array_equal(bits32(y), fxp.decode(Mo, Eo).view(np.uint32))


@pytest.mark.parametrize("n", [1, 3, 1000, 4099])
def test_f64_and_int_vs_oracle(efl, n):
    rng = np.random.default_rng(n)
    xb = rng.integers(0, 1 << 63, n, dtype=np.uint64) | (rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
    xd = xb.view(np.float64)
    fp = efl.paillier.fixedpoint.encode(dev(xd))
    Mo, Eo = fxp.encode(xd)
    assert np.array_equal(host(fp.mantissa), Mo) and np.array_equal(host(fp.exponent), Eo)
    assert np.array_equal(bits64(efl.paillier.fixedpoint.decode(fp, torch.float64)),
                          fxp.decode(Mo, Eo, np.float64).view(np.uint64))
    for dt in (np.int8, np.int16, np.int32, np.int64):
        xi = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, n, dtype=np.int64).astype(dt)
        fp = efl.paillier.fixedpoint.encode(dev(xi))
        assert np.array_equal(host(fp.mantissa), xi.astype(np.int64))


@pytest.mark.parametrize("knob", [(21, 256), (21, 512), (21, 1024), (22, 2), (23, 1), (23, 3), (24, 0), (24, 1)])
def test_f64_encode_shapes_identical(efl, knob):
    """Every launch shape of the fp64 encode (efl_fxp_tune 21-24: workgroup size, units per lane,
    NT mask, XCD-aware order) gives the oracle's bits, ragged tails and tiles smaller than a grid
    included (fixed_point.cc:144-192)."""
    lib = efl.lib.raw()
    n = (1 << 20) + 13
    rng = np.random.default_rng(knob[0] * 1000 + knob[1])
    xb = rng.integers(0, 1 << 63, n, dtype=np.uint64) | (rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
    xd = xb.view(np.float64)
    Mo, Eo = fxp.encode(xd)
    prev = lib.efl_fxp_tune(*knob)
    assert prev >= 0
    try:
        for dp in (False, True):
            fp = efl.paillier.fixedpoint.encode(dev(xd), decrease_precision=dp)
            if not dp:
                assert np.array_equal(host(fp.mantissa), Mo) and np.array_equal(host(fp.exponent), Eo)
            else:
                Md, Ed = fxp.encode(xd, decrease_precision=True)
                assert np.array_equal(host(fp.mantissa), Md) and np.array_equal(host(fp.exponent), Ed)
    finally:
        lib.efl_fxp_tune(knob[0], prev)


@pytest.mark.parametrize("offset", [1, 2, 3])
def test_unaligned_views(efl, offset):
    n = 10007
    x = rand_bits(n + offset, 99).view(np.float32)
    xt = dev(x)[offset:]
    assert xt.data_ptr() % 16 != 0
    fp = efl.paillier.fixedpoint.encode(xt)
    Mo, Eo = fxp.encode(x[offset:])
    assert np.array_equal(host(fp.mantissa), Mo)
    Mt = torch.empty(n + offset, dtype=torch.int64, device="cuda")[offset:]
    Et = torch.empty(n + offset, dtype=torch.int64, device="cuda")[offset:]
    Mt.copy_(fp.mantissa)
    Et.copy_(fp.exponent)
    y = efl.lib.ops.fixed_point_to_float_point(Mt, Et)
    assert np.array_equal(bits32(y), fxp.decode(Mo, Eo).view(np.uint32))


def test_shapes_and_host_staging(efl):
    x = torch.randn(7, 33, 5, generator=torch.Generator().manual_seed(3))
    fp = efl.paillier.fixedpoint.encode(x)          # CPU tensor in -> CPU tensors out
    assert fp.mantissa.device.type == "cpu" and fp.mantissa.shape == x.shape
    Mo, Eo = fxp.encode(x.numpy())
    assert np.array_equal(fp.mantissa.numpy(), Mo) and np.array_equal(fp.exponent.numpy(), Eo)
    y = efl.paillier.fixedpoint.decode(fp)
    assert y.device.type == "cpu" and torch.equal(y, x)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32])
def test_large_host_tensors_take_the_pipeline(efl, dtype):
    """Host tensors of HOST_PIPELINE_MIN_ELEMS or more go through the pinned three-stream pipeline
    (several chunks and a ragged last one here, a pageable source, a non-contiguous view): the same
    bits as the device path, back on the host, for both directions and decrease_precision."""
    n = efl.lib.HOST_PIPELINE_MIN_ELEMS * 2 + 77
    g = torch.Generator().manual_seed(9)
    if dtype.is_floating_point:
        base = torch.randn(n + 1, generator=g, dtype=dtype)
        base[:4] = torch.tensor([0.0, -0.0, 2.0 ** 23 + 1, 1e-40], dtype=dtype)
    else:
        base = torch.randint(-2**31, 2**31 - 1, (n + 1,), generator=g, dtype=dtype)
    x = base[1:]                                     # offset view of a pageable tensor
    for dp in (False, True):
        M, E = efl.lib.ops.convert_to_fixed_point(x, decrease_precision=dp)
        Md, Ed = efl.lib.ops.convert_to_fixed_point(x.cuda(), decrease_precision=dp)
        assert M.device.type == "cpu" and M.shape == x.shape
        assert torch.equal(M, Md.cpu()) and torch.equal(E, Ed.cpu())
    if dtype.is_floating_point:
        y = efl.lib.ops.fixed_point_to_float_point(M, E, dtype)
        yd = efl.lib.ops.fixed_point_to_float_point(Md, Ed, dtype)
        assert y.device.type == "cpu" and y.dtype == dtype
        assert torch.equal(y.view(-1).view(torch.uint8), yd.cpu().view(-1).view(torch.uint8))


def test_errors(efl):
    with pytest.raises(efl.errors.InvalidArgumentError, match="same size"):
        efl.lib.ops.fixed_point_to_float_point(dev(np.zeros(4, np.int64)), dev(np.zeros(5, np.int64)))
    with pytest.raises(efl.errors.InvalidArgumentError):
        efl.paillier.fixedpoint.encode(torch.zeros(4, dtype=torch.uint8, device="cuda"))
    with pytest.raises(efl.errors.InvalidArgumentError):
        efl.lib.ops.fixed_point_to_float_point(dev(np.zeros(4, np.int64)), dev(np.zeros(4, np.int64)),
                                               torch.int32)


@pytest.mark.parametrize("knob", [(0, 1), (1, 1), (2, 2), (3, 2), (4, 1), (5, 0), (4, 3), (6, 128), (7, 512), (8, 512),
                                  (6, 1024), (14, 1), (15, 0), (16, 1)])
def test_tuning_variants_identical(efl, knob):
    lib = efl.lib.raw()
    n = (1 << 18) + 7
    x = rand_bits(n, 7).view(np.float32)
    Mo, Eo = fxp.encode(x)
    yo = fxp.decode(Mo, Eo).view(np.uint32)
    prev = lib.efl_fxp_tune(*knob)
    try:
        fp = efl.paillier.fixedpoint.encode(dev(x))
        assert np.array_equal(host(fp.mantissa), Mo) and np.array_equal(host(fp.exponent), Eo)
        assert np.array_equal(bits32(efl.paillier.fixedpoint.decode(fp)), yo)
    finally:
        lib.efl_fxp_tune(knob[0], prev)


# ----------------------------------------------------------------------------- batched

def test_batched_ragged(efl):
    rng = np.random.default_rng(11)
    sizes = [0, 1, 2, 3, 16384, 4097, 100000] + [int(s) for s in rng.integers(1, 40000, 200)]
    xs_np = [rand_bits(s, i).view(np.float32) for i, s in enumerate(sizes)]
    xs = [dev(a) for a in xs_np]
    xs[5] = dev(np.concatenate([[0], xs_np[5].view(np.uint32)]).astype(np.uint32).view(np.float32))[1:]
    Ms, Es = efl.lib.ops.convert_to_fixed_point_batched(xs, decrease_precision=False)
    for a, M, E in zip(xs_np, Ms, Es):
        Mo, Eo = fxp.encode(a)
        assert np.array_equal(host(M), Mo) and np.array_equal(host(E), Eo)
    ys = efl.lib.ops.fixed_point_to_float_point_batched(Ms, Es)
    for a, y in zip(xs_np, ys):
        Mo, Eo = fxp.encode(a)
        assert np.array_equal(bits32(y), fxp.decode(Mo, Eo).view(np.uint32))


@pytest.mark.parametrize("knob", [(10, 256), (10, 128), (11, 1), (11, 4), (12, 256), (12, 128), (13, 1), (13, 4),
                                  (17, 1), (17, 2), (17, 3), (18, 1), (18, 2), (18, 3), (19, 7), (26, 2), (26, 4),
                                  (26, 8), (27, 2), (27, 4), (27, 8)])
def test_batched_tuning_variants_identical(efl, knob):
    """Every batched fp32 tile shape and tile order (efl_fxp_tune 10-13, 17-19: 2-D grid, flat,
    flat XCD-aware, persistent walk and its workgroup count; 26-27 tiles per workgroup) gives the
    same bits; ragged sizes,
    tensors smaller than a tile, and (for the persistent walk with 7 workgroups) many tiles each."""
    lib = efl.lib.raw()
    if knob[0] == 19:
        prev_order = (lib.efl_fxp_tune(17, 3), lib.efl_fxp_tune(18, 3))
    sizes = [1, 5, 4095, 16384, 30001, 2, 65536 + 3]
    xs_np = [rand_bits(n, 40 + n).view(np.float32) for n in sizes]
    prev = lib.efl_fxp_tune(*knob)
    assert prev >= 0
    xs = [dev(a) for a in xs_np]
    # one tensor 4 bytes off 16-B alignment: its tiles take the element path in every order
    xs[2] = dev(np.concatenate([[0], xs_np[2].view(np.uint32)]).astype(np.uint32).view(np.float32))[1:]
    try:
        Ms, Es = efl.lib.ops.convert_to_fixed_point_batched(xs)
        ys = efl.lib.ops.fixed_point_to_float_point_batched(Ms, Es)
    finally:
        lib.efl_fxp_tune(knob[0], prev)
        if knob[0] == 19:
            lib.efl_fxp_tune(17, prev_order[0])
            lib.efl_fxp_tune(18, prev_order[1])
    for a, M, E, y in zip(xs_np, Ms, Es, ys):
        Mo, Eo = fxp.encode(a)
        assert np.array_equal(host(M), Mo) and np.array_equal(host(E), Eo)
        assert np.array_equal(bits32(y), fxp.decode(Mo, Eo).view(np.uint32))


def test_batched_embedding_slices(efl):
    """BASELINE config 3 shape: 4096 x 64 KiB fp32 slices, N(0, 0.01), seed 1."""
    g = torch.Generator(device="cuda").manual_seed(1)
    big = torch.randn(4096 * 16384, device="cuda", generator=g) * 0.01
    xs = list(big.view(4096, 16384).unbind(0))
    Ms, Es = efl.lib.ops.convert_to_fixed_point_batched(xs)
    ys = efl.lib.ops.fixed_point_to_float_point_batched(Ms, Es)
    y = torch.stack(ys)
    assert torch.equal(y.view(-1)[big != 0], big[big != 0])
    idx = np.random.default_rng(0).integers(0, 4096, 8)
    for i in idx:
        Mo, Eo = fxp.encode(host(xs[i]))
        assert np.array_equal(host(Ms[i]), Mo) and np.array_equal(host(Es[i]), Eo)


@pytest.mark.parametrize("coalesce", ["single", True])
def test_batched_config3_separate_full_size(efl, coalesce):
    """BASELINE config 3 exactly as bench.py's `config3` (layout "separate") builds it: 4096
    [128, 128] fp32 slices, N(0, 0.01), seed 1, every slice and every output its own allocation.
    coalesce="single" (the default) keeps one table entry per slice, so the batched kernels
    (efl_fxp_encode_batched / efl_fxp_decode_batched) run with count = 4096; True merges the
    runs the caching allocator happened to lay out back to back. Every element of all 4096 slices
    is compared bit for bit with the oracle (fixed_point.cc:106-138 encode, :235-248 decode, FTZ)."""
    slices = 4096
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(128, 128, device="cuda", generator=g) * 0.01 for _ in range(slices)]
    Ms = [torch.empty(128, 128, dtype=torch.int64, device="cuda") for _ in range(slices)]
    Es = [torch.empty(128, 128, dtype=torch.int64, device="cuda") for _ in range(slices)]
    ys = [torch.empty(128, 128, device="cuda") for _ in range(slices)]
    enc = efl.lib.BatchTables(xs, Ms, Es, coalesce=coalesce)
    dec = efl.lib.BatchTables(Ms, Es, ys, coalesce=coalesce)
    assert not enc.single and not dec.single
    if coalesce == "single":
        assert enc.count == slices and dec.count == slices
    else:
        assert 1 < enc.count < slices and 1 < dec.count < slices
    for t in (enc, dec):
        assert t.max_n == max(r[3] for r in t.runs)
    efl.lib.encode_batched_into(enc, 1, False)
    efl.lib.decode_batched_into(dec, 1, 1)
    torch.cuda.synchronize()
    x_h = host(torch.stack(xs)).reshape(-1)
    Mo, Eo = fxp.encode(x_h)
    M_h, E_h = host(torch.stack(Ms)).reshape(-1), host(torch.stack(Es)).reshape(-1)
    bad = np.nonzero((M_h != Mo) | (E_h != Eo))[0]
    assert bad.size == 0, f"encode differs at {bad.size} elements, first {bad[:4]} (slice {bad[0] // 16384})"
    yo = fxp.decode(Mo, Eo, ftz=True).view(np.uint32)
    y_h = bits32(torch.stack(ys)).reshape(-1)
    bad = np.nonzero(y_h != yo)[0]
    assert bad.size == 0, f"decode differs at {bad.size} elements, first {bad[:4]}"
    # per-slice checksums (a second, order-sensitive view of the same comparison)
    ck = lambda a: (a.reshape(slices, -1).astype(np.uint64) * np.arange(1, 16385, dtype=np.uint64)).sum(1)
    assert np.array_equal(ck(M_h.view(np.uint64)), ck(Mo.view(np.uint64)))


@pytest.mark.parametrize("coalesce", ["single", True, False])
def test_batched_tables_coalescing_identical(efl, coalesce):
    """BatchTables over slices of one table: as one run through the streaming kernels ("single",
    the default, and True when the slices are adjacent in all three streams) and one entry per slice
    through the batched kernels (False): the same bits. With a gap in one output buffer the batch
    is two runs: merged into two entries (True) or one entry per slice, batched kernels both."""
    S, n = 300, 5000
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(S * n, device="cuda", generator=g)
    x[::97] = 0.0
    M = torch.empty(S * n, dtype=torch.int64, device="cuda")
    E = torch.empty_like(M)
    y = torch.empty_like(x)
    xs, Ms, Es, ys = ([b[i * n:(i + 1) * n] for i in range(S)] for b in (x, M, E, y))
    enc = efl.lib.BatchTables(xs, Ms, Es, coalesce=coalesce)
    dec = efl.lib.BatchTables(Ms, Es, ys, coalesce=coalesce)
    assert enc.single == (coalesce in ("single", True)) and enc.count == {"single": 1, True: 1, False: S}[coalesce]
    efl.lib.encode_batched_into(enc, 1)
    efl.lib.decode_batched_into(dec, 1, 1)
    Mo, Eo = fxp.encode(host(x))
    assert np.array_equal(host(M), Mo) and np.array_equal(host(E), Eo)
    assert np.array_equal(bits32(y), fxp.decode(Mo, Eo).view(np.uint32))
    # a gap in one output stream: two runs (merged and chunked with coalesce=True, else one entry
    # per slice), through the batched kernels
    M2 = torch.empty(S * n + 2, dtype=torch.int64, device="cuda")
    gap = [M2[i * n + (2 if i >= S // 2 else 0):][:n] for i in range(S)]
    t = efl.lib.BatchTables(xs, gap, Es, coalesce=coalesce)
    assert not t.single and t.count == (2 if coalesce is True else S)
    efl.lib.encode_batched_into(t, 1)
    assert np.array_equal(np.concatenate([host(m) for m in gap]), Mo)


# ------------------------------------------------------------------- full size (256 MiB)

def test_full_size_properties(efl):
    """BASELINE config 2 size (67,108,864 fp32): size-independent properties, and every element of M,
    E and the decoded y compared with the oracle's."""
    n = 1 << 26
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, device="cuda", generator=g)
    fp = efl.paillier.fixedpoint.encode(x)
    y = efl.paillier.fixedpoint.decode(fp)
    nz = x != 0
    # default (FTZ, the op as TF runs it): the round trip is the identity on every bit pattern
    assert torch.equal(y.view(torch.int32), x.view(torch.int32))
    # bare loop: identity on every non-zero N(0,1) value; zeros become 2^-127
    y0 = efl.lib.ops.fixed_point_to_float_point(fp.mantissa, fp.exponent, flush_denormal=False)
    assert torch.equal(y0[nz], x[nz])
    assert torch.all(y0[~nz].view(torch.int32) == 0x00400000)
    # mantissas are odd (normalised) except the zero quirk, |M| < 2^24
    M, E = fp.mantissa, fp.exponent
    assert torch.all((M[nz] & 1) == 1) and torch.all(M.abs() < (1 << 24))
    # 1 % sampled bit compare against the oracle
    idx = torch.from_numpy(np.random.default_rng(0).integers(0, n, n // 100)).cuda()
    xs = host(x[idx])
    Mo, Eo = fxp.encode(xs)
    assert np.array_equal(host(M[idx]), Mo) and np.array_equal(host(E[idx]), Eo)
    # every element against an oracle pass over the whole tensor (not a checksum), and
    # the decode of the oracle's own mantissas / exponents against the GPU decode, bit for bit
    Mo_all, Eo_all = fxp.encode(host(x))
    assert np.array_equal(host(M), Mo_all) and np.array_equal(host(E), Eo_all)
    assert np.array_equal(bits32(y), fxp.decode(Mo_all, Eo_all).view(np.uint32))


# ------------------------------------------------- slices of the exhaustive fp32 sweep
# tools/exhaustive_fxp.py runs all 2^32 patterns (profiles/r02/exhaustive_fp32.json); here the
# same check on 2^20-pattern slices at the boundaries: +0 and the denormals, the |x| in [2^23, 2^24)
# band that loses its implicit bit, inf / NaN, and the negative mirror of each.

@pytest.mark.parametrize("start", [0x00000000, 0x007F0000, 0x4AF80000, 0x4B7F0000, 0x7F780000, 0x7FF00000,
                                   0x80000000, 0xCAF80000, 0xFF780000])
@pytest.mark.parametrize("dp", [0, 1])
def test_exhaustive_slice_vs_literal_loop_and_gmp(efl, start, dp):
    from tools import exhaustive_fxp as ex
    dev = efl.lib.require_gpu()
    count = 1 << 20
    assert ex.gpu_hash(efl, start, count, dp, dev) == ex.cpu_hash(start, count, dp, 8)


def test_exhaustive_all_fp32_patterns(efl):
    """Every one of the 2^32 fp32 bit patterns, both decrease_precision values, decode in both
    MXCSR modes: the GPU kernels equal the reference loop (restated statement for statement) + GMP
    (tools/exhaustive_fxp.py; ~15 s on the GPU box's 16 host threads)."""
    from tools import exhaustive_fxp as ex
    import bench
    dev = efl.lib.require_gpu()
    threads = bench.usable_cores()[0]
    chunk = 1 << 26
    for dp in (0, 1):
        for start in range(0, 1 << 32, chunk):
            assert ex.gpu_hash(efl, start, chunk, dp, dev) == ex.cpu_hash(start, chunk, dp, threads), (dp, hex(start))
