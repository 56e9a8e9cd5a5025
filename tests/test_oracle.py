"""CPU: pin the oracle (oracle/) against the reference's recorded outputs and GMP itself.

* SURVEY.md Appendix A holds outputs of the reference loop bodies run in this container
  (tests/golden/survey_appendix_a.json) -> the C and numpy encode restatements must match them.
* tests/golden/fxp_golden.npz decode outputs were produced by GMP 6.2.1 in the reference's call
  order (tests/golden/make_golden.py) -> the plain-C decode restatement must match bit for bit.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import fxp

G = np.load(os.path.join(GOLDEN, "fxp_golden.npz"))
H = np.load(os.path.join(GOLDEN, "fxp_hex_golden.npz"))
with open(os.path.join(GOLDEN, "survey_appendix_a.json")) as f:
    SURVEY = json.load(f)


def _f32(bits):
    return np.array([int(b, 16) for b in bits], np.uint32).view(np.float32)


@pytest.mark.parametrize("case", SURVEY["cases"], ids=lambda c: f"{c['bits']}-dp{c['dp']}")
def test_survey_appendix_a(case):
    x = _f32([case["bits"]])
    M, E = fxp.encode(x, case["dp"])
    assert (int(M[0]), int(E[0])) == (case["M"], case["E"])
    Mn, En = fxp.np_encode_f32(x, case["dp"])
    assert (int(Mn[0]), int(En[0])) == (case["M"], case["E"])
    # the survey ran the bare loop (MXCSR default): no flush to zero
    y = fxp.decode(M, E, np.float32, ftz=False).view(np.uint32)[0]
    want = int(case["decoded_bits"] or case["bits"], 16)
    assert int(y) == want
    assert int(fxp.gmp_decode(M, E, np.float32, ftz=False).view(np.uint32)[0]) == want


def test_survey_identity_round_trip():
    x = _f32(SURVEY["identity_round_trip_dp0"])
    M, E = fxp.encode(x, 0)
    assert np.array_equal(fxp.decode(M, E).view(np.uint32), x.view(np.uint32))


@pytest.mark.parametrize("dp", [0, 1])
def test_encode_f32_golden(dp):
    x = G["f32_bits"].view(np.float32)
    M, E = fxp.encode(x, dp)
    assert np.array_equal(M, G[f"f32_M_dp{dp}"]) and np.array_equal(E, G[f"f32_E_dp{dp}"])
    Mn, En = fxp.np_encode_f32(x, dp)
    assert np.array_equal(Mn, M) and np.array_equal(En, E)


@pytest.mark.parametrize("dp", [0, 1])
def test_encode_f64_golden(dp):
    x = G["f64_bits"].view(np.float64)
    M, E = fxp.encode(x, dp)
    assert np.array_equal(M, G[f"f64_M_dp{dp}"]) and np.array_equal(E, G[f"f64_E_dp{dp}"])
    Mn, En = fxp.np_encode_f64(x, dp)
    assert np.array_equal(Mn, M) and np.array_equal(En, E)


@pytest.mark.parametrize("name", ["int8", "int16", "int32", "int64"])
def test_encode_int_golden(name):
    x = G[name]
    M, E = fxp.encode(x)
    assert np.array_equal(M, x.astype(np.int64)) and not E.any()


@pytest.mark.parametrize("dp", [0, 1])
@pytest.mark.parametrize("ftz", [0, 1])
def test_round_trip_f32_golden(dp, ftz):
    y = fxp.decode(G[f"f32_M_dp{dp}"], G[f"f32_E_dp{dp}"], np.float32, ftz).view(np.uint32)
    assert np.array_equal(y, G[f"f32_rt_dp{dp}_ftz{ftz}"])
    yn = fxp.np_decode_f32(G[f"f32_M_dp{dp}"], G[f"f32_E_dp{dp}"], ftz).view(np.uint32)
    assert np.array_equal(yn, y)


@pytest.mark.parametrize("dp", [0, 1])
def test_round_trip_f64_golden(dp):
    y = fxp.decode(G[f"f64_M_dp{dp}"], G[f"f64_E_dp{dp}"], np.float64).view(np.uint64)
    assert np.array_equal(y, G[f"f64_rt_dp{dp}"])


@pytest.mark.parametrize("ftz", [0, 1])
def test_decode_i64_golden(ftz):
    y = fxp.decode(G["dec_M"], G["dec_E"], np.float32, ftz).view(np.uint32)
    assert np.array_equal(y, G[f"dec_f32_ftz{ftz}"])
    assert np.array_equal(fxp.np_decode_f32(G["dec_M"], G["dec_E"], ftz).view(np.uint32), y)


def test_decode_i64_f64_golden():
    y = fxp.decode(G["dec_M"], G["dec_E"], np.float64).view(np.uint64)
    assert np.array_equal(y, G["dec_f64"])
    assert np.array_equal(fxp.np_get_d_bits(G["dec_M"], G["dec_E"]), y)


def _hex_strings():
    b = H["buf"].tobytes()
    o = H["offs"]
    return [b[o[i]:o[i + 1]].decode() for i in range(o.size - 1)]


@pytest.mark.parametrize("ftz", [0, 1])
def test_decode_hex_golden(ftz):
    y = fxp.decode_hex(_hex_strings(), H["E"], np.float32, ftz).view(np.uint32)
    assert np.array_equal(y, H[f"f32_ftz{ftz}"])


def test_decode_hex_f64_golden():
    y = fxp.decode_hex(_hex_strings(), H["E"], np.float64).view(np.uint64)
    assert np.array_equal(y, H["f64"])


def test_gmp_live_random():
    """Fresh seeded (M, E) pairs: C restatement == GMP, both FTZ modes and f64."""
    rng = np.random.default_rng(1234)
    n = 50000
    bits = rng.integers(0, 64, n)
    M = rng.integers(0, 2**63 - 1, n, dtype=np.int64) >> (63 - bits).astype(np.int64)
    M = np.where(rng.random(n) < 0.5, -M, M)
    E = rng.integers(-1200, 1100, n).astype(np.int64)
    for ftz in (0, 1):
        assert np.array_equal(fxp.decode(M, E, np.float32, ftz).view(np.uint32),
                              fxp.gmp_decode(M, E, np.float32, ftz).view(np.uint32))
    assert np.array_equal(fxp.decode(M, E, np.float64).view(np.uint64),
                          fxp.gmp_decode(M, E, np.float64).view(np.uint64))


def test_normal_round_trip_property():
    """for N(0,1) fp32 only exact zeros change after encode->decode."""
    rng = np.random.default_rng(0)
    x = rng.standard_normal(1 << 20).astype(np.float32)
    x[::4096] = 0.0
    M, E = fxp.encode(x, 0)
    y = fxp.decode(M, E, np.float32, ftz=False)
    diff = y.view(np.uint32) != x.view(np.uint32)
    assert np.array_equal(np.nonzero(diff)[0], np.nonzero(x == 0)[0])
    assert (y[x == 0].view(np.uint32) == 0x00400000).all()   # +0.0 -> 2^-127 quirk
    y_ftz = fxp.decode(M, E, np.float32, ftz=1)
    assert np.array_equal(y_ftz.view(np.uint32), x.view(np.uint32))   # FTZ hides the quirk


def test_baseline_matches_oracle():
    rng = np.random.default_rng(5)
    x = rng.standard_normal(100003).astype(np.float32)
    M, E, y = fxp.baseline_encode_decode(x, 4)
    Mo, Eo = fxp.encode(x)
    assert np.array_equal(M, Mo) and np.array_equal(E, Eo)
    assert np.array_equal(y.view(np.uint32), fxp.decode(Mo, Eo, np.float32, ftz=1).view(np.uint32))


def test_decode_size_mismatch():
    with pytest.raises(ValueError, match="same size"):
        fxp.decode(np.zeros(3, np.int64), np.zeros(4, np.int64))


@pytest.mark.parametrize("dp", [0, 1])
def test_literal_loop_matches_restatement(dp):
    """The timed baseline runs the reference's loop body statement for statement (float-convert
    ctz, the 0u - 127 shift; oracle/fxp_gmp.c encode_f32_literal); the restatement every other
    check uses must equal it: 2^20 random patterns plus a stride through all of fp32."""
    rng = np.random.default_rng(31 + dp)
    bits = np.concatenate([rng.integers(0, 2**32, 1 << 20, dtype=np.uint64).astype(np.uint32),
                           np.arange(0, 2**32, 4093, dtype=np.uint64).astype(np.uint32),
                           G["f32_bits"]])
    x = bits.view(np.float32)
    M1, E1 = fxp.encode(x, dp)
    M2, E2 = fxp.literal_encode_f32(x, dp)
    assert np.array_equal(M1, M2) and np.array_equal(E1, E2)
