"""Generate the committed golden fixtures for the fixed-point codec (Stage F).

Provenance of each expected output (see DESIGN.md "Oracle and pinning"):

* encode (M, E)  -- oracle/fxp_oracle.c, cross-checked here against the independent numpy
                    restatement (oracle/fxp.py np_encode_*) and, in tests/test_oracle.py, against
                    the reference-loop outputs the survey recorded (survey_appendix_a.json).
* decode         -- GMP 6.2.1 itself (oracle/fxp_gmp.c: mpf_set_z / mpf_set_str ->
                    mpf_mul_2exp / mpf_div_2exp -> mpf_get_d -> (float)), i.e. the library the
                    reference's FixedPointToFloatPoint calls (fixed_point.cc:235-265); `ftz` = 1
                    runs it with MXCSR FTZ|DAZ as in TensorFlow's threadpool threads.

Run:  python tests/golden/make_golden.py      (needs gcc + /opt/conda GMP; CPU only)
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import fxp  # noqa: E402


def f32_patterns() -> np.ndarray:
    rng = np.random.default_rng(0)
    pats = []
    fr_fixed = [0, 1, 2, (1 << 13) - 1, 1 << 13, (1 << 13) + 1, 1 << 22, 0x7FFFFF, 0x400001]
    for be in range(256):
        frs = fr_fixed + [int(v) for v in rng.integers(0, 1 << 23, 3)]
        for fr in frs:
            for s in (0, 1):
                pats.append((s << 31) | (be << 23) | fr)
    pats += [int(v) for v in rng.integers(0, 1 << 32, 4096, dtype=np.uint64)]
    return np.array(pats, np.uint64).astype(np.uint32)


def f64_patterns() -> np.ndarray:
    rng = np.random.default_rng(1)
    pats = []
    fr_fixed = [0, 1, (1 << 42) - 1, 1 << 42, (1 << 42) + 1, 1 << 51, (1 << 52) - 1]
    for be in range(2048):
        frs = fr_fixed + [int(v) for v in rng.integers(0, 1 << 52, 1, dtype=np.uint64)]
        for fr in frs:
            for s in (0, 1):
                pats.append((s << 63) | (be << 52) | fr)
    pats += [int(v) for v in rng.integers(0, 1 << 63, 4096, dtype=np.uint64)]
    pats += [int(v) | (1 << 63) for v in rng.integers(0, 1 << 63, 4096, dtype=np.uint64)]
    return np.array(pats, np.uint64)


def decode_pairs():
    """(M, E) pairs for the int64-mantissa decode: boundaries of every IEEE regime."""
    rng = np.random.default_rng(2)
    Ms, Es = [], []

    def add(a, L, p):
        Ms.extend([a, -a])
        Es.extend([L - p, L - p])

    for L in list(range(-1090, -1015)) + list(range(-160, -115)) + list(range(120, 132)) + \
            list(range(1015, 1030)):
        for p in (0, 1, 5, 23, 24, 25, 52, 53, 54, 62):
            a = (1 << p) | int(rng.integers(0, 1 << p)) if p else 1
            add(a, L, p)
    # half-way cases for the f32 rounding and truncation-then-round (double rounding) cases
    for _ in range(2000):
        p = int(rng.integers(25, 63))
        a = (1 << p) | int(rng.integers(0, 1 << p))
        r = int(rng.integers(0, 4))
        if r == 0:   # exact f32 tie after truncation to 53 bits, sticky bits below 53
            a = (a >> (p - 24)) << (p - 24) | (1 << (p - 25))
            if p > 53:
                a |= int(rng.integers(1, 1 << (p - 53)))
        add(a, int(rng.integers(-140, 120)), p)
    # just below the f32 normal range: FTZ tininess is decided after rounding (x86)
    for p in range(20, 63):
        for a in ((1 << (p + 1)) - 1, (1 << (p + 1)) - (1 << max(p - 24, 0)),
                  (1 << (p + 1)) - (1 << max(p - 25, 0))):
            for L in (-127, -128, -149, -150, -151):
                add(a, L, p)
    # random full-range
    n = 6000
    bits = rng.integers(0, 64, n)
    M = rng.integers(0, 2**63 - 1, n, dtype=np.int64) >> (63 - bits).astype(np.int64)
    M = np.where(rng.random(n) < 0.5, -M, M)
    E = rng.integers(-1300, 1200, n).astype(np.int64)
    Ms.extend(M.tolist())
    Es.extend(E.tolist())
    # extremes
    for m in (0, 1, -1, 2**63 - 1, -2**63, -(2**63 - 1)):
        for e in (0, -1, 1, -150, -1074, -1075, 1023, 1024, 2**20, -2**20, 2**40, -2**40):
            Ms.append(m)
            Es.append(e)
    return np.array(Ms, np.int64), np.array(Es, np.int64)


def hex_cases():
    rng = np.random.default_rng(3)
    strs, E = [], []
    for k in range(1500):
        nd = int(rng.integers(1, 260))
        s = "".join("0123456789abcdef"[int(v)] for v in rng.integers(0, 16, nd)).lstrip("0") or "0"
        if k % 3 == 0:
            s = "-" + s
        if k % 11 == 0:
            s = s.upper()
        strs.append(s)
        E.append(int(rng.integers(-1300, 160)) - 2 * nd)
    strs += ["0", "-0", "1", "-1", "f" * 512, "-" + "f" * 512, "1" + "0" * 255, "7fffffffffffffff",
             "8000000000000000", "-8000000000000000", "ffffffffffffffffff"]
    E += [0, 0, -150, -127, -2048, -2048, -1100, -62, -63, -63, -72]
    return strs, np.array(E, np.int64)


def main():
    fxp.build()
    out = {}

    x32 = f32_patterns()
    out["f32_bits"] = x32
    f = x32.view(np.float32)
    for dp in (0, 1):
        M, E = fxp.encode(f, dp)
        Mn, En = fxp.np_encode_f32(f, dp)
        assert (M == Mn).all() and (E == En).all(), "C and numpy encode restatements disagree"
        out[f"f32_M_dp{dp}"] = M
        out[f"f32_E_dp{dp}"] = E
        for ftz in (0, 1):
            y = fxp.gmp_decode(M, E, np.float32, ftz)
            out[f"f32_rt_dp{dp}_ftz{ftz}"] = y.view(np.uint32)

    x64 = f64_patterns()
    out["f64_bits"] = x64
    d = x64.view(np.float64)
    for dp in (0, 1):
        M, E = fxp.encode(d, dp)
        Mn, En = fxp.np_encode_f64(d, dp)
        assert (M == Mn).all() and (E == En).all()
        out[f"f64_M_dp{dp}"] = M
        out[f"f64_E_dp{dp}"] = E
        out[f"f64_rt_dp{dp}"] = fxp.gmp_decode(M, E, np.float64).view(np.uint64)

    Mi, Ei = decode_pairs()
    out["dec_M"] = Mi
    out["dec_E"] = Ei
    for ftz in (0, 1):
        out[f"dec_f32_ftz{ftz}"] = fxp.gmp_decode(Mi, Ei, np.float32, ftz).view(np.uint32)
    out["dec_f64"] = fxp.gmp_decode(Mi, Ei, np.float64).view(np.uint64)

    rng = np.random.default_rng(4)
    out["int8"] = rng.integers(-128, 128, 512).astype(np.int8)
    out["int16"] = rng.integers(-32768, 32768, 512).astype(np.int16)
    out["int32"] = rng.integers(-2**31, 2**31, 512, dtype=np.int64).astype(np.int32)
    out["int64"] = np.concatenate([rng.integers(-2**63, 2**63 - 1, 509, dtype=np.int64),
                                   np.array([-2**63, 2**63 - 1, 0], np.int64)])

    np.savez_compressed(os.path.join(HERE, "fxp_golden.npz"), **out)

    strs, Eh = hex_cases()
    buf, offs = fxp.pack_hex(strs)
    hex_out = {"buf": buf, "offs": offs, "E": Eh}
    for ftz in (0, 1):
        y, bad = fxp.gmp_decode_hex(strs, Eh, np.float32, ftz)
        assert bad == 0
        hex_out[f"f32_ftz{ftz}"] = y.view(np.uint32)
    y, bad = fxp.gmp_decode_hex(strs, Eh, np.float64)
    hex_out["f64"] = y.view(np.uint64)
    np.savez_compressed(os.path.join(HERE, "fxp_hex_golden.npz"), **hex_out)
    for k, v in sorted(out.items()):
        print(f"{k:18s} {v.dtype} {v.shape}")
    print("hex", len(strs), "strings,", buf.size, "bytes")


if __name__ == "__main__":
    main()
