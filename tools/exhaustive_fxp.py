#!/usr/bin/env python3
"""Exhaustive fp32 parity of the Stage-F kernels: every one of the 2^32 fp32 bit patterns, both
decrease_precision values, both decode rounding modes.

For each 2^26-pattern chunk the GPU side (libefl_hip.so: efl_fxp_encode, efl_fxp_decode with and
without FTZ) and the CPU side (oracle/fxp_gmp.c exhaustive_hash_f32: the reference's encode loop
body restated statement for statement, fixed_point.cc:107-137, then GMP 6.2.1's mpf decode in the
reference's call order, fixed_point.cc:238-245, under the default MXCSR and under FTZ|DAZ) each
reduce their outputs to three position-weighted sums mod 2^64 (mantissa/exponent, decoded bits
per mode). Equal sums for every chunk = the GPU equals the reference loop + GMP on all 2^32 inputs
(a differing element changes its chunk's sum unless the difference is a multiple of 2^64 / w,
which an odd weight w excludes). Prints one JSON line.

    python tools/exhaustive_fxp.py [--chunk-log2 26] [--threads N] [--limit CHUNKS]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402

K1, K2, K3 = 0x9E3779B97F4A7C15, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9
MASK = (1 << 64) - 1


def s64(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def gpu_hash(efl, start, count, dp, dev):
    i = torch.arange(start, start + count, dtype=torch.int64, device=dev)
    v = torch.where(i >= 1 << 31, i - (1 << 32), i).to(torch.int32)
    x = v.view(torch.float32)
    M, E = efl.lib.convert_to_fixed_point(x, decrease_precision=bool(dp))
    w = 2 * i + 1
    h = [int(((M * s64(K1) + E * s64(K2)) * w).sum().item()) & MASK]
    for ftz in (False, True):
        y = efl.lib.fixed_point_to_float_point(M, E, torch.float32, flush_denormal=ftz)
        yb = y.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        h.append(int((yb * s64(K3) * w).sum().item()) & MASK)
    return h


def cpu_hash(start, count, dp, threads):
    from oracle import fxp
    L = fxp.lib()
    L.exhaustive_hash_f32.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_uint64)]
    out = (ctypes.c_uint64 * 3)()
    L.exhaustive_hash_f32(start & 0xFFFFFFFF, count, dp, threads, out)
    return [int(v) for v in out]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk-log2", type=int, default=26)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--limit", type=int, default=None, help="first N chunks only (smoke)")
    args = ap.parse_args()
    import efl
    sys.path.insert(0, ROOT)
    from bench import usable_cores
    threads = args.threads or usable_cores()[0]
    dev = efl.lib.require_gpu()
    chunk = 1 << args.chunk_log2
    nchunks = (1 << 32) // chunk
    if args.limit:
        nchunks = min(nchunks, args.limit)
    t0 = time.time()
    bad = []
    t_gpu = t_cpu = 0.0
    for dp in (0, 1):
        for c in range(nchunks):
            start = c * chunk
            a = time.time()
            g = gpu_hash(efl, start, chunk, dp, dev)
            torch.cuda.synchronize()
            b = time.time()
            h = cpu_hash(start, chunk, dp, threads)
            t_gpu += b - a
            t_cpu += time.time() - b
            if g != h:
                bad.append({"dp": dp, "start": hex(start),
                            "which": [k for k, (x, y) in enumerate(zip(g, h)) if x != y]})
            if c % 8 == 7:
                print(f"dp {dp} chunk {c + 1}/{nchunks} mismatches {len(bad)} {time.time() - t0:.0f}s",
                      file=sys.stderr, flush=True)
    print(json.dumps({"tool": "exhaustive_fxp", "library": efl.lib.version(),
                      "patterns": nchunks * chunk, "of": 1 << 32, "decrease_precision": [0, 1],
                      "decode_modes": ["bare loop (MXCSR default)", "FTZ|DAZ (TF threadpool)"],
                      "cpu_side": "literal encode loop (fixed_point.cc:107-137) + GMP mpf decode (:238-245)",
                      "mismatched_chunks": bad, "all_equal": not bad, "threads": threads,
                      "gpu_s": round(t_gpu, 1), "cpu_s": round(t_cpu, 1), "wall_s": round(time.time() - t0, 1)}),
          flush=True)
    return 0 if not bad else 1


if __name__ == "__main__":
    sys.exit(main())
