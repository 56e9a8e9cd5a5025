#!/usr/bin/env python3
"""BASELINE config 3 beside config 2 for profiling: `--reps` steps of the batched encode + decode over
4096 separate 64 KiB fp32 slices (the bench's config3) at each batched tile shape in --shapes (the
shipped default first; the encode's K is in the kernel's name, k_batched<EncF32Pair, 512, K, 7>, so
a rocprofv3 pass tells the arms apart), then the same number of streaming steps over one 64 Mi-element
tensor (the same bytes). Meant to run under rocprofv3 (kernel trace, or one PMC pass: FETCH_SIZE /
WRITE_SIZE / TCP_UTCL1_* / TA_* / TD_* counters) so the batched and streaming kernels of one run can
be compared per launch. Prints one JSON line (the round trips are checked)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402

import efl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--order", type=int, nargs=2, default=None, help="efl_fxp_tune 17 / 18 (batched tile order)")
    ap.add_argument("--shapes", default="default;512,2,512,2",
                    help="';'-separated batched shapes: 'default' or enc_block,enc_k,dec_block,dec_k[,enc_order,dec_order"
                         "[,enc_tiles,dec_tiles]] (tune 10-13, 17-18, 26-27)")
    a = ap.parse_args()
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    if a.order:
        lib.efl_fxp_tune(17, a.order[0])
        lib.efl_fxp_tune(18, a.order[1])
    S, N = 4096, 16384
    g = torch.Generator(device=dev).manual_seed(1)
    # 4 x 4096 separate allocations as the bench makes them, filled with a few multi-tensor launches
    # (not 8192 single ones: under a --pmc pass every dispatch is serialised)
    xs = [torch.empty(128, 128, device=dev) for _ in range(S)]
    torch._foreach_copy_(xs, list((torch.randn(S, 128, 128, device=dev, generator=g) * 0.01).unbind(0)))
    Ms = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)]
    Es = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)]
    ys = [torch.empty(128, 128, device=dev) for _ in range(S)]
    enc_t, dec_t = efl.lib.BatchTables(xs, Ms, Es), efl.lib.BatchTables(Ms, Es, ys)
    sh = torch.cuda.current_stream().cuda_stream

    def wall(fn, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    def batched():
        efl.lib.encode_batched_into(enc_t, 1, False, sh)
        efl.lib.decode_batched_into(dec_t, 1, 1, sh)
    arms = {}
    for spec in filter(None, a.shapes.split(";")):
        shape = None if spec == "default" else [int(v) for v in spec.split(",")]
        old = None
        if shape:
            kinds = (10, 11, 12, 13, 17, 18, 26, 27)[:len(shape)]
            old = [lib.efl_fxp_tune(kind, v) for kind, v in zip(kinds, shape)]
            efl.lib.check(min(0, *old))
        torch._foreach_zero_(ys)
        for _ in range(3):
            batched()
        ms = wall(batched, a.reps)
        ok = all(torch.equal(x, y) for x, y in zip(xs[::97], ys[::97]))
        arms[spec] = {"batched_step_ms": round(ms, 4), "roundtrip_ok": ok}
        if old:
            for kind, v in zip(kinds, old):
                lib.efl_fxp_tune(kind, v)
    del Ms, Es, ys, enc_t, dec_t
    x = torch.randn(S * N, device=dev, generator=g)
    M = torch.empty(S * N, dtype=torch.int64, device=dev)
    E = torch.empty_like(M)
    y = torch.empty_like(x)

    def stream():
        efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), S * N, 0, sh))
        efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, S * N, S * N, 1, sh))
    for _ in range(3):
        stream()
    ms_s = wall(stream, a.reps)
    print(json.dumps({"tool": "config3_probe", "version": efl.lib.version(), "reps": a.reps, "arms": arms,
                      "stream_step_ms": round(ms_s, 4),
                      "stream_roundtrip_ok": bool(torch.equal(x, y))}))


if __name__ == "__main__":
    main()
