#!/usr/bin/env python3
"""Same-process A/B of Stage-F library builds (each .so loaded with its own ctypes handle, so the
kernels of every build run on the same box, interleaved): per build, the streaming encode / decode
of the bench's config-2 tensor (64 Mi fp32) and the batched encode / decode of config 3 (4096 x
16,384 fp32 in separate allocations), each launch timed with HIP events on the launch stream,
medians over ROUNDS x REPS interleaved repetitions. The round trip of every build is checked bit
for bit. Prints one JSON line.

    python tools/ab_fxp_libs.py name=path.so [name=path.so ...]
"""
import ctypes
import json
import sys

import numpy as np
import torch

ROUNDS, REPS = 7, 20
S, N = 4096, 16384
BIG = 65536 * 1024


def load(path):
    L = ctypes.CDLL(path)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    L.efl_version.restype = ctypes.c_char_p
    L.efl_fxp_encode.argtypes = [vp, i32, vp, vp, i64, i32, vp]
    L.efl_fxp_decode.argtypes = [vp, vp, vp, i32, i64, i64, i32, vp]
    L.efl_fxp_encode_batched.argtypes = [vp, i32, vp, vp, vp, i64, i64, i32, vp]
    L.efl_fxp_decode_batched.argtypes = [vp, vp, vp, i32, vp, i64, i64, i32, vp]
    for f in ("efl_fxp_encode", "efl_fxp_decode", "efl_fxp_encode_batched", "efl_fxp_decode_batched"):
        getattr(L, f).restype = i32
    return L


def main():
    libs = {a.split("=", 1)[0]: load(a.split("=", 1)[1]) for a in sys.argv[1:]}
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(BIG, device=dev, generator=g)
    M = torch.empty(BIG, dtype=torch.int64, device=dev)
    E = torch.empty_like(M)
    y = torch.empty_like(x)
    xs = [torch.randn(128, 128, device=dev, generator=g) * 0.01 for _ in range(S)]
    Ms = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)]
    Es = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)]
    ys = [torch.empty(128, 128, device=dev) for _ in range(S)]

    def table(ts):
        return torch.tensor([t.data_ptr() for t in ts], dtype=torch.int64, device=dev)
    tx, tM, tE, ty = table(xs), table(Ms), table(Es), table(ys)
    ns = torch.full((S,), N, dtype=torch.int64, device=dev)

    def ops(L):
        def s_enc():
            assert L.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), BIG, 0, sh) == 0

        def s_dec():
            assert L.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, BIG, BIG, 1, sh) == 0

        def b_enc():
            assert L.efl_fxp_encode_batched(tx.data_ptr(), 1, tM.data_ptr(), tE.data_ptr(), ns.data_ptr(),
                                            S, N, 0, sh) == 0

        def b_dec():
            assert L.efl_fxp_decode_batched(tM.data_ptr(), tE.data_ptr(), ty.data_ptr(), 1, ns.data_ptr(),
                                            S, N, 1, sh) == 0
        return {"stream": (s_enc, s_dec), "batched": (b_enc, b_dec)}
    arms = {name: ops(L) for name, L in libs.items()}
    res = {name: {w: {"encode": [], "decode": []} for w in ("stream", "batched")} for name in libs}
    ok = {}
    for name, a in arms.items():
        y.zero_()
        for t in ys:
            t.zero_()
        for w in ("stream", "batched"):
            for _ in range(3):
                a[w][0]()
                a[w][1]()
        torch.cuda.synchronize()
        ok[name] = bool(torch.equal(x.view(torch.int32), y.view(torch.int32))) and \
            bool(torch.equal(torch.stack(xs).view(torch.int32), torch.stack(ys).view(torch.int32)))
    for _ in range(ROUNDS):
        for name, a in arms.items():
            for w in ("stream", "batched"):
                enc, dec = a[w]
                ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(REPS)]
                for e in ev:
                    e[0].record(st)
                    enc()
                    e[1].record(st)
                    dec()
                    e[2].record(st)
                torch.cuda.synchronize()
                res[name][w]["encode"] += [e[0].elapsed_time(e[1]) for e in ev]
                res[name][w]["decode"] += [e[1].elapsed_time(e[2]) for e in ev]
    out = {"tool": "ab_fxp_libs", "rounds": ROUNDS, "reps": REPS,
           "versions": {n: L.efl_version().decode() for n, L in libs.items()}, "roundtrip_ok": ok}
    kb = 20 * BIG
    for name in libs:
        for w in ("stream", "batched"):
            e = float(np.median(res[name][w]["encode"]))
            d = float(np.median(res[name][w]["decode"]))
            out[f"{name}/{w}"] = {"encode_ms": round(e, 4), "decode_ms": round(d, 4),
                                  "encode_frac": round(kb / (e * 1e-3) / 8e12, 4),
                                  "decode_frac": round(kb / (d * 1e-3) / 8e12, 4),
                                  "step_frac": round(2 * kb / ((e + d) * 1e-3) / 8e12, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
