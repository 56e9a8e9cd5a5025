#!/usr/bin/env python3
"""Does config 3 lose to config 2 through where its 4 x 4096 small tensors sit in memory? Times the
batched encode and decode (HIP events per launch, medians over interleaved repetitions) over the
same 4096 x 16,384 fp32 slices placed three ways, beside the streaming kernels on one tensor of the
same bytes:
  separate    4 x 4096 torch allocations (the bench's config3: 64 / 128 KiB each, so the caching
              allocator packs them into 2 MiB segments)
  views       the slices are views of four contiguous buffers (embedding slices of one table)
  stream      config 2's streaming kernels over one 64 Mi-element tensor
Run it twice, once with PYTORCH_HIP_ALLOC_CONF=expandable_segments:True, to see the allocator's
segment layout's share. Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402

S, N, REPS, ROUNDS = 4096, 16384, 20, 5
# C3_ARMS="name:enc_block,enc_k,dec_block,dec_k,enc_order,dec_order;..." (efl_fxp_tune 10-13, 17, 18):
# batched launch shapes to time on both layouts; default: the library's own
ARMS = [a for a in os.environ.get("C3_ARMS", "").split(";") if a]


def main():
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    g = torch.Generator(device=dev).manual_seed(1)
    sh = torch.cuda.current_stream().cuda_stream
    st = torch.cuda.current_stream()
    sep = ([torch.randn(128, 128, device=dev, generator=g) * 0.01 for _ in range(S)],
           [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)],
           [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)],
           [torch.empty(128, 128, device=dev) for _ in range(S)])
    big = (torch.randn(S, 128, 128, device=dev, generator=g) * 0.01,
           torch.empty(S, 128, 128, dtype=torch.int64, device=dev),
           torch.empty(S, 128, 128, dtype=torch.int64, device=dev),
           torch.empty(S, 128, 128, device=dev))
    views = tuple([b[i] for i in range(S)] for b in big)
    tables = {name: (efl.lib.BatchTables(t[0], t[1], t[2]), efl.lib.BatchTables(t[1], t[2], t[3]))
              for name, t in (("separate", sep), ("views", views))}
    x, M, E, y = (b.reshape(-1) for b in big)

    def batched(name):
        enc_t, dec_t = tables[name]
        return (lambda: efl.lib.encode_batched_into(enc_t, 1, False, sh),
                lambda: efl.lib.decode_batched_into(dec_t, 1, 1, sh))

    stream = (lambda: efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), S * N, 0, sh)),
              lambda: efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, S * N, S * N, 1, sh)))
    arms = {"separate": batched("separate"), "views": batched("views"), "stream": stream}
    shapes = {"default": None}
    for a in ARMS:
        name, vals = a.split(":")
        shapes[name] = [int(v) for v in vals.split(",")]

    def tuned(shape, fn):
        def run():
            if shape is None:
                return fn()
            old = [lib.efl_fxp_tune(kind, v) for kind, v in zip((10, 11, 12, 13, 17, 18), shape)]
            try:
                return fn()
            finally:
                for kind, v in zip((10, 11, 12, 13, 17, 18), old):
                    lib.efl_fxp_tune(kind, v)
        return run
    arms = {"stream": stream}
    for sname, shape in shapes.items():
        for lay in ("separate", "views"):
            enc, dec = batched(lay)
            key = lay if sname == "default" else f"{lay}/{sname}"
            arms[key] = (tuned(shape, enc), tuned(shape, dec))
    res = {k: {"encode": [], "decode": []} for k in arms}
    for enc, dec in arms.values():
        for _ in range(3):
            enc()
            dec()
    torch.cuda.synchronize()
    for _ in range(ROUNDS):
        for name, (enc, dec) in arms.items():
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(REPS)]
            for e in ev:
                e[0].record(st)
                enc()
                e[1].record(st)
                dec()
                e[2].record(st)
            torch.cuda.synchronize()
            res[name]["encode"] += [e[0].elapsed_time(e[1]) for e in ev]
            res[name]["decode"] += [e[1].elapsed_time(e[2]) for e in ev]
    ok = all(torch.equal(a, b) for a, b in zip(sep[0][::97], sep[3][::97])) and \
        all(torch.equal(a, b) for a, b in zip(views[0][::97], views[3][::97]))
    out = {"tool": "config3_layout_probe", "version": efl.lib.version(),
           "alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF", ""), "reps": REPS * ROUNDS, "roundtrip_ok": ok}
    for name, r in res.items():
        e, d = float(np.median(r["encode"])), float(np.median(r["decode"]))
        out[name] = {"encode_ms": round(e, 4), "decode_ms": round(d, 4),
                     "hbm_frac": round(40 * S * N / ((e + d) * 1e-3) / 8e12, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
