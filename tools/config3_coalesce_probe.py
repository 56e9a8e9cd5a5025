#!/usr/bin/env python3
"""Config 3 with and without run coalescing (efl.lib.coalesce_runs / BatchTables(coalesce=...)).
The same 4096 x 16,384 fp32 slices placed two ways (the bench's 4 x 4096 separate allocations, and
views of four contiguous buffers: embedding slices of one table), batched encode + decode timed with
HIP events per launch (medians over interleaved repetitions), for each of:
  plain        one table entry per slice (round 3's batched path)
  coalesced    adjacent slices merged into runs (one streaming launch when the batch is one run)
and, for each, the fp32 batched tile shapes given in C3_SHAPES="name:enc_block,enc_k,dec_block,dec_k
[,enc_order,dec_order[,enc_tiles,dec_tiles]];..." (efl_fxp_tune 10-13, 17-18, 26-27). C3_LAYOUTS limits the layouts (default
"separate,views"). Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402

S, N, REPS, ROUNDS = 4096, 16384, 20, 5
SHAPES = [a for a in os.environ.get("C3_SHAPES", "k1:512,1,512,1").split(";") if a]


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
    layouts = {k: v for k, v in {"separate": sep, "views": views}.items()
               if k in os.environ.get("C3_LAYOUTS", "separate,views").split(",")}
    tables, runs = {}, {}
    for lay, t in layouts.items():
        for co in (False, True):
            key = f"{lay}/{'coalesced' if co else 'plain'}"
            tables[key] = (efl.lib.BatchTables(t[0], t[1], t[2], coalesce=co),
                           efl.lib.BatchTables(t[1], t[2], t[3], coalesce=co))
            runs[key] = [tables[key][0].count, tables[key][1].count]

    def pair(key):
        enc_t, dec_t = tables[key]
        return (lambda: efl.lib.encode_batched_into(enc_t, 1, False, sh),
                lambda: efl.lib.decode_batched_into(dec_t, 1, 1, sh))

    def tuned(shape, fn):
        def run():
            if shape is None:
                return fn()
            kinds = (10, 11, 12, 13, 17, 18, 26, 27)[:len(shape)]
            old = [lib.efl_fxp_tune(kind, v) for kind, v in zip(kinds, shape)]
            try:
                return fn()
            finally:
                for kind, v in zip(kinds, old):
                    lib.efl_fxp_tune(kind, v)
        return run

    shapes = {"default": None}
    for a in SHAPES:
        name, vals = a.split(":")
        shapes[name] = [int(v) for v in vals.split(",")]
    arms = {}
    for key in tables:
        for sname, shape in shapes.items():
            enc, dec = pair(key)
            arms[key if sname == "default" else f"{key}/{sname}"] = (tuned(shape, enc), tuned(shape, dec))
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
    ok = all(torch.equal(a, b) for t in layouts.values() for a, b in zip(t[0][::97], t[3][::97]))
    out = {"tool": "config3_coalesce_probe", "version": efl.lib.version(), "reps": REPS * ROUNDS,
           "roundtrip_ok": ok, "runs": runs}
    for name, r in res.items():
        e, d = float(np.median(r["encode"])), float(np.median(r["decode"]))
        out[name] = {"encode_ms": round(e, 4), "decode_ms": round(d, 4),
                     "hbm_frac": round(40 * S * N / ((e + d) * 1e-3) / 8e12, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
