#!/usr/bin/env python3
"""Stage-F kernel variant sweep on the bench workload (256 MiB fp32), interleaved rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24). Prints per-variant median/min kernel times and the
achieved algorithmic GB/s. Knobs: efl_fxp_tune kinds 0 enc variant, 1 dec variant, 2 K, 3 grid
cap, 4 NT mode."""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402

dev = efl.lib.require_gpu()
lib = efl.lib.raw()
n = 65536 * 1024
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
M = torch.empty(n, dtype=torch.int64, device=dev)
E = torch.empty(n, dtype=torch.int64, device=dev)
y = torch.empty_like(x)
s = torch.cuda.current_stream()
sh = s.cuda_stream

variants = []
for var, K, cap, nt in itertools.product((0, 1), (1, 2, 4), (0, 2048), (0, 2, 3)):
    variants.append({"var": var, "K": K, "cap": cap, "nt": nt})
rounds = int(os.environ.get("SWEEP_ROUNDS", "5"))
reps = 4
res = {i: {"enc": [], "dec": []} for i in range(len(variants))}


def setv(v):
    for kind, val in ((0, v["var"]), (1, v["var"]), (2, v["K"]), (3, v["cap"]), (4, v["nt"])):
        assert lib.efl_fxp_tune(kind, val) >= 0


ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
for r in range(rounds):
    for i, v in enumerate(variants):
        setv(v)
        for _ in range(reps + 1):
            ev[0].record(s)
            efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), n, 0, sh))
            ev[1].record(s)
            efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, n, n, 0, sh))
            ev[2].record(s)
            torch.cuda.synchronize()
            if _ == 0:
                continue   # first launch after a switch: warm
            res[i]["enc"].append(ev[0].elapsed_time(ev[1]))
            res[i]["dec"].append(ev[1].elapsed_time(ev[2]))
    nz = x != 0
    assert torch.equal(y[nz], x[nz])

rows = []
for i, v in enumerate(variants):
    e, d = np.array(res[i]["enc"]), np.array(res[i]["dec"])
    rows.append(dict(v, enc_med=float(np.median(e)), enc_min=float(e.min()),
                     dec_med=float(np.median(d)), dec_min=float(d.min()),
                     enc_GBs=20 * n / (np.median(e) * 1e-3) / 1e9,
                     dec_GBs=20 * n / (np.median(d) * 1e-3) / 1e9))
rows.sort(key=lambda r: r["enc_med"] + r["dec_med"])
for r in rows:
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))
