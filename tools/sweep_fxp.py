#!/usr/bin/env python3
"""Stage-F launch-shape sweep on the bench workload (256 MiB fp32), interleaved rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24). Each direction is swept with the other at its
default. Prints per-shape median/min kernel time and achieved algorithmic GB/s (20 B/element).
efl_fxp_tune kind = 2*field + dir: field 0 layout, 1 K, 2 NT mask, 3 block; kind 8 grid cap."""
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
# the library's defaults (csrc/fxp.hip g_shape): read back by setting, then restored below
_DEF = {0: ((0, 0), (1, 1), (2, 7), (3, 256)), 1: ((0, 0), (1, 1), (2, 1), (3, 128))}
DEFAULT = {d: {f: lib.efl_fxp_tune(2 * f + d, v) for f, v in _DEF[d]} for d in (0, 1)}
for d in (0, 1):
    for f, v in DEFAULT[d].items():
        lib.efl_fxp_tune(2 * f + d, v)
LAYOUTS = [int(v) for v in os.environ.get("SWEEP_LAYOUTS", "0,1").split(",")]
NTS = [int(v) for v in os.environ.get("SWEEP_NT", "0,1,2,3").split(",")]
DIRS = [{"encode": 0, "decode": 1}[d] for d in os.environ.get("SWEEP_DIRS", "encode,decode").split(",")]
shapes = [dict(layout=l, K=k, nt=t, block=b) for l, k, t, b in
          itertools.product(LAYOUTS, (1, 2), NTS, (128, 256, 512))]
rounds = int(os.environ.get("SWEEP_ROUNDS", "4"))
reps = 3


def apply(d, shp):
    for f, key in ((0, "layout"), (1, "K"), (2, "nt"), (3, "block")):
        assert lib.efl_fxp_tune(2 * f + d, shp[key]) >= 0


def restore(d):
    for f, v in DEFAULT[d].items():
        lib.efl_fxp_tune(2 * f + d, v)


ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
res = {(d, i): [] for d in DIRS for i in range(len(shapes))}
for r in range(rounds):
    for d in DIRS:
        for i, shp in enumerate(shapes):
            apply(d, shp)
            for j in range(reps + 1):
                ev[0].record(s)
                efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), n, 0, sh))
                ev[1].record(s)
                efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, n, n, 0, sh))
                ev[2].record(s)
                torch.cuda.synchronize()
                if j:
                    res[(d, i)].append(ev[d].elapsed_time(ev[d + 1]))
            restore(d)
    nz = x != 0
    assert torch.equal(y[nz], x[nz])

out = []
for (d, i), t in res.items():
    t = np.array(t)
    out.append(dict(dir="encode" if d == 0 else "decode", **shapes[i], med_ms=float(np.median(t)),
                    min_ms=float(t.min()), GBs=20 * n / (np.median(t) * 1e-3) / 1e9))
out.sort(key=lambda r: (r["dir"], r["med_ms"]))
for r in out:
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))
