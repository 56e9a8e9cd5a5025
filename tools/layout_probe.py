#!/usr/bin/env python3
"""Does the relative placement of the encode's two output streams matter? The config-2 encode
writes M[i] and E[i] (two int64 arrays, 512 MiB each) at the same offsets at the same time; if the
HBM address map sends equal offsets of two arrays to the same channel and bank, the two write
streams would fight over rows. This probe carves x, M, E and y out of one allocation with E
shifted by `delta` bytes past the end of M (and y past x), and times encode and decode per delta
with HIP events, rounds interleaved so box drift lands on every arm. One JSON line.
"""
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
DELTAS = [int(v) for v in os.environ.get("LAYOUT_DELTAS", "0,256,4096,65536,1048576,2101248,8392704").split(",")]
STEPS, ROUNDS = 40, 6
maxd = max(DELTAS)
# one slab: x (4n) | y (4n + maxd) | M (8n) | gap maxd | E (8n)
slab = torch.empty(4 * n + 4 * n + maxd + 8 * n + maxd + 8 * n + 4096, dtype=torch.uint8, device=dev)
base = slab.data_ptr()
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
s = torch.cuda.current_stream()
sh = s.cuda_stream


def ptrs(d):
    px = base
    py = px + 4 * n + d
    pm = base + 8 * n + maxd + 4096
    pe = pm + 8 * n + d
    return px, py, pm, pe


res = {d: {"enc": [], "dec": []} for d in DELTAS}
for r in range(ROUNDS):
    for d in DELTAS:
        px, py, pm, pe = ptrs(d)
        slab[: 4 * n].view(torch.float32).copy_(x)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        for _ in range(3):
            efl.lib.check(lib.efl_fxp_encode(px, 1, pm, pe, n, 0, sh))
            efl.lib.check(lib.efl_fxp_decode(pm, pe, py, 1, n, n, 1, sh))
        ev[0].record(s)
        for _ in range(STEPS):
            lib.efl_fxp_encode(px, 1, pm, pe, n, 0, sh)
        ev[1].record(s)
        for _ in range(STEPS):
            lib.efl_fxp_decode(pm, pe, py, 1, n, n, 1, sh)
        ev[2].record(s)
        ev[2].synchronize()
        if r:
            res[d]["enc"].append(ev[0].elapsed_time(ev[1]) / STEPS)
            res[d]["dec"].append(ev[1].elapsed_time(ev[2]) / STEPS)
out = {}
for d, v in res.items():
    e, dc = float(np.median(v["enc"])), float(np.median(v["dec"]))
    out[str(d)] = {"enc_ms": round(e, 4), "dec_ms": round(dc, 4), "enc_frac": round(20 * n / (e * 1e-3) / 8e12, 4),
                   "dec_frac": round(20 * n / (dc * 1e-3) / 8e12, 4)}
print(json.dumps({"tool": "layout_probe", "version": efl.lib.version(), "elements": n, "steps": STEPS,
                  "rounds": ROUNDS - 1, "by_delta_bytes": out}), flush=True)
