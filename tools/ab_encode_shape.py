#!/usr/bin/env python3
"""A/B of the encode launch shape inside the bench step (encode then decode, back to back, no sync
between steps), interleaved rounds in one process so box and clock drift land on both arms.
Arm "old": 128 lanes, nontemporal loads, plain stores. Arm "nt": 256 lanes, nontemporal loads and
stores. Arm "new" (the default): 256 lanes, nontemporal loads, `nt sc1` stores. Prints one JSON line: median step ms and per-kernel ms per arm."""
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
# arm = (encode block, encode NT mask, decode block, decode NT mask); AB_ARMS="name:b,nt,b,nt;..."
ARMS = {"old": (128, 1, 128, 1), "nt": (256, 3, 128, 1), "new": (256, 7, 128, 1)}
if os.environ.get("AB_ARMS"):
    ARMS = {a.split(":")[0]: tuple(int(v) for v in a.split(":")[1].split(","))
            for a in os.environ["AB_ARMS"].split(";")}
STEPS = 20


def arm(name):
    eb, ent, db, dnt = ARMS[name]
    lib.efl_fxp_tune(6, eb)    # kind 2*field + dir: field 3 block, field 2 NT mask
    lib.efl_fxp_tune(4, ent)
    lib.efl_fxp_tune(7, db)
    lib.efl_fxp_tune(5, dnt)


res = {a: {"step": [], "enc": [], "dec": []} for a in ARMS}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * STEPS + 1)]
for r in range(12):
    for a in ARMS:
        arm(a)
        for _ in range(3):
            lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), n, 0, sh)
            lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, n, n, 0, sh)
        torch.cuda.synchronize()
        ev[0].record(s)
        for i in range(STEPS):
            efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), n, 0, sh))
            ev[2 * i + 1].record(s)
            efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, n, n, 0, sh))
            ev[2 * i + 2].record(s)
        torch.cuda.synchronize()
        if r < 2:
            continue
        res[a]["step"].append(ev[0].elapsed_time(ev[-1]) / STEPS)
        res[a]["enc"] += [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(STEPS)]
        res[a]["dec"] += [ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(STEPS)]
nz = x != 0
assert torch.equal(y[nz], x[nz])
out = {a: {k: round(float(np.median(v)), 4) for k, v in d.items()} for a, d in res.items()}
for a in out:
    out[a]["step_frac_of_8TBs"] = round(40 * n / (out[a]["step"] * 1e-3) / 8e12, 4)
print(json.dumps({"elements": n, "steps_per_round": STEPS, "rounds": 10, "arms": ARMS, **out}))
