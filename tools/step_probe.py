#!/usr/bin/env python3
"""Where does the bench step's time go? Interleaved arms of the config-2 step (256 MiB fp32:
encode then decode, back to back), one process, rounds alternating so box drift lands on every arm.

Arms (env STEP_ARMS="name:enc_block,enc_nt,enc_k,dec_block,dec_nt,dec_k[,graph];..." overrides):
  base      the library defaults, plain stream loop, wall clock only (what bench.py times)
  events    the same with two HIP events per step (the round-1 bench's timed loop)
  graph     the default step captured once as a hipGraph of 10 steps and replayed
  dec_nt7   decode with `nt sc1` stores (its output then leaves no dirty lines in the XCD L2s)
  enc_k2    encode with 2 units per lane per tile
  enc_b512  encode with 512-lane workgroups
Prints one JSON line: per arm the median wall ms per step and (events arm) per-kernel ms.
"""
import json
import os
import sys
import time

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
FLAGS = int(os.environ.get("STEP_DEC_FLAGS", "1"))

# (enc block, enc NT, enc K, dec block, dec NT, dec K, mode)
DEFAULT = (512, 7, 1, 128, 1, 1)
ARMS = {"base": DEFAULT + ("loop",), "events": DEFAULT + ("events",), "graph": DEFAULT + ("graph",),
        "dec_nt7": (256, 7, 1, 128, 7, 1, "loop"), "enc_k2": (256, 7, 2, 128, 1, 1, "loop"),
        "enc_b512": (512, 7, 1, 128, 1, 1, "loop")}
if os.environ.get("STEP_ARMS"):
    # name:enc_block,enc_nt,enc_k,dec_block,dec_nt,dec_k[,mode[,xcd_enc,xcd_dec,e_first]]
    ARMS = {}
    for a in os.environ["STEP_ARMS"].split(";"):
        name, spec = a.split(":")
        parts = spec.split(",")
        extra = tuple(int(v) for v in parts[7:10]) if len(parts) > 7 else (0, 0, 0)
        ARMS[name] = tuple(int(v) for v in parts[:6]) + ((parts[6] if len(parts) > 6 else "loop"),) + extra
STEPS = int(os.environ.get("STEP_STEPS", "50"))
ROUNDS = int(os.environ.get("STEP_ROUNDS", "8"))


def configure(arm):
    eb, ent, ek, db, dnt, dk = arm[:6]
    xe, xd, ef = arm[7:10] if len(arm) > 7 else (0, 0, 0)
    for kind, v in ((6, eb), (4, ent), (2, ek), (7, db), (5, dnt), (3, dk), (14, xe), (15, xd), (16, ef)):
        efl.lib.check(min(0, lib.efl_fxp_tune(kind, v)))


def step(sh):
    efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), n, 0, sh))
    efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, n, n, FLAGS, sh))


graphs = {}


def graph_for(name):
    if name not in graphs:
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step(side.cuda_stream)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            sh = torch.cuda.current_stream().cuda_stream
            for _ in range(10):
                step(sh)
        graphs[name] = g
    return graphs[name]


res = {a: {"wall": [], "enc": [], "dec": []} for a in ARMS}
s = torch.cuda.current_stream()
sh = s.cuda_stream
for r in range(ROUNDS):
    for name, arm in ARMS.items():
        configure(arm)
        mode = arm[6]
        for _ in range(3):
            step(sh)
        if mode == "graph":
            g = graph_for(name)
            g.replay()
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
                torch.cuda.Event(enable_timing=True)) for _ in range(STEPS)] if mode == "events" else None
        t0 = time.perf_counter()
        if mode == "graph":
            for _ in range(STEPS // 10):
                g.replay()
        elif mode == "events":
            for k in range(STEPS):
                evs[k][0].record(s)
                efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), n, 0, sh))
                evs[k][1].record(s)
                efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, n, n, FLAGS, sh))
                evs[k][2].record(s)
        else:
            for _ in range(STEPS):
                step(sh)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / (STEPS // 10 * 10 if mode == "graph" else STEPS) * 1e3
        if r == 0:
            continue
        res[name]["wall"].append(wall)
        if evs:
            res[name]["enc"] += [e[0].elapsed_time(e[1]) for e in evs]
            res[name]["dec"] += [e[1].elapsed_time(e[2]) for e in evs]
nz = x != 0
configure(DEFAULT + ("loop",))
step(sh)
torch.cuda.synchronize()
ok = bool(torch.equal(y[nz], x[nz]))
out = {}
for a, d in res.items():
    o = {k: round(float(np.median(v)), 4) for k, v in d.items() if v}
    o["GiBs"] = round(n * 4 / 2 ** 30 / (o["wall"] * 1e-3), 1)
    o["step_frac_of_8TBs"] = round(40 * n / (o["wall"] * 1e-3) / 8e12, 4)
    out[a] = o
print(json.dumps({"tool": "step_probe", "version": efl.lib.version(), "elements": n, "steps": STEPS,
                  "rounds": ROUNDS - 1, "dec_flags": FLAGS, "roundtrip_ok": ok,
                  "arms": {a: list(v) for a, v in ARMS.items()}, **out}), flush=True)
