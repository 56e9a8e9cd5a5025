#!/usr/bin/env python3
"""Workload for measuring what the register spills of the shipping Stage-P kernels cost
(round-2 VERDICT: k_decrypt<32, G>, k_fxp_add28<32, G>, k_matmul28). Runs each op a few times at
the shapes the path uses; meant to run under rocprofv3:

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/spill_probe.py
    rocprofv3 --pmc SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_WAVE_CYCLES SQ_INSTS \\
              -d OUT -- python3 tools/spill_probe.py

Scratch accesses are FLAT instructions (scratch_load / scratch_store), so SQ_ACTIVE_INST_FLAT /
SQ_WAVE_CYCLES bounds the share of wave time the spills can take (global loads and stores are FLAT
too, so the bound includes them). tools/pmc_spill.py reduces the counter CSV per kernel.

Workloads: 1024-bit key (the examples'): decrypt of 262,144 / 100,352 / 32,768 ciphertexts (the
MNIST layer's sizes pick different families), fxp_add (shift + add) of 100,352; 4096-bit key (the
reference default): decrypt of 65,536."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402

import efl  # noqa: E402

REPS = int(os.environ.get("SPILL_REPS", "3"))
dev = efl.lib.require_gpu()
with open(os.path.join(ROOT, "tests", "golden", "paillier_kat.json")) as f:
    KEYS = {k["n_bytes"]: k for k in json.load(f)["keys"]}


def keypair(nb):
    k = KEYS[nb]
    kp = efl.paillier.Keypair(seed=5)
    kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))
    return kp


out = {}
kp = keypair(128)
g = torch.Generator(device=dev).manual_seed(1)
for n in (262144, 100352, 32768):
    m = torch.randint(-2**40, 2**40, (n,), dtype=torch.int64, device=dev, generator=g)
    c = kp.encrypt(m)
    for _ in range(REPS):
        d = kp.decrypt(c, dtype=torch.int64)
    torch.cuda.synchronize()
    out[f"decrypt1024_{n}"] = bool(torch.equal(d, m))
n = 100352
x = kp.encrypt(torch.randint(-2**20, 2**20, (n,), dtype=torch.int64, device=dev, generator=g))
y = kp.encrypt(torch.randint(-2**20, 2**20, (n,), dtype=torch.int64, device=dev, generator=g))
xe = torch.randint(-40, -20, (n,), dtype=torch.int64, device=dev, generator=g)
ye = torch.randint(-40, -20, (n,), dtype=torch.int64, device=dev, generator=g)
for _ in range(REPS):
    z, ze = kp.shift_add(x.tensor, xe, y.tensor, ye)
torch.cuda.synchronize()
kp4 = keypair(512)
n = 65536
m = torch.randint(-2**40, 2**40, (n,), dtype=torch.int64, device=dev, generator=g)
c = kp4.encrypt(m)
for _ in range(REPS):
    d = kp4.decrypt(c, dtype=torch.int64)
torch.cuda.synchronize()
out["decrypt4096_65536"] = bool(torch.equal(d, m))
print(json.dumps({"tool": "spill_probe", "version": efl.lib.version(), "reps": REPS, "ok": out}), flush=True)
