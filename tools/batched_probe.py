#!/usr/bin/env python3
"""Interleaved A/B of the batched fp32 tile shapes (efl_fxp_tune kinds 10-13) on BASELINE config 3:
4096 separate 64 KiB tensors, one batched encode + one batched decode launch per step. Arms =
(enc block, enc K, dec block, dec K); env BATCH_ARMS="name:b,k,b,k;..." overrides. One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402

ARMS = {"256x4": (256, 4, 256, 4), "256x2": (256, 2, 256, 2), "256x1": (256, 1, 256, 1),
        "512x4": (512, 4, 512, 4), "512x2": (512, 2, 512, 2), "512x1": (512, 1, 512, 1)}
# arm = (enc block, enc K, dec block, dec K[, enc order, dec order]); order (efl_fxp_tune 17 / 18):
# 0 2-D grid, 1 flat, 2 flat XCD-aware, 3 persistent (7th field: its workgroups, efl_fxp_tune 19)
if os.environ.get("BATCH_ARMS"):
    ARMS = {a.split(":")[0]: tuple(int(v) for v in a.split(":")[1].split(",")) for a in os.environ["BATCH_ARMS"].split(";")}
dev = efl.lib.require_gpu()
lib = efl.lib.raw()
S, N = 4096, 16384
g = torch.Generator(device=dev).manual_seed(1)
xs = [torch.randn(128, 128, device=dev, generator=g) * 0.01 for _ in range(S)]
Ms = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)]
Es = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(S)]
ys = [torch.empty(128, 128, device=dev) for _ in range(S)]
enc_t, dec_t = efl.lib.BatchTables(xs, Ms, Es), efl.lib.BatchTables(Ms, Es, ys)
sh = torch.cuda.current_stream().cuda_stream


def step():
    efl.lib.encode_batched_into(enc_t, 1, False, sh)
    efl.lib.decode_batched_into(dec_t, 1, 1, sh)


res = {a: [] for a in ARMS}
for r in range(9):
    for a, arm in ARMS.items():
        eb, ek, db, dk = arm[:4]
        oe, od = arm[4:6] if len(arm) >= 6 else (0, 0)
        pg = arm[6] if len(arm) >= 7 else 2048
        for kind, v in ((10, eb), (11, ek), (12, db), (13, dk), (17, oe), (18, od), (19, pg)):
            efl.lib.check(min(0, lib.efl_fxp_tune(kind, v)))
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30):
            step()
        torch.cuda.synchronize()
        if r:
            res[a].append((time.perf_counter() - t0) / 30 * 1e3)
ok = all(torch.equal(x, y) for x, y in zip(xs[::97], ys[::97]))
out = {a: {"ms": round(float(np.median(v)), 4), "GiBs": round(S * N * 4 / 2**30 / (np.median(v) * 1e-3), 1),
           "hbm_frac": round(40 * S * N / (np.median(v) * 1e-3) / 8e12, 4)} for a, v in res.items()}
print(json.dumps({"tool": "batched_probe", "version": efl.lib.version(), "arms": ARMS, "roundtrip_ok": ok, **out}))
