#!/usr/bin/env python3
"""BASELINE config 3: a batch of 4096 x 64 KiB fp32 embedding slices (16,384 elements each,
N(0, 0.01), seed 1) on one MI355X. Encrypt+decrypt of the whole batch as ONE batched launch per
direction (device pointer/length tables) vs the naive per-slice launches. Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402

SLICES, ELEMS = 4096, 16384
dev = efl.lib.require_gpu()
lib = efl.lib.raw()
if os.environ.get("EFL_BATCH_ENC_NT"):   # A/B of the batched encode's store flags (efl_fxp_tune 9)
    lib.efl_fxp_tune(9, int(os.environ["EFL_BATCH_ENC_NT"]))
g = torch.Generator(device=dev).manual_seed(1)
# separate allocations per slice (realistic: embedding rows live in different tensors)
xs = [torch.randn(128, 128, device=dev, generator=g) * 0.01 for _ in range(SLICES)]
Ms = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(SLICES)]
Es = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(SLICES)]
ys = [torch.empty(128, 128, device=dev) for _ in range(SLICES)]
enc_t = efl.lib.BatchTables(xs, Ms, Es)
dec_t = efl.lib.BatchTables(Ms, Es, ys)
s = torch.cuda.current_stream()
sh = s.cuda_stream


def batched():
    efl.lib.encode_batched_into(enc_t, 1, False, sh)
    efl.lib.decode_batched_into(dec_t, 1, 0, sh)


def naive():
    for x, M, E, y in zip(xs, Ms, Es, ys):
        lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), ELEMS, 0, sh)
    for x, M, E, y in zip(xs, Ms, Es, ys):
        lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, ELEMS, ELEMS, 0, sh)


def timeit(fn, steps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(steps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, e0.elapsed_time(e1) / steps


batched()
torch.cuda.synchronize()
for x, y in zip(xs[:64], ys[:64]):
    nz = x != 0
    assert torch.equal(y[nz], x[nz])
wall_b, dev_b = timeit(batched)
wall_n, dev_n = timeit(naive, 5)
nbytes = SLICES * ELEMS * 4
print(json.dumps({
    "config": "config 3: 4096 x 64 KiB fp32 slices, batched encode+decode",
    "batched_ms": round(wall_b, 4), "batched_GiBs": round(nbytes / 2**30 / (wall_b * 1e-3), 2),
    "batched_hbm_frac": round(40 * SLICES * ELEMS / (wall_b * 1e-3) / 8e12, 4),
    "naive_per_slice_ms": round(wall_n, 3), "naive_GiBs": round(nbytes / 2**30 / (wall_n * 1e-3), 2),
    "launches_naive": 2 * SLICES, "launches_batched": 2}))
