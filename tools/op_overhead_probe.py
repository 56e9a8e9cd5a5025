#!/usr/bin/env python3
"""Where the Paillier layer's op time goes outside the kernels: wall time per call (device
synchronised on both sides) against HIP-event time of the same call, for the ops and sizes of the
paillier_mnist dense step (1024-bit key): decrypt of [256, 392], [392, 128] and [256, 128], the
[256, 392] x [392, 128] matmul and the [256, 392] encrypt. Each op runs twice: with the HIP default
memory pool's release threshold at its default (0: stream-ordered scratch is unmapped at every
synchronisation) and at 2^63 (kept mapped), so the cost of re-mapping the ops' stream-ordered
scratch slabs shows up as the difference.

    python tools/op_overhead_probe.py > out.jsonl
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402

import efl  # noqa: E402

REPS = int(os.environ.get("PROBE_REPS", "5"))
dev = efl.lib.require_gpu()
with open(os.path.join(ROOT, "tests", "golden", "paillier_kat.json")) as f:
    K = {k["n_bytes"]: k for k in json.load(f)["keys"]}[128]
kp = efl.paillier.Keypair(seed=5)
kp.set_keys_ints(int(K["n"], 16), int(K["hs"], 16), K["a_bits"] // 8, 10, int(K["p"], 16), int(K["q"], 16))
g = torch.Generator(device=dev).manual_seed(1)

hip = ctypes.CDLL("libamdhip64.so")


def set_release_threshold(v):
    pool = ctypes.c_void_p()
    assert hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), ctypes.c_int(dev.index or 0)) == 0
    val = ctypes.c_uint64(v)
    assert hip.hipMemPoolSetAttribute(pool, ctypes.c_int(4), ctypes.byref(val)) == 0   # ReleaseThreshold


def measure(name, fn):
    fn()
    torch.cuda.synchronize()
    walls, gpus = [], []
    s = torch.cuda.current_stream()
    for _ in range(REPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        gpus.append(e0.elapsed_time(e1))
    walls.sort()
    gpus.sort()
    return {"op": name, "wall_ms": round(walls[len(walls) // 2], 3), "event_ms": round(gpus[len(gpus) // 2], 3)}


cts = {}
for shape in ((256, 392), (392, 128), (256, 128)):
    m = torch.randint(-2**40, 2**40, shape, dtype=torch.int64, device=dev, generator=g)
    cts[shape] = (kp.encrypt(m), m)
x = cts[(256, 392)][0]
xe = torch.randint(-30, -20, (256, 392), dtype=torch.int64, device=dev, generator=g)
wm = torch.randint(-2**10, 2**10, (392, 128), dtype=torch.int64, device=dev, generator=g)
we = torch.randint(-14, -10, (392, 128), dtype=torch.int64, device=dev, generator=g)
m_enc = torch.randint(-2**40, 2**40, (256, 392), dtype=torch.int64, device=dev, generator=g)

for thr, tag in ((0, "release_threshold_0"), (1 << 63, "release_threshold_max")):
    set_release_threshold(thr)
    for shape, (c, m) in cts.items():
        line = measure(f"decrypt {list(shape)}", lambda c=c: kp.decrypt(c, dtype=torch.int64))
        print(json.dumps({"pool": tag, **line}), flush=True)
    line = measure("matmul [256,392]x[392,128]", lambda: kp.matmul(x.tensor, xe, wm, we))
    print(json.dumps({"pool": tag, **line}), flush=True)
    line = measure("encrypt [256,392]", lambda: kp.encrypt(m_enc))
    print(json.dumps({"pool": tag, **line}), flush=True)
set_release_threshold(0)
print(json.dumps({"tool": "op_overhead_probe", "version": efl.lib.version(), "reps": REPS}), flush=True)
