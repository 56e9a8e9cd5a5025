#!/usr/bin/env python3
"""Drives tools/libmont_probe.so: times S Montgomery squarings mod a 1024-bit odd modulus for N
elements with 32-bit limbs (production sliced.h) and 28-bit lazy limbs (sliced28.h), checks both
against Python's pow(x, 2^S, m), prints one JSON line per variant."""
import ctypes
import json
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libmont_probe.so"))
vp = ctypes.c_void_p
lib.mont_probe.argtypes = [ctypes.c_int, vp, vp, ctypes.c_uint32, vp, vp, ctypes.c_longlong, ctypes.c_int, vp]
L28 = lib.mont_probe_limbs28()
N = int(os.environ.get("MP_N", "262144"))
S = int(os.environ.get("MP_S", "512"))
rng = random.Random(5)
m = rng.getrandbits(1024) | 1 | (1 << 1023)
L32 = 32


def words(v, L, bits=32):
    mask = (1 << bits) - 1
    return np.array([(v >> (bits * k)) & mask for k in range(L)], dtype=np.uint32)


dev = torch.device("cuda")
variants = {
    0: dict(m=words(m, L32), r2=words(pow(2, 2 * 32 * L32, m), L32), minv=(-pow(m, -1, 1 << 32)) % (1 << 32)),
    1: dict(m=words(m, L28, 28), r2=words(pow(2, 2 * 28 * L28, m), L28, 28), minv=(-pow(m, -1, 1 << 28)) % (1 << 28)),
}
xs = [rng.randrange(1, m) for _ in range(N)]
X = torch.from_numpy(np.stack([words(v, L32) for v in xs[:4096]] * (N // 4096)).view(np.int32)).to(dev)
want = {i: pow(xs[i % 4096], 1 << S, m) for i in (0, 1, 2, 4095, N - 1)}
stream = torch.cuda.current_stream().cuda_stream
for v, c in variants.items():
    M = torch.from_numpy(c["m"].view(np.int32)).to(dev)
    R2 = torch.from_numpy(c["r2"].view(np.int32)).to(dev)
    out = torch.zeros_like(X)
    run = lambda: lib.mont_probe(v, M.data_ptr(), R2.data_ptr(), c["minv"], X.data_ptr(), out.data_ptr(), N, S, stream)
    assert run() == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint32)
    ok = all(sum(int(o[i, k]) << (32 * k) for k in range(L32)) == w for i, w in want.items())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        run()
    e1.record()
    e1.synchronize()
    t = e0.elapsed_time(e1) / 3 * 1e-3
    L = L32 if v == 0 else L28
    macs32 = N * (S + 2) * 2 * 1024 * 1024 / 32 / 32        # 32-bit-equivalent MACs of the work
    print(json.dumps({"variant": ["32-bit limbs, carry chain", "28-bit limbs, lazy accumulators"][v],
                      "limbs": L, "elements": N, "squarings": S, "ms": round(t * 1e3, 3),
                      "squarings_per_s": round(N * S / t), "equiv_32bit_TMACs": round(macs32 / t / 1e12, 3),
                      "correct": ok}), flush=True)
