#!/usr/bin/env python3
"""Stage P throughput on one MI355X (BASELINE.md §2 'Stage P'): elements/s for encrypt given hsa,
encrypt with fresh randomness (fixed-base table), and CRT decrypt, at N = 262,144 and the MNIST
shape [256, 392], for the key sizes the GPU path supports. One JSON line per (key, op)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import efl  # noqa: E402
from efl.privacy import paillier_cipher as pc  # noqa: E402

dev = efl.lib.require_gpu()
lib = efl.lib.raw()
sizes = [int(s) for s in os.environ.get("PL_SIZES", "262144,100352").split(",")]
keys = [(int(b), int(g)) for b, g in (x.split(":") for x in os.environ.get("PL_KEYS", "64:1,128:1,128:10,256:1").split(","))]


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


import random  # noqa: E402
for n_bytes, g in keys:
    t0 = time.perf_counter()
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    kp = efl.paillier.Keypair(seed=7)
    kp.set_keys_ints(n, hs, n_bytes // 2, g, p, q, n_bytes)
    setup = time.perf_counter() - t0
    k = kp.key
    for N in sizes:
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev)
        out = torch.empty((N, k.lc), dtype=torch.int32, device=dev)
        hsa = kp.fbpowm(n=N).limbs
        s = torch.cuda.current_stream().cuda_stream
        res = {"n_bits": 8 * n_bytes, "group_size": g, "N": N, "key_setup_s": round(setup, 2)}
        if k.ln <= 64:
            t = timed(lambda: efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), hsa.data_ptr(),
                                                               out.data_ptr(), N, 7, 0, s)))
            res["encrypt_given_hsa_per_s"] = round(N / t)
            t = timed(lambda: efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), None, out.data_ptr(),
                                                               N, 7, 0, s)), reps=1)
            res["encrypt_fresh_per_s"] = round(N / t)
        ct = out
        mag = torch.empty((N, k.ln), dtype=torch.int32, device=dev)
        neg = torch.empty(N, dtype=torch.int8, device=dev)
        t = timed(lambda: efl.lib.check(lib.efl_pl_decrypt(*k.args(), ct.data_ptr(), mag.data_ptr(), neg.data_ptr(),
                                                           N, s)), reps=1)
        res["decrypt_per_s"] = round(N / t)
        dec = kp.decrypt(pc.CipherTensor(ct[:64], (64,), k), dtype=torch.int64)
        res["round_trip_ok"] = bool(torch.equal(dec, m[:64]))
        print(json.dumps(res), flush=True)
