#!/usr/bin/env python3
"""Stage P throughput on one MI355X (BASELINE.md §2 'Stage P'): elements/s for encrypt given hsa,
encrypt with fresh randomness (fixed-base table), and CRT decrypt, for every key size and every
kernel family compiled for it (efl_pl_tune: 0 = one lane per element, 16/32 = sliced).
One JSON line per (key, N, family). Kernel-only timing with HIP events on the launch stream.

Env: PL_KEYS "n_bytes:group_size,..." (default 64:1,128:1,128:10,256:1,256:10,512:1),
     PL_N     elements per launch for n < 4096 bits (default 262144), PL_N4096 (default 65536)."""
import json
import os
import random
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
keys = [(int(b), int(g)) for b, g in (x.split(":") for x in
                                       os.environ.get("PL_KEYS", "64:1,128:1,128:10,256:1,256:10,512:1").split(","))]
N_SMALL = int(os.environ.get("PL_N", "262144"))
N_4096 = int(os.environ.get("PL_N4096", "65536"))


def timed(fn, reps=1):
    fn()                                   # warmup (and first-launch code object load)
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / 1e3 / reps


# KAT-free keys: deterministic Miller-Rabin keys per size (host keygen is not on the hot path)
for n_bytes, g in keys:
    t0 = time.perf_counter()
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    kp = efl.paillier.Keypair(seed=7)
    kp.set_keys_ints(n, hs, n_bytes // 2, g, p, q, n_bytes)
    setup = time.perf_counter() - t0
    k = kp.key.ensure_table()   # the owner's n^2 table is deferred (KeyBlock)
    N = N_4096 if k.ln >= 128 else N_SMALL
    m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev)
    out = torch.empty((N, k.lc), dtype=torch.int32, device=dev)
    mag = torch.empty((N, k.ln), dtype=torch.int32, device=dev)
    neg = torch.empty(N, dtype=torch.int8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    fams_enc, fams_dec = pc.SLICINGS[k.ln]
    base_enc, base_dec = pc.kernel_slicing(k.ln, False), pc.kernel_slicing(k.ln, True)
    hsa = kp.fbpowm(n=N).limbs
    for c in fams_enc:
        pc.set_kernel_slicing(k.ln, False, c)
        res = {"n_bits": 8 * n_bytes, "group_size": g, "N": N, "op_family": c, "key_setup_s": round(setup, 2)}
        if g == 1:
            t = timed(lambda: efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), hsa.data_ptr(),
                                                               out.data_ptr(), N, 7, 0, s)), reps=3)
            res["encrypt_given_hsa_per_s"] = round(N / t)
        t = timed(lambda: efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), None, out.data_ptr(),
                                                           N, 7, 0, s)))
        res["encrypt_fresh_per_s"] = round(N / t)
        print(json.dumps(res), flush=True)
    pc.set_kernel_slicing(k.ln, False, base_enc)
    ct = out
    for c in fams_dec:
        pc.set_kernel_slicing(k.ln, True, c)
        t = timed(lambda: efl.lib.check(lib.efl_pl_decrypt(*k.args(), ct.data_ptr(), mag.data_ptr(),
                                                           neg.data_ptr(), N, s)))
        dec = kp.decrypt(pc.CipherTensor(ct[:256], (256,), k), dtype=torch.int64)
        print(json.dumps({"n_bits": 8 * n_bytes, "group_size": g, "N": N, "dec_family": c,
                          "decrypt_per_s": round(N / t), "round_trip_ok": bool(torch.equal(dec, m[:256]))}),
              flush=True)
    pc.set_kernel_slicing(k.ln, True, base_dec)
    del out, mag, neg, hsa
    torch.cuda.empty_cache()
