#!/usr/bin/env python3
"""Kernel-family sweep of Paillier fresh-randomness encryption with the round-2 table window: for
each n^2 family (limbs per lane C; 0 = one lane per element) the key block (and its radix-2^28 table
for that family) is rebuilt, then N encryptions are timed with HIP events. One JSON line per key."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402
from efl.privacy import paillier_cipher as pc  # noqa: E402

dev = efl.lib.require_gpu()
lib = efl.lib.raw()
s = torch.cuda.current_stream()
sh = s.cuda_stream
KEYS = ((64, 32, 1, 262144, (0, 8, 16, 32)), (128, 64, 10, 262144, (0, 8, 16, 32)),
        (256, 128, 1, 131072, (0, 8, 16, 32)), (512, 256, 1, 65536, (8, 16, 32)))
if os.environ.get("PLFAM_KEYS"):
    KEYS = tuple(k for k in KEYS if str(8 * k[0]) in os.environ["PLFAM_KEYS"].split(","))
if os.environ.get("PLFAM_N"):          # e.g. 100352: the MNIST activation's element count
    KEYS = tuple(k[:3] + (int(os.environ["PLFAM_N"]),) + k[4:] for k in KEYS)
for n_bytes, a_bytes, g, N, fams in KEYS:
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    ln = n_bytes // 4
    out = {"tool": "sweep_pl_family", "n_bits": 8 * n_bytes, "elements": N, "version": efl.lib.version()}
    default = pc.kernel_slicing(ln, False)
    for C in fams:
        pc.set_kernel_slicing(ln, False, C)
        kp = efl.paillier.Keypair(seed=5)
        kp.set_keys_ints(n, hs, a_bytes, g, None, None, n_bytes)
        k = kp.key.ensure_table()   # the owner's n^2 table is deferred (KeyBlock)
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev)
        ct = torch.empty((N, k.lc), dtype=torch.int32, device=dev)

        def enc():
            efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), None, ct.data_ptr(), N, 7, 0, sh))
        enc()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            enc()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[f"C{C}"] = {"ms": round(float(np.median(ts)), 3), "per_s": round(N / (np.median(ts) * 1e-3)),
                        "table28": k.desc.off_table28 >= 0, "W": k.table_window}
        if n_bytes == 128:
            # the receiver's MNIST product (bench.py STAGE_P_MATMUL) in this family
            u, v, w = 256, 392, 128
            gen = torch.Generator(device=dev).manual_seed(3)
            xm, xe = efl.lib.convert_to_fixed_point(torch.randn(u, v, device=dev, generator=gen))
            ym, ye = efl.lib.convert_to_fixed_point((torch.rand(v, w, device=dev, generator=gen) - 0.5) * 0.2,
                                                    decrease_precision=True)
            X = torch.empty((u * v, k.lc), dtype=torch.int32, device=dev)
            efl.lib.check(lib.efl_pl_encrypt(*k.args(), xm.data_ptr(), None, X.data_ptr(), u * v, 11, 0, sh))
            zp = torch.empty((u * w, k.lc), dtype=torch.int32, device=dev)
            zn = torch.empty_like(zp)
            ze = torch.empty((u, w), dtype=torch.int64, device=dev)

            def mm():
                efl.lib.check(lib.efl_pl_matmul(*k.args(), X.data_ptr(), xe.data_ptr(), ym.data_ptr(), ye.data_ptr(),
                                                zp.data_ptr(), zn.data_ptr(), ze.data_ptr(), u, v, w, sh))
            mm()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            mm()
            mm()
            e1.record(s)
            e1.synchronize()
            out[f"C{C}"]["matmul_ms"] = round(e0.elapsed_time(e1) / 2, 3)
        del kp, k, ct
        torch.cuda.empty_cache()
    pc.set_kernel_slicing(ln, False, default)
    out["default"] = default
    print(json.dumps(out), flush=True)
