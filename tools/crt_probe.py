#!/usr/bin/env python3
"""The key owner's CRT encryption, kernel by kernel (for rocprofv3 --kernel-trace --stats): for each
Stage-P key, REPS rounds of [sub fbpowm p, sub fbpowm q, efl_pl_crt_join without and with m]
beside the public-key efl_pl_encrypt, same draws (join alone, and join + g(m) product). Prints per-leg HIP-event times as JSON lines.

    python tools/crt_probe.py [--reps 5]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import efl
    from efl.privacy import paillier_cipher as pc
    from bench import STAGE_P_KEYS
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    for label, n_bytes, a_bytes, g, N in STAGE_P_KEYS:
        n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
        kp = efl.paillier.Keypair(seed=7)
        kp.set_keys_ints(n, hs, a_bytes, g, p, q, n_bytes)
        k = kp.key.ensure_table()   # the owner's n^2 table is deferred (KeyBlock)
        subs = k.crt_keys()
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev)
        ct = torch.empty((N, k.lc), dtype=torch.int32, device=dev)
        ct2 = torch.empty_like(ct)
        xs = [torch.empty((N, sk.lc), dtype=torch.int32, device=dev) for sk in subs]
        hsa = torch.empty((N, k.lc), dtype=torch.int32, device=dev)
        legs = {
            "public": lambda: lib.efl_pl_encrypt(*k.args(), m.data_ptr(), None, ct.data_ptr(), N, 7, 0, sh),
            "fbpowm_p": lambda: lib.efl_pl_fbpowm(*subs[0].args(), None, xs[0].data_ptr(), N, 7, 0, sh),
            "fbpowm_q": lambda: lib.efl_pl_fbpowm(*subs[1].args(), None, xs[1].data_ptr(), N, 7, 0, sh),
            "join": lambda: lib.efl_pl_crt_join(*k.args(), xs[0].data_ptr(), xs[1].data_ptr(), None, hsa.data_ptr(), N, sh),
            "join_encrypt": lambda: lib.efl_pl_crt_join(*k.args(), xs[0].data_ptr(), xs[1].data_ptr(), m.data_ptr(),
                                                        ct2.data_ptr(), N, sh),
        }
        out = {"key": label, "elements": N, "ms": {}}
        for name, fn in legs.items():
            efl.lib.check(fn())
        for name, fn in legs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                efl.lib.check(fn())
            e1.record(stream)
            e1.synchronize()
            out["ms"][name] = round(e0.elapsed_time(e1) / args.reps, 3)
        out["bit_identical"] = bool(torch.equal(ct, ct2))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
