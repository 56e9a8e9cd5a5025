"""The key owner's CRT encryption with both walks as one list of waves (efl_pl_tune(16, 5, 0), the
default) against one launch per sub-key (efl_pl_tune(16, 5, 1)), interleaved on one box, at the
element counts the paillier_mnist layers use and around them. 1024-bit key (the examples'), HIP
events on the launch stream. One JSON line per element count.

    python tools/crt_fused_probe.py [--reps 10] [--rounds 3]
"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    pc.table_budget(16 << 30)
    n, hs, p, q = pc.generate_keypair_ints(128, 24, random.Random(128))
    owner = efl.paillier.Keypair(seed=7)
    owner.set_keys_ints(n, hs, 64, 10, p, q, 128)
    s = torch.cuda.current_stream(dev)
    prev = lib.efl_pl_tune(16, 5, -1)
    for N in (4096, 32768, 50176, 100352, 131072, 262144):
        g = torch.Generator(device=dev).manual_seed(N)
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev, generator=g)
        t = {0: [], 1: []}
        outs = {}
        for _ in range(a.rounds):
            for mode in (0, 1):
                lib.efl_pl_tune(16, 5, mode)
                outs[mode] = owner.encrypt(m, counter_base=0).tensor.limbs
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(s)
                for _ in range(a.reps):
                    owner.encrypt(m, counter_base=0)
                ev[1].record(s)
                ev[1].synchronize()
                t[mode].append(ev[0].elapsed_time(ev[1]) / a.reps)
        same = bool(torch.equal(outs[0], outs[1]))
        m0, m1 = float(np.median(t[0])), float(np.median(t[1]))
        print(json.dumps({"tool": "crt_fused_probe", "elements": N, "one_list_ms": round(m0, 4),
                          "per_key_ms": round(m1, 4), "one_list_per_s": round(N / m0 * 1e3),
                          "per_key_per_s": round(N / m1 * 1e3), "speedup": round(m1 / m0, 3),
                          "same_ciphertexts": same, "library": efl.lib.version()}), flush=True)
    lib.efl_pl_tune(16, 5, prev)


if __name__ == "__main__":
    main()
