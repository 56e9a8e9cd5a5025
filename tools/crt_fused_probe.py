"""The key owner's CRT encryption per efl_pl_tune(16, 5, v) mode: 1 one launch per sub-key and the
join launch, 2 an element's two walks in one wave with the join at its end (0, the default, picks
2 where it applies), interleaved on one box, at the
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
        modes = (1, 2, 0)
        t = {v: [] for v in modes}
        outs = {}
        for _ in range(a.rounds):
            for v in modes:
                lib.efl_pl_tune(16, 5, v)
                outs[v] = owner.encrypt(m, counter_base=0).tensor.limbs
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(s)
                for _ in range(a.reps):
                    owner.encrypt(m, counter_base=0)
                ev[1].record(s)
                ev[1].synchronize()
                t[v].append(ev[0].elapsed_time(ev[1]) / a.reps)
        same = all(bool(torch.equal(outs[v], outs[1])) for v in modes)
        ms = {v: float(np.median(t[v])) for v in modes}
        print(json.dumps({"tool": "crt_fused_probe", "elements": N,
                          "ms": {"per_key": round(ms[1], 4), "pair": round(ms[2], 4), "default": round(ms[0], 4)},
                          "per_s": {"per_key": round(N / ms[1] * 1e3), "pair": round(N / ms[2] * 1e3),
                                    "default": round(N / ms[0] * 1e3)},
                          "same_ciphertexts": same, "library": efl.lib.version()}), flush=True)
    lib.efl_pl_tune(16, 5, prev)


if __name__ == "__main__":
    main()
