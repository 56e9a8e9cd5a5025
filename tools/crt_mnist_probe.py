"""The key owner's CRT encryption at the paillier_mnist activation (100,352 mantissas, 1024-bit
example key) and the public-key holder's n^2 encryption, `--reps` times each, for a kernel trace
(rocprofv3 --kernel-trace --stats -- python3 tools/crt_mnist_probe.py): which launches the CRT
path's time goes to (the p^2 and q^2 walks, the join) against the n^2 walk.

    python tools/crt_mnist_probe.py [--reps 10] [--parts P]
"""
import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--parts", type=int, default=0)
    ap.add_argument("--n", type=int, default=100352)
    a = ap.parse_args()
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    pc.table_budget(16 << 30)
    n, hs, p, q = pc.generate_keypair_ints(128, 24, random.Random(128))
    owner = efl.paillier.Keypair(seed=7)
    owner.set_keys_ints(n, hs, 64, 10, p, q, 128)
    holder = efl.paillier.Keypair(seed=7)
    holder.set_keys_ints(n, hs, 64, 10, None, None, 128)
    prev = lib.efl_pl_tune(32, 4, a.parts)
    g = torch.Generator(device=dev).manual_seed(0)
    m = torch.randint(-2**40, 2**40, (a.n,), dtype=torch.int64, device=dev, generator=g)
    for kp in (owner, holder):
        kp.encrypt(m, counter_base=0)
        torch.cuda.synchronize()
        for _ in range(a.reps):
            kp.encrypt(m, counter_base=0)
        torch.cuda.synchronize()
    lib.efl_pl_tune(32, 4, prev)
    print("done", efl.lib.version())


if __name__ == "__main__":
    main()
