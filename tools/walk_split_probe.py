"""Row-split fixed-base walks (efl_pl_tune(ln, 4, P)) A/B on one GPU: the 1024-bit example key, the
key owner's CRT encryption and the public-key holder's n^2 encryption, at the paillier_mnist
activation (100,352 elements) and at 262,144, for P = 1 (unsplit), 2..5 and 0 (chosen per launch);
interleaved rounds, HIP events on the launch stream, median over rounds. Results are checked equal
to the unsplit ciphertexts.

    python tools/walk_split_probe.py [--rounds 3] [--reps 5]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n-bytes", type=int, default=128)
    a = ap.parse_args()
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    s = torch.cuda.current_stream(dev)
    pc.table_budget(32 << 30)          # owner and holder each with their production tables
    n, hs, p, q = pc.generate_keypair_ints(a.n_bytes, 24, random.Random(a.n_bytes))
    owner = efl.paillier.Keypair(seed=7)
    owner.set_keys_ints(n, hs, a.n_bytes // 2, 10, p, q, a.n_bytes)
    holder = efl.paillier.Keypair(seed=7)
    holder.set_keys_ints(n, hs, a.n_bytes // 2, 10, None, None, a.n_bytes)
    owner.key.crt_keys()
    ln = owner.key.ln
    arms = [1, 2, 3, 4, 5, 0]
    out = []
    for N in (100352, 262144):
        g = torch.Generator(device=dev).manual_seed(0)
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev, generator=g)
        times = {(who, P): [] for who in ("owner_crt", "holder_n2") for P in arms}
        ref = {}
        for _ in range(a.rounds):
            for who, kp in (("owner_crt", owner), ("holder_n2", holder)):
                for P in arms:
                    prev = lib.efl_pl_tune(ln, 4, P)
                    try:
                        c = kp.encrypt(m, counter_base=0).tensor.limbs
                        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                        ev[0].record(s)
                        for _ in range(a.reps):
                            kp.encrypt(m, counter_base=0)
                        ev[1].record(s)
                        ev[1].synchronize()
                    finally:
                        lib.efl_pl_tune(ln, 4, prev)
                    times[(who, P)].append(ev[0].elapsed_time(ev[1]) / a.reps)
                    if (who, N) not in ref:
                        ref[(who, N)] = c
                    elif not torch.equal(c, ref[(who, N)]):
                        raise SystemExit(f"{who} P={P}: ciphertexts differ")
        for (who, P), ts in times.items():
            t = float(np.median(ts))
            line = {"tool": "walk_split_probe", "n_bits": 8 * a.n_bytes, "elements": N, "path": who, "parts": P,
                    "ms": round(t, 4), "encrypts_per_s": round(N / t * 1e3), "library": efl.lib.version()}
            out.append(line)
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
