#!/usr/bin/env python3
"""Same-process A/B of the key owner's CRT encryption tail (efl_pl_tune(ln, 6, v)): 1 = round 5's
split-and-join launches, 0 = round 6's product tree across lanes (S chosen), 16 / 8 = the tree with
a fixed S. The paillier_mnist activation (100,352 mantissas, 1024-bit example key, group size 10)
and two other element counts, each mode timed with HIP events over `reps` launches, interleaved over
`rounds`; medians. Ciphertexts of every mode are compared bit for bit. One JSON line.

    python tools/crt_tail_ab.py [--reps 5] [--rounds 5]
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--modes", default="1,0,16,8")
    ap.add_argument("--shapes", default="100352,100675,50176")
    a = ap.parse_args()
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    pc.table_budget(16 << 30)
    n, hs, p, q = pc.generate_keypair_ints(128, 24, random.Random(128))
    kp = efl.paillier.Keypair(seed=7)
    kp.set_keys_ints(n, hs, 64, 10, p, q, 128)
    k = kp.key
    k.crt_keys()
    modes = [int(v) for v in a.modes.split(",")]
    out = {"tool": "crt_tail_ab", "library": efl.lib.version(), "reps": a.reps, "rounds": a.rounds, "shapes": {}}
    prev = lib.efl_pl_tune(16, 6, -1)
    for N in (int(v) for v in a.shapes.split(",")):
        g = torch.Generator(device=dev).manual_seed(N)
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev, generator=g)
        cts = {v: torch.empty((N, k.lc), dtype=torch.int32, device=dev) for v in modes}
        times = {v: [] for v in modes}

        def enc(v):
            efl.lib.check(lib.efl_pl_ctx_encrypt(k.ctx, m.data_ptr(), None, cts[v].data_ptr(), N, 7, 0, 0, sh))
        for v in modes:
            lib.efl_pl_tune(16, 6, v)
            enc(v)
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for v in modes:
                lib.efl_pl_tune(16, 6, v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.reps):
                    enc(v)
                e1.record(st)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.reps)
        same = all(torch.equal(cts[v], cts[modes[0]]) for v in modes)
        out["shapes"][str(N)] = {"same_ciphertexts": same,
                                 **{f"mode{v}_ms": round(float(np.median(times[v])), 4) for v in modes}}
    lib.efl_pl_tune(16, 6, prev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
