"""efl_pl_matmul on the MNIST receiver product ([256, 392] ciphertexts x [392, 128] weights, 1024-bit
example key) for each term split S (efl_pl_tune(ln, 3, S); 0 = the per-launch choice): one JSON line
per setting with bench.py's matmul record (kernel ms, products per output, issue fraction).

    python tools/matmul_sweep.py [S ...]      # default: 0 1 2 4 8 16
"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("splits", nargs="*", type=int, default=[0, 1, 2, 4, 8, 16])
    ap.add_argument("--families", default="", help="comma list of n^2 kernel families (16,32); default as set")
    a = ap.parse_args()
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    stream = torch.cuda.current_stream(dev)
    label, n_bytes, a_bytes, g, _ = bench.STAGE_P_KEYS[1]
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    args = argparse.Namespace(no_cpu_baseline=True, warmup=0, cpu_threads=1)
    ln = n_bytes // 4
    prev, prev_fam = lib.efl_pl_tune(ln, 3, -1), lib.efl_pl_tune(ln, 0, -1)
    fams = [int(f) for f in a.families.split(",") if f] or [prev_fam]
    try:
        for fam in fams:
            if lib.efl_pl_tune(ln, 0, fam) < 0:
                raise SystemExit(f"efl_pl_tune(ln, 0, {fam}) refused")
            kp = efl.paillier.Keypair(seed=7)        # the key block's radix-2^28 layout is per family
            kp.set_keys_ints(n, hs, a_bytes, g, p, q, n_bytes)
            for S in a.splits:
                if lib.efl_pl_tune(ln, 3, S) < 0:
                    raise SystemExit(f"efl_pl_tune(ln, 3, {S}) refused")
                r = bench.stage_p_matmul(args, efl, pc, kp, lib, stream.cuda_stream, stream, dev)
                print(json.dumps({"lib": os.path.basename(efl.lib.LIB_PATH), "family": fam, "splits_setting": S,
                                  "key": label, **r}), flush=True)
    finally:
        lib.efl_pl_tune(ln, 3, prev)
        lib.efl_pl_tune(ln, 0, -2)


if __name__ == "__main__":
    main()
