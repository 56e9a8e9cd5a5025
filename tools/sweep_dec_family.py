#!/usr/bin/env python3
"""Decryption kernel family vs launch size: for each key size and element count, time CRT
decryption (efl_pl_decrypt, HIP events, kernel-only) with every sliced family C compiled for it
(limbs per lane; G = ln / C lanes per element), interleaved over repeats. Picks the default of
efl_pl_tune's per-launch sizing (decrypt_family in csrc/paillier.hip). One JSON line per key.

    python tools/sweep_dec_family.py [--keys 1024,2048,4096] [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402
from efl.privacy import paillier_cipher as pc  # noqa: E402

SIZES = {1024: (4096, 16384, 32768, 50176, 100352, 262144), 2048: (4096, 16384, 32768, 65536, 131072),
         4096: (1024, 4096, 16384, 65536)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", default="1024,2048,4096")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    with open(os.path.join(ROOT, "tests", "golden", "paillier_kat.json")) as f:
        keys = {8 * k["n_bytes"]: k for k in json.load(f)["keys"]}
    s = torch.cuda.current_stream()
    for bits in (int(b) for b in a.keys.split(",")):
        k = keys[bits]
        kp = efl.paillier.Keypair(seed=3)
        kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1, int(k["p"], 16), int(k["q"], 16))
        kb = kp.key
        ln = kb.ln
        fams = [c for c in pc.SLICINGS[ln][1] if c]
        res = {"tool": "sweep_dec_family", "n_bits": bits, "version": efl.lib.version(), "ms": {}, "Mps": {}}
        for n in SIZES[bits]:
            m = torch.randint(-2**40, 2**40, (n,), dtype=torch.int64, device=dev)
            ct = kp.encrypt(m).tensor.limbs
            mag = torch.empty((n, ln), dtype=torch.int32, device=dev)
            neg = torch.empty(n, dtype=torch.int8, device=dev)
            times = {c: [] for c in fams}
            prev = pc.kernel_slicing(ln, True)
            try:
                for r in range(a.reps + 1):
                    for c in fams:
                        pc.set_kernel_slicing(ln, True, c)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(s)
                        efl.lib.check(lib.efl_pl_decrypt(*kb.args(), ct.data_ptr(), mag.data_ptr(), neg.data_ptr(), n,
                                                         s.cuda_stream))
                        e1.record(s)
                        e1.synchronize()
                        if r:
                            times[c].append(e0.elapsed_time(e1))
            finally:
                pc.reset_kernel_slicing(ln, True)
            res["ms"][n] = {c: round(float(np.median(v)), 3) for c, v in times.items()}
            res["Mps"][n] = {c: round(n / float(np.median(v)) / 1e3, 3) for c, v in times.items()}
            res.setdefault("best", {})[n] = min(times, key=lambda c: np.median(times[c]))
            del prev
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
