#!/usr/bin/env python3
"""Decryption A/B between library builds (run once per build, alternating, in one gpurun call; the
build comes from EFL_HIP_LIB): CRT decryption of N int64 mantissas at the 2048- and 4096-bit keys
(the G = 2 / G = 4 sliced families, round 6's folded squarings), timed with HIP events over `reps`
launches, the plaintexts checked. One JSON line.

    EFL_HIP_LIB=.../libefl_hip_nofold.so python tools/dec_ab.py --label nofold
"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    pc.table_budget(16 << 30)
    out = {"tool": "dec_ab", "label": a.label, "library": efl.lib.version(), "keys": {}}
    for n_bytes, N in ((256, 65536), (512, 65536)):
        n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
        kp = efl.paillier.Keypair(seed=7)
        kp.set_keys_ints(n, hs, n_bytes // 2, 1, p, q, n_bytes)
        k = kp.key
        g = torch.Generator(device=dev).manual_seed(0)
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev, generator=g)
        ct = kp.encrypt(m, counter_base=0).tensor
        mag = torch.empty((N, k.ln), dtype=torch.int32, device=dev)
        neg = torch.empty(N, dtype=torch.int8, device=dev)

        def dec():
            efl.lib.check(lib.efl_pl_decrypt(*k.args(), ct.limbs.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, sh))
        dec()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            dec()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        ok = bool(torch.equal(kp.decrypt(ct, dtype=torch.int64), m))
        out["keys"][f"{8 * n_bytes}"] = {"elements": N, "ms": round(ms, 3), "elements_per_s": round(N / ms * 1e3),
                                         "family": pc.kernel_slicing(k.ln, True), "roundtrip_ok": ok}
        k.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
