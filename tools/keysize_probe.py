#!/usr/bin/env python3
"""Stage P throughput at key sizes off and past the round-3 classes: 3072-bit n (runs zero-padded
in the 4096-bit kernels) and 8192-bit n (round 4's 16-lane n^2 family). Per size: host keygen
time, key block + table build, the public-path encryption, the key owner's encryption by CRT and the
decryption, each on N int64 plaintexts already in HBM (median of a few runs, HIP events around the
op on torch's current stream), and a round-trip check. One JSON line per key size."""
import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402

import efl  # noqa: E402
from efl.privacy import paillier_cipher as pc  # noqa: E402


def timed(fn, reps):
    out, ts = None, []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return out, statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, nargs="+", default=[384, 1024])
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = efl.lib.require_gpu()
    for n_bytes in args.bytes:
        t0 = time.perf_counter()
        n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
        t1 = time.perf_counter()
        pub = efl.paillier.Keypair(seed=5)
        pub.set_keys_ints(n, hs, n_bytes // 2, 1, n_bytes=n_bytes)
        pub.key.ensure_table()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        own = efl.paillier.Keypair(seed=5)
        own.set_keys_ints(n, hs, n_bytes // 2, 1, p, q, n_bytes)
        own.encrypt(torch.zeros(1, dtype=torch.int64, device=dev))      # the CRT sub-keys
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        m = torch.randint(-2**62, 2**62, (args.n,), dtype=torch.int64, device=dev)
        pub.encrypt(m[:64])                                               # warm
        ct, t_enc = timed(lambda: pub.encrypt(m, counter_base=0), args.reps)
        ct2, t_crt = timed(lambda: own.encrypt(m, counter_base=0), args.reps)
        same = torch.equal(ct.tensor.limbs, ct2.tensor.limbs)
        d, t_dec = timed(lambda: own.decrypt(ct, dtype=torch.int64), args.reps)
        ok = torch.equal(d, m)
        print(json.dumps({
            "tool": "keysize_probe", "n_bits": n.bit_length(), "limb_class_bits": 32 * pub.key.ln,
            "elements": args.n, "table_window": pub.key.table_window,
            "families": {"n2_ops": pc.kernel_slicing(pub.key.ln, False), "decrypt": pc.kernel_slicing(pub.key.ln, True)},
            "keygen_s": round(t1 - t0, 3), "key_block_s": round(t2 - t1, 3), "crt_subkeys_s": round(t3 - t2, 3),
            "encrypt_per_s": round(args.n / (t_enc * 1e-3)), "encrypt_crt_per_s": round(args.n / (t_crt * 1e-3)),
            "decrypt_per_s": round(args.n / (t_dec * 1e-3)), "crt_equals_public": same, "round_trip_ok": ok,
            "version": efl.lib.version()}), flush=True)
        del pub, own, ct, ct2, d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
