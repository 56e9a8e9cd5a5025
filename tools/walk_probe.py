#!/usr/bin/env python3
"""Fixed-base walk timing (encryption's hs^(a') through the table, SURVEY.md §8(d) Stage P): the n^2
encryption (efl_pl_encrypt, fresh randomness) and the key owner's two CRT walks (efl_pl_fbpowm under
the sub-keys) at the MNIST activation shape and at 262,144 elements, 1024-bit example key (g = 10),
kernel-only HIP events. Run against variant builds (EFL_HIP_LIB=...libefl_hip_<V>.so) to A/B walk
changes; with the EFL_WALK_PROBE=1 build every product reads one L2-resident table entry, which
bounds what hiding the entries' HBM latency could gain. Prints one JSON line per library."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402

import efl  # noqa: E402
from efl.privacy import paillier_cipher as pc  # noqa: E402


def ev_time(fn, reps=5):
    fn()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    sh = torch.cuda.current_stream().cuda_stream
    n_bytes = int(os.environ.get("WP_NBYTES", "128"))
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    kp = efl.paillier.Keypair(seed=7)
    kp.set_keys_ints(n, hs, n_bytes // 2, 10 if n_bytes == 128 else 1, p, q, n_bytes)
    k = kp.key.ensure_table()   # the owner's n^2 table is deferred (KeyBlock)
    subs = k.crt_keys()
    out = {"tool": "walk_probe", "library": efl.lib.LIB_PATH.rsplit("/", 1)[-1], "version": efl.lib.version(),
           "n_bits": 8 * n_bytes, "table_window": k.table_window}
    for N in (256 * 392, 262144):
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev)
        ct = torch.empty((N, k.lc), dtype=torch.int32, device=dev)
        xs = [torch.empty((N, sk.lc), dtype=torch.int32, device=dev) for sk in subs]
        t_enc = ev_time(lambda: efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), None, ct.data_ptr(), N, 7, 0,
                                                                 sh)))
        t_w = [ev_time(lambda sk=sk, x=x: efl.lib.check(lib.efl_pl_fbpowm(*sk.args(), None, x.data_ptr(), N, 7, 0, sh)))
               for sk, x in zip(subs, xs)]
        out[str(N)] = {"encrypt_ms": round(t_enc, 4), "walk_p_ms": round(t_w[0], 4), "walk_q_ms": round(t_w[1], 4),
                       "encrypt_per_s": round(N / t_enc * 1e3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
