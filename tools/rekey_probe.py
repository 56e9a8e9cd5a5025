#!/usr/bin/env python3
"""Cost of one re-key (PaillierHook with update_step_interval, paillier.py:195-202) on the key
owner: host key generation (generate_keypair_ints: native Miller-Rabin + CRT hs), the key block with
its fixed-base table built on the GPU, and the CRT sub-keys of the owner's encryption (built on its
first encryption); device memory held per keypair, the peak during a re-key of a live keypair, and
what is left after the keypair is dropped. One JSON line per key size."""
import gc
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import torch  # noqa: E402

import efl  # noqa: E402
from efl.privacy import paillier_cipher as pc  # noqa: E402

MIB = float(1 << 20)


def main():
    dev = efl.lib.require_gpu()
    for n_bytes in (128, 256, 512):
        torch.cuda.synchronize()
        gc.collect()
        base = torch.cuda.memory_allocated(dev)
        kp = efl.paillier.Keypair(seed=3)
        gen = []
        for rep in range(3):                       # re-keys of one live keypair, as the hook does
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats(dev)
            before = torch.cuda.memory_allocated(dev)
            t0 = time.perf_counter()
            n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(1000 * n_bytes + rep))
            t1 = time.perf_counter()
            kp.set_keys_ints(n, hs, n_bytes // 2, 1, p, q, n_bytes)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            kp.encrypt(torch.zeros(1, dtype=torch.int64, device=dev))    # builds the CRT sub-keys
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            subs = kp.key.crt_keys() or ()
            gen.append({"keygen_s": round(t1 - t0, 3), "key_block_s": round(t2 - t1, 3),
                        "crt_subkeys_s": round(t3 - t2, 3),
                        "table_MiB": round(kp.key.block_bytes / MIB, 1),
                        "crt_tables_MiB": round(sum(s.block_bytes for s in subs) / MIB, 1),
                        "held_before_MiB": round((before - base) / MIB, 1),
                        "held_after_MiB": round((torch.cuda.memory_allocated(dev) - base) / MIB, 1),
                        "peak_MiB": round((torch.cuda.max_memory_allocated(dev) - base) / MIB, 1)})
            del subs
        del kp
        gc.collect()
        torch.cuda.synchronize()
        left = torch.cuda.memory_allocated(dev) - base
        print(json.dumps({"tool": "rekey_probe", "n_bits": 8 * n_bytes, "version": efl.lib.version(),
                          "rekeys": gen, "left_after_drop_MiB": round(left / MIB, 1)}), flush=True)


if __name__ == "__main__":
    main()
