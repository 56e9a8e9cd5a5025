#!/usr/bin/env python3
"""Encryption throughput against the fixed-base table's window W (efl_pl_key.table_window): wider
windows cut the table products per encryption (ceil(a_bits / W)) but grow the table (rows x (2^W - 1)
entries, two layouts) and its key-setup time, and turn its lookups into random reads beyond the
256 MB Infinity Cache. The 1024-bit example key (512-bit a), 262,144 and 100,352 fresh-randomness
encryptions, HIP events; the output is checked by decrypting a sample. Prints one JSON line per W.

    python tools/table_window_probe.py [--n-bytes 512 --a-bytes 256 --group 1 --sizes 65536] [W ...]
"""
import argparse
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


def main():
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-bytes", type=int, default=128)
    ap.add_argument("--a-bytes", type=int, default=64)
    ap.add_argument("--group", type=int, default=10)
    ap.add_argument("--sizes", type=int, nargs="+", default=[262144, 100352])
    ap.add_argument("--crt", action="store_true", help="also time the key owner's encryption by CRT")
    ap.add_argument("windows", type=int, nargs="*", default=[12, 13, 14, 15, 16])
    a = ap.parse_args()
    n_bytes, a_bytes, g = a.n_bytes, a.a_bytes, a.group
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    for W in a.windows:
        kp = efl.paillier.Keypair(seed=7)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kp.set_keys_ints(n, hs, a_bytes, g, p, q, n_bytes, table_window=W)
        k = kp.key.ensure_table()   # the owner's n^2 table is deferred (KeyBlock): built here, timed
        torch.cuda.synchronize()
        setup = time.perf_counter() - t0
        line = {"n_bits": 8 * n_bytes, "W": k.table_window, "rows": k.desc.table_rows, "cols": k.desc.table_cols,
                "key_block_MiB": round(k.block_bytes / 2**20, 1), "key_setup_ms": round(setup * 1e3, 1)}
        for N in a.sizes:
            m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev,
                              generator=torch.Generator(device=dev).manual_seed(N))
            ct = torch.empty((N, k.lc), dtype=torch.int32, device=dev)

            def enc():
                efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), None, ct.data_ptr(), N, 7, 0, sh))
            enc()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                enc()
            e1.record(st)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 5
            c = min(N, 256)
            got = kp.decrypt(pc.CipherTensor(ct[:c], (c,), k), dtype=torch.int64)
            line[str(N)] = {"ms": round(ms, 3), "encrypts_per_s": round(N / ms * 1e3), "ok": bool(torch.equal(got, m[:c]))}
            subs = k.crt_keys() if a.crt else None
            if subs:
                xs = [torch.empty((N, sk.lc), dtype=torch.int32, device=dev) for sk in subs]
                cc = torch.empty_like(ct)

                def enc_crt():
                    for sk, x in zip(subs, xs):
                        efl.lib.check(lib.efl_pl_fbpowm(*sk.args(), None, x.data_ptr(), N, 7, 0, sh))
                    efl.lib.check(lib.efl_pl_crt_join(*k.args(), xs[0].data_ptr(), xs[1].data_ptr(), m.data_ptr(),
                                                      cc.data_ptr(), N, sh))
                enc_crt()
                e0.record(st)
                for _ in range(5):
                    enc_crt()
                e1.record(st)
                e1.synchronize()
                ms = e0.elapsed_time(e1) / 5
                line[str(N)].update({"crt_ms": round(ms, 3), "crt_encrypts_per_s": round(N / ms * 1e3),
                                     "crt_equal": bool(torch.equal(cc, ct)),
                                     "crt_tables_MiB": round(sum(sk.block_bytes for sk in subs) / 2**20, 1)})
        print(json.dumps(line), flush=True)
        del kp, k
        import gc
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
