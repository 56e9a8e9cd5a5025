"""Timing-only probe of efl_pl_matmul on the MNIST receiver product ([256, 392] ciphertexts x
[392, 128] weights, 1024-bit example key) for the library named by EFL_HIP_LIB — including
EFL_MAT_PROBE variant builds whose results are deliberately wrong (no correctness check here;
bench.py --stage p checks the default build). One JSON line: kernel ms per matmul (HIP events).

    EFL_HIP_LIB=.../libefl_hip_mmscan.so python tools/matmul_probe.py
"""
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
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    label, n_bytes, a_bytes, g, _ = bench.STAGE_P_KEYS[1]
    n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
    kp = efl.paillier.Keypair(seed=7)
    kp.set_keys_ints(n, hs, a_bytes, g, p, q, n_bytes)
    k = kp.key.ensure_table()   # the owner's n^2 table is deferred (KeyBlock)
    u, v, w = bench.STAGE_P_MATMUL
    gen = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(u, v, device=dev, generator=gen)
    lim = (6.0 / (v + w)) ** 0.5
    W = (torch.rand(v, w, device=dev, generator=gen) * 2 - 1) * lim
    xm, xe = efl.lib.convert_to_fixed_point(x)
    ym, ye = efl.lib.convert_to_fixed_point(W, decrease_precision=True)
    X = torch.empty((u * v, k.lc), dtype=torch.int32, device=dev)
    efl.lib.check(lib.efl_pl_encrypt(*k.args(), xm.data_ptr(), None, X.data_ptr(), u * v, 11, 0, sh))
    zpos = torch.empty((u * w, k.lc), dtype=torch.int32, device=dev)
    zneg = torch.empty_like(zpos)
    ze = torch.empty((u, w), dtype=torch.int64, device=dev)

    def mm():
        efl.lib.check(lib.efl_pl_matmul(*k.args(), X.data_ptr(), xe.data_ptr(), ym.data_ptr(), ye.data_ptr(),
                                        zpos.data_ptr(), zneg.data_ptr(), ze.data_ptr(), u, v, w, sh))

    mm()
    reps = 3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        mm()
    e1.record(stream)
    e1.synchronize()
    ref = zpos[:64].clone()
    print(json.dumps({"lib": os.path.basename(efl.lib.LIB_PATH), "shape": [u, v, w],
                      "ms": round(e0.elapsed_time(e1) / reps, 3),
                      "zpos_hash": int(ref.to(torch.int64).sum().item())}), flush=True)


if __name__ == "__main__":
    main()
