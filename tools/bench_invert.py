"""efl_pl_invert (PaillierInvert, Pornin's batched binary GCD) on N random units mod n^2: kernel ms
per call (HIP events) for the 512- and 1024-bit example keys and the 2048-bit one; EFL_HIP_LIB picks
the library (A/B). Checks a sample of inverses with Python ints. One JSON line per key."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

import torch  # noqa: E402


def main():
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    s = torch.cuda.current_stream(dev)
    N = 32768
    for n_bytes in (64, 128, 256):
        n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
        kp = efl.paillier.Keypair(seed=7)
        kp.set_keys_ints(n, hs, n_bytes // 2, 1, p, q, n_bytes)
        rng = random.Random(1)
        n2 = n * n
        vals = [rng.randrange(1, n2) for _ in range(N)]
        x = efl.HexTensor.from_ints(vals)
        ct = kp._cipher(x)
        kp.invert(ct)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(s)
        for _ in range(reps):
            out = kp.invert(ct)
        e1.record(s)
        e1.synchronize()
        got = out.to_hex().to_ints() if hasattr(out, "to_hex") else out.tensor.to_hex().to_ints()
        for j in range(0, N, N // 64):
            assert got[j] == pow(vals[j], -1, n2), j
        print(json.dumps({"lib": os.path.basename(efl.lib.LIB_PATH), "n_bits": 8 * n_bytes, "N": N,
                          "ms_per_call": round(e0.elapsed_time(e1) / reps, 3)}), flush=True)


if __name__ == "__main__":
    main()
