#!/usr/bin/env python3
"""Do the mask kernels' output streams collide in HBM? The share (two outputs at the same element
offset), mask_rows (send and keep0 at the same offsets) and noise (one output) kernels on the
[65536, 1024] fp32 tensor, timed with HIP events, once with every output its own torch allocation
(what efl.secret_sharing does) and once per stagger: all outputs carved from one buffer, output k
starting `stagger` x k bytes past a 2 MiB boundary. Medians over interleaved rounds. One JSON line.

    python tools/mask_layout_probe.py [--staggers 0,4096,69632,1052672] [--rounds 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--staggers", default="0,4096,69632,1052672")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import efl
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    sh = torch.cuda.current_stream(dev).cuda_stream
    R, C = 65536, 1024
    n = R * C
    x = torch.randn(R, C, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    xp = x.data_ptr()
    # output sizes in floats: share (o0, o1); rows (send 3/2, keep0, keep1 1/2)
    layouts = {"separate": None, **{f"stagger{s}": int(s) for s in a.staggers.split(",")}}
    bufs = {}
    for name, st in layouts.items():
        if st is None:
            o = [torch.empty(n, device=dev) for _ in range(2)]
            r = [torch.empty(n * 3 // 2, device=dev), torch.empty(n, device=dev), torch.empty(n // 2, device=dev)]
            bufs[name] = ([t.data_ptr() for t in o], [t.data_ptr() for t in r], o + r)
            continue
        align = 2 << 20
        sizes = [n, n]
        total = sum(sizes) * 4 + align * 3 + st * 3
        big = torch.empty(total // 4 + 1, device=dev)
        base = (big.data_ptr() + align - 1) // align * align

        def carve(sizes):
            ptrs, off = [], base
            for k, sz in enumerate(sizes):
                ptrs.append(off + st * k)
                off = (off + st * k + sz * 4 + align - 1) // align * align
            return ptrs
        so = carve([n, n])
        big2 = torch.empty((n * 3 * 4 + align * 3 + st * 3) // 4 + 1, device=dev)
        base = (big2.data_ptr() + align - 1) // align * align
        sr = carve([n * 3 // 2, n, n // 2])
        bufs[name] = (so, sr, [big, big2])
    cases = {
        "noise": (8, lambda o, r: lib.efl_ss_noise(xp, o[0], o[1], n, 0, 7, 0, 1.0, sh)),
        "share": (12, lambda o, r: lib.efl_ss_noise(xp, o[0], o[1], n, 1, 7, 0, 1.0, sh)),
        "mask_rows": (16, lambda o, r: lib.efl_ss_mask_rows(xp, r[0], r[1], r[2], R, C, 7, 0, sh)),
    }
    times = {(k, l): [] for k in cases for l in layouts}
    for _ in range(a.rounds):
        for k, (_, fn) in cases.items():
            for l in layouts:
                o, r, _keep = bufs[l]
                fn(o, r)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.steps):
                    fn(o, r)
                e1.record()
                e1.synchronize()
                times[(k, l)].append(e0.elapsed_time(e1) / a.steps)
    out = {"tool": "mask_layout_probe", "library": efl.lib.version(), "shape": [R, C], "results": {}}
    for k, (bpe, _) in cases.items():
        out["results"][k] = {}
        for l in layouts:
            ms = float(np.median(times[(k, l)]))
            out["results"][k][l] = {"ms": round(ms, 4), "frac": round(bpe * n / (ms * 1e-3) / 1e9 / PEAK_GBS, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
