"""Stage-F encode / decode time for every dtype ConvertToFixedPoint takes (fixed_point.cc:53-192),
64 Mi elements each, HIP events on the launch stream; one JSON line per (library, dtype) with the
achieved algorithmic GB/s (encode: element size + 16 B; decode of fp32/fp64: 16 B + element size).
EFL_HIP_LIB picks the library (A/B of launch shapes).

    python tools/bench_fxp_dtypes.py [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import efl
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    s = torch.cuda.current_stream(dev)
    sh = s.cuda_stream
    n = 1 << 26
    g = torch.Generator(device=dev).manual_seed(0)
    M = torch.empty(n, dtype=torch.int64, device=dev)
    E = torch.empty(n, dtype=torch.int64, device=dev)
    for name, dt in (("float32", torch.float32), ("float64", torch.float64), ("int32", torch.int32),
                     ("int64", torch.int64)):
        if dt.is_floating_point:
            x = torch.randn(n, device=dev, generator=g, dtype=dt)
        else:
            x = torch.randint(-2**30, 2**30, (n,), device=dev, generator=g, dtype=dt)
        code = efl.lib.dt_code(dt)
        enc = lambda: efl.lib.check(lib.efl_fxp_encode(x.data_ptr(), code, M.data_ptr(), E.data_ptr(), n, 0, sh))
        res = {"lib": os.path.basename(efl.lib.LIB_PATH), "dtype": name, "elements": n}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        enc()
        ev[0].record(s)
        for _ in range(a.reps):
            enc()
        ev[1].record(s)
        ev[1].synchronize()
        t = ev[0].elapsed_time(ev[1]) / a.reps
        res["encode_ms"] = round(t, 4)
        res["encode_GBs"] = round(n * (x.element_size() + 16) / (t * 1e-3) / 1e9, 1)
        if dt.is_floating_point:
            y = torch.empty_like(x)
            flags = 1 if efl.lib.flush_denormal() else 0
            dec = lambda: efl.lib.check(lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), code, n, n, flags, sh))
            dec()
            ev[0].record(s)
            for _ in range(a.reps):
                dec()
            ev[1].record(s)
            ev[1].synchronize()
            t = ev[0].elapsed_time(ev[1]) / a.reps
            res["decode_ms"] = round(t, 4)
            res["decode_GBs"] = round(n * (16 + x.element_size()) / (t * 1e-3) / 1e9, 1)
            if dt == torch.float64:
                assert torch.equal(y.view(torch.int64), x.view(torch.int64)) or torch.equal(y[x != 0], x[x != 0])
        print(json.dumps(res), flush=True)
        del x


if __name__ == "__main__":
    main()
