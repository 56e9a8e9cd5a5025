#!/usr/bin/env python3
"""Secret-sharing masks on one MI355X: the per-element kernels of
csrc/mask.hip on a 256 MiB fp32 tensor ([65536, 1024], the BASELINE config-2 shape), timed with HIP
events on the launch stream, against their HBM roofline, beside the numpy oracle (the TF op chain
restated: uniform, mul, slices, adds, concat) on a bounded CPU sample. One JSON line per kernel.

Algorithmic bytes per fp32 element (read x once, write every output once):
  noise (op 0)            4 + 4            =  8 B
  share (op 1), weight (op 2)  4 + 4 + 4   = 12 B
  mask_cols (mode A)      4 + 6 + 4 + 2    = 16 B  (send 3/2, keep a - e, keep 1/2)
  mask_rows (mode B)      4 + 6 + 4 + 2    = 16 B
  dp_noise (efl_dp_noise, both modes: Box-Muller normal, noise, / microbatches)  4 + 4 = 8 B
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402

PEAK_GBS = 8000.0
ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=65536)
ap.add_argument("--cols", type=int, default=1024)
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--rounds", type=int, default=3, help="interleaved rounds over all kernels; the median is reported")
ap.add_argument("--no-cpu-baseline", action="store_true")
args = ap.parse_args()

dev = efl.lib.require_gpu()
lib = efl.lib.raw()
R, C = args.rows, args.cols
n = R * C
x = torch.randn(R, C, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
o0, o1 = torch.empty_like(x), torch.empty_like(x)
send_c = torch.empty(R, C * 3 // 2, device=dev)
k1_c = torch.empty(R, C // 2, device=dev)
send_r = torch.empty(R * 3 // 2, C, device=dev)
k1_r = torch.empty(R // 2, C, device=dev)
s = torch.cuda.current_stream()
sh = s.cuda_stream
xp, p0, p1 = x.data_ptr(), o0.data_ptr(), o1.data_ptr()

cases = {
    "noise": (8, lambda: lib.efl_ss_noise(xp, p0, p1, n, 0, 7, 0, 1.0, sh)),
    "share": (12, lambda: lib.efl_ss_noise(xp, p0, p1, n, 1, 7, 0, 1.0, sh)),
    "weight_noise": (12, lambda: lib.efl_ss_noise(xp, p0, p1, n, 2, 7, 0, 2.0, sh)),
    "mask_cols": (16, lambda: lib.efl_ss_mask_cols(xp, send_c.data_ptr(), p0, k1_c.data_ptr(), R, C, 7, 0, sh)),
    "mask_rows": (16, lambda: lib.efl_ss_mask_rows(xp, send_r.data_ptr(), p0, k1_r.data_ptr(), R, C, 7, 0, sh)),
    "dp_noise_elementwise": (8, lambda: lib.efl_dp_noise(xp, p0, n, 0, 1.0, 256.0, 7, 0, sh)),
    "dp_noise_gaussian": (8, lambda: lib.efl_dp_noise(xp, p0, n, 1, 1.1, 256.0, 7, 0, sh)),
}


def _dp_blocks(nb, mode):
    def run():
        old = lib.efl_fxp_tune(20, nb)
        rc = lib.efl_dp_noise(xp, p0, n, mode, 1.0 if mode == 0 else 1.1, 256.0, 7, 0, sh)
        lib.efl_fxp_tune(20, old)
        return rc
    return run


# efl_fxp_tune(20, nb): the DP noise kernel at 1 / 2 / 4 Philox blocks per lane (A/B of the default)
for _nb in (1, 2, 4):
    cases[f"dp_noise_elementwise_nb{_nb}"] = (8, _dp_blocks(_nb, 0))


def _mask_shape(nb, st, fn):
    def run():
        lib.efl_fxp_tune(25, nb)
        lib.efl_fxp_tune(28, st)
        rc = fn()
        lib.efl_fxp_tune(25, -2)       # back to the per-kernel defaults
        lib.efl_fxp_tune(28, -2)
        return rc
    return run


# efl_fxp_tune(25, nb) / (28, st): the secret-sharing mask kernels at 1 / 2 / 4 lane groups per
# lane and plain / nontemporal / `nt sc1` stores (MASK_SWEEP=0 skips the sweep)
if os.environ.get("MASK_SWEEP", "1") == "1":
    for _name in ("noise", "share", "mask_cols", "mask_rows"):
        for _nb in (1, 2, 4):
            for _st in (0, 2, 7):
                cases[f"{_name}_nb{_nb}_st{_st}"] = (cases[_name][0], _mask_shape(_nb, _st, cases[_name][1]))


def _rows_layout(half, nb, st, fn):
    """efl_fxp_tune(29, half): mask_rows with the row pair over the two halves of a wave (1, the
    default) or in one lane (0, round 5's kernel), at nb lane groups per lane and store flavour st"""
    def run():
        lib.efl_fxp_tune(29, half)
        lib.efl_fxp_tune(25, nb)
        lib.efl_fxp_tune(28, st)
        rc = fn()
        lib.efl_fxp_tune(29, 1)
        lib.efl_fxp_tune(25, -2)
        lib.efl_fxp_tune(28, -2)
        return rc
    return run


cases["mask_rows_pair"] = (16, _rows_layout(0, 1, 7, cases["mask_rows"][1]))


def _noise_halves(half, st, fn):
    """efl_fxp_tune(30, half): share / weight noise with the outputs over the halves of a wave"""
    def run():
        lib.efl_fxp_tune(30, half)
        lib.efl_fxp_tune(28, st)
        rc = fn()
        lib.efl_fxp_tune(30, 1)
        lib.efl_fxp_tune(28, -2)
        return rc
    return run


cases["share_one_lane"] = (12, _noise_halves(0, 7, cases["share"][1]))
cases["weight_noise_one_lane"] = (12, _noise_halves(0, 7, cases["weight_noise"][1]))
if os.environ.get("MASK_SWEEP", "1") == "1":
    for _st in (0, 2, 7):
        cases[f"share_half_st{_st}"] = (12, _noise_halves(1, _st, cases["share"][1]))
        cases[f"weight_noise_half_st{_st}"] = (12, _noise_halves(1, _st, cases["weight_noise"][1]))
if os.environ.get("MASK_SWEEP", "1") == "1" or os.environ.get("MASK_ROWS_SWEEP") == "1":
    for _nb in (1, 2, 4):
        for _st in (0, 2, 7):
            cases[f"mask_rows_half_nb{_nb}_st{_st}"] = (16, _rows_layout(1, _nb, _st, cases["mask_rows"][1]))


def cpu_sample(name, rows=1024):
    """The oracle (numpy, the reference's op chain) on the first `rows` rows; GiB/s of input."""
    from oracle import mask
    xs = x[:rows].cpu().numpy()
    fn = {"noise": lambda: mask.noise(xs, 7, 0, 0), "share": lambda: mask.noise(xs, 7, 0, 1),
          "weight_noise": lambda: mask.noise(xs, 7, 0, 2, 2.0),
          "mask_cols": lambda: mask.mask_cols(xs, 7, 0), "mask_rows": lambda: mask.mask_rows(xs, 7, 0),
          "dp_noise_elementwise": lambda: mask.dp_noise(xs, 7, 0, 0, 1.0, 256.0),
          "dp_noise_gaussian": lambda: mask.dp_noise(xs, 7, 0, 1, 1.1, 256.0)}[name]
    fn()
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        fn()
        reps += 1
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(xs.nbytes / dt / 2**30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"[{rows}, {C}] fp32 slice, numpy oracle/mask.py (uniform + elementwise + concat), {reps} reps"}


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.steps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.steps


for name, (bpe, fn) in cases.items():
    for _ in range(5):
        efl.lib.check(fn())
torch.cuda.synchronize()
# interleaved rounds: a box's clock drift over the run hits every kernel alike
times = {name: [] for name in cases}
for _ in range(args.rounds):
    for name, (bpe, fn) in cases.items():
        times[name].append(timed(fn))
for name, (bpe, fn) in cases.items():
    ms = float(np.median(times[name]))
    gbs = bpe * n / (ms * 1e-3) / 1e9
    line = {"kernel": name, "elements": n, "shape": [R, C], "ms": round(ms, 4),
            "ms_rounds": [round(t, 4) for t in times[name]],
            "GiB_per_s_plaintext": round(4 * n / (ms * 1e-3) / 2**30, 2),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_GBS, 4), "bytes_per_elem": bpe},
            "library": efl.lib.version()}
    if not args.no_cpu_baseline and name in ("noise", "share", "weight_noise", "mask_cols", "mask_rows",
                                             "dp_noise_elementwise", "dp_noise_gaussian"):
        line["cpu_baseline"] = cpu_sample(name)
    print(json.dumps(line), flush=True)
