#!/usr/bin/env python3
"""Hex text <-> limbs kernels (the DT_STRING form ciphertexts cross the wire in, gmp_utils.cc:146-150,
paillier.cc:127; FixedPointToFloatPoint<string> fixed_point.cc:255-257) on one GPU. Times with
HIP events on the launch stream, median of reps; prints one JSON line.

  write   efl_hex_lengths + efl_hex_write of N ciphertexts (2 ln limbs each) -> text
  parse   efl_hex_parse of that text back into limbs (checked equal)
  fdecode efl_fxp_decode_hex of N short plaintext mantissas (decrypted values, ~10-20 digits)

Algorithmic bytes: write reads 4 L + writes ~8 L chars per element; parse the reverse."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import efl  # noqa: E402
from efl.privacy import paillier_cipher as pc  # noqa: E402

dev = efl.lib.require_gpu()
lib = efl.lib.raw()
s = torch.cuda.current_stream()
sh = s.cuda_stream
out = {"tool": "bench_hex", "version": efl.lib.version()}


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


for label, L, N in (("1024-bit n (2048-bit ciphertexts), MNIST [256,392]", 64, 256 * 392),
                    ("4096-bit n (8192-bit ciphertexts)", 256, 65536)):
    g = torch.Generator(device=dev).manual_seed(L)
    limbs = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device=dev, generator=g)
    lens = torch.empty(N, dtype=torch.int64, device=dev)
    offs = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    lib.efl_hex_lengths(limbs.data_ptr(), L, None, lens.data_ptr(), N, sh)
    torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item())
    chars = torch.empty(total, dtype=torch.uint8, device=dev)

    def write():
        efl.lib.check(lib.efl_hex_lengths(limbs.data_ptr(), L, None, lens.data_ptr(), N, sh))
        efl.lib.check(lib.efl_hex_write(limbs.data_ptr(), L, None, offs.data_ptr(), chars.data_ptr(), N, sh))

    back = torch.empty_like(limbs)
    bad = torch.empty(1, dtype=torch.int64, device=dev)

    def parse():
        efl.lib.check(lib.efl_hex_parse(chars.data_ptr(), offs.data_ptr(), L, back.data_ptr(), None, N,
                                        bad.data_ptr(), sh))

    t_w = timed(write)
    t_p = timed(parse)
    ok = bool(torch.equal(back, limbs)) and int(bad.item()) == -1
    # spot-check the text against Python's format
    h = chars[: int(offs[3].item())].cpu().numpy().tobytes().decode()
    o = offs[:4].cpu().tolist()
    want = [format(int.from_bytes(limbs[r].cpu().numpy().astype("<u4").tobytes(), "little"), "x") for r in range(3)]
    ok = ok and [h[o[r]:o[r + 1]] for r in range(3)] == want
    bw = N * L * 4 + total
    out[label] = {"elements": N, "chars": total, "write_ms": round(t_w, 4), "parse_ms": round(t_p, 4),
                  "write_GBs": round(bw / t_w / 1e6, 1), "parse_GBs": round(bw / t_p / 1e6, 1), "ok": ok}

# FixedPointToFloatPoint<string>: decrypted mantissas as hex (short text), N = MNIST activation
N = 256 * 392
rng = np.random.default_rng(0)
m = rng.integers(-2**50, 2**50, N)
strs = [format(int(v), "x") if v >= 0 else "-" + format(-int(v), "x") for v in m]
hx = efl.HexTensor.from_strings(strs)
E = torch.from_numpy(rng.integers(-60, -20, N)).to(dev)
chars_d, offs_d = hx.device_buffers(dev)
y = torch.empty(N, dtype=torch.float32, device=dev)
bad = torch.empty(1, dtype=torch.int64, device=dev)


def fdec():
    efl.lib.check(lib.efl_fxp_decode_hex(chars_d.data_ptr(), offs_d.data_ptr(), E.data_ptr(), y.data_ptr(), 1, N, 1,
                                         bad.data_ptr(), sh))


t_f = timed(fdec)
yo = (torch.from_numpy(m.astype(np.float64)) * torch.pow(2.0, E.cpu().double())).float()
out["fdecode"] = {"elements": N, "chars": int(offs_d[-1].item()), "ms": round(t_f, 4),
                  "ok": bool(torch.equal(y.cpu(), yo))}
print(json.dumps(out), flush=True)
