#!/usr/bin/env python3
"""Benchmark of the forward-encryption hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1], "config 2"): one 256 MiB fp32 tensor [65536, 1024], N(0,1),
seed = rank, resident in HBM. One STEP = encrypt + decrypt of the whole tensor, i.e.
ConvertToFixedPoint (fp32 -> int64 mantissa + int64 exponent) followed by FixedPointToFloatPoint
(back to fp32), both through libefl_hip.so's C ABI (efls-train/cc/efl/math/fixed_point.cc).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

value = (N x 0.25 GiB) / (max over ranks of the time of K steps / K)        [GiB/s, weak scaling]
Multi-GPU: every rank owns its own 256 MiB shard (the path is element-wise: no payload exchange);
the only collective is the broadcast of the 32-byte key seed from rank 0 (timed apart): RCCL when
every rank has its own GPU, gloo when ranks share one (efl.distributed.choose_backend).

The timed region holds nothing but the K steps (no events, no host work between launches).
roofline: per-kernel average durations come from a second pass of K steps right after it, with HIP
events recorded around every launch on the stream the kernels run on. Algorithmic bytes:
20 B/element per kernel (encode: 4 read + 16 written; decode: 16 read + 4 written), SURVEY.md §8(d).
Decode runs in the reference's TF-runtime rounding mode (FTZ, efl.lib.flush_denormal()).
cpu_baseline: the reference CPU op (oracle/: the literal encode loop of fixed_point.cc:107-137 +
the GMP mpf decode of :235-248, FTZ|DAZ like a TF threadpool thread, contiguous blocks like TF
Shard over every usable host core) timed on this box on the same tensor (rank 0, N = 1 only).
Extra keys at N = 1: "config3" (BASELINE config 3: 4096 x 64 KiB slices, one batched launch per
direction, and the naive per-slice launches), "pinned_path" (the north_star's rate including
pinned H2D/D2H copies: efl.framework.host_pipeline over the same tensor, encrypt leg pinned fp32 ->
pinned M+E, decrypt leg back) and "config5" (the two-process gRPC loopback end to end,
tools/bench_e2e.py, rate including copies).

    python bench.py --stage p      Stage P report (SURVEY.md §8(d) last row), one JSON line per key:
Paillier encrypt (fresh randomness through the fixed-base table) and CRT decrypt of int64
mantissas on one GPU, elements/s, against the VALU roofline (32x32->64 multiply-accumulates of the
Montgomery products vs the measured v_mad_u64_u32 issue rate), beside the reference's GMP path
(oracle/paillier_gmp.c pl_gmp_bench: key state built once, threads like TF Shard) on this box.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "GiB/s device-resident encrypt+decrypt, 256 MiB fp32 tensor, 1/2/4/8 GPUs"
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
ROWS, COLS = 65536, 1024       # 256 MiB fp32
BYTES_PER_ELEM_KERNEL = 20     # each of encode / decode
GIB = float(1 << 30)


def usable_cores():
    """Host cores this process may run on: the affinity mask, capped by a cgroup CPU quota
    (cgroup v2 cpu.max) when one is set. Returns (count, how it was found)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    if quota is not None and math.ceil(quota) < aff:
        return max(1, int(math.ceil(quota))), f"cgroup cpu.max quota {quota:g} CPUs (affinity {aff})"
    return aff, f"sched_getaffinity: {aff} CPUs" + (f" (cgroup quota {quota:g})" if quota else "")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--backend", choices=("nccl", "gloo"), default=None,
                   help="process-group backend for N > 1 (default: nccl if every rank has a GPU)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip the config3 / pinned_path keys")
    p.add_argument("--cpu-threads", type=int,
                   default=int(os.environ["EFL_BENCH_CPU_THREADS"]) if os.environ.get("EFL_BENCH_CPU_THREADS")
                   else None, help="CPU baseline threads (default: every usable core)")
    p.add_argument("--tune", default=os.environ.get("EFL_FXP_TUNE", ""),
                   help="comma list kind=value for efl_fxp_tune (variant exploration)")
    p.add_argument("--rows", type=int, default=ROWS)
    p.add_argument("--stage", choices=("f", "p"), default="f",
                   help="f: the BASELINE.json metric (fixed-point codec); p: the Paillier report")
    return p.parse_args(argv)


def broadcast_seed(world, rank):
    """Broadcast of the key material (32-byte seed) from rank 0 — the path's only collective
    (efl.distributed.broadcast_key_material; RCCL over xGMI on an 8-GPU node); timed apart."""
    if world == 1:
        return os.urandom(32), 0.0
    from efl import distributed as edist
    seed, _ = edist.broadcast_key_material()          # warm the communicator
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        seed, _ = edist.broadcast_key_material(seed if rank == 0 else None)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return seed, (time.perf_counter() - t0) / 10 * 1e6


def load_traffic():
    """Per-launch HBM bytes from the rocprofv3 PMC passes (tools/pmc_traffic.py), if recorded."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def cpu_baseline(x_dev, threads, how, ftz):
    """The reference op on the host: literal encode loop + GMP mpf decode, `threads` contiguous
    blocks. The whole tensor takes about 0.1-0.3 s per pass on 16+ cores; median of 3."""
    from oracle import fxp
    x = x_dev.cpu().numpy().reshape(-1)
    fxp.baseline_encode_decode(x[: 1 << 20], threads, ftz=ftz)          # warm
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        fxp.baseline_encode_decode(x, threads, ftz=ftz)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": round(x.nbytes / GIB / t, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"whole 256 MiB tensor ({x.size} fp32): the literal encode loop "
                      f"(fixed_point.cc:107-137, float-convert ctz) + GMP mpf decode (:235-248) under "
                      f"MXCSR {'FTZ|DAZ' if ftz else 'default'}, contiguous blocks like TF Shard on "
                      f"{threads} threads ({how}), median of 3",
            "ms_per_step": round(t * 1e3, 2)}


def config3(efl, dev, steps, layout="separate"):
    """BASELINE config 3: 4096 64 KiB fp32 tensors ([128, 128] embedding slices, N(0, 0.01),
    seed 1): one batched encode + one batched decode launch over device pointer tables, against
    the naive 2 x 4096 per-slice launches. layout "separate": 4 x 4096 torch allocations (each
    slice its own tensor); "views": the slices are views of one [4096, 128, 128] table per stream
    (embedding slices of one table), which efl.lib.BatchTables sends through the streaming kernels
    as one run."""
    lib = efl.lib.raw()
    slices, elems = 4096, 16384
    g = torch.Generator(device=dev).manual_seed(1)
    if layout == "views":
        big = (torch.randn(slices, 128, 128, device=dev, generator=g) * 0.01,
               torch.empty(slices, 128, 128, dtype=torch.int64, device=dev),
               torch.empty(slices, 128, 128, dtype=torch.int64, device=dev),
               torch.empty(slices, 128, 128, device=dev))
        xs, Ms, Es, ys = ([b[i] for i in range(slices)] for b in big)
    else:
        xs = [torch.randn(128, 128, device=dev, generator=g) * 0.01 for _ in range(slices)]
        Ms = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(slices)]
        Es = [torch.empty(128, 128, dtype=torch.int64, device=dev) for _ in range(slices)]
        ys = [torch.empty(128, 128, device=dev) for _ in range(slices)]
    enc_t = efl.lib.BatchTables(xs, Ms, Es)
    dec_t = efl.lib.BatchTables(Ms, Es, ys)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    flags = 1 if efl.lib.flush_denormal() else 0

    def batched():
        efl.lib.encode_batched_into(enc_t, 1, False, sh)
        efl.lib.decode_batched_into(dec_t, 1, flags, sh)

    def naive():
        for x, M, E in zip(xs, Ms, Es):
            lib.efl_fxp_encode(x.data_ptr(), 1, M.data_ptr(), E.data_ptr(), elems, 0, sh)
        for M, E, y in zip(Ms, Es, ys):
            lib.efl_fxp_decode(M.data_ptr(), E.data_ptr(), y.data_ptr(), 1, elems, elems, flags, sh)

    def wall(fn, k):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / k

    for y in ys:
        y.zero_()
    t_b = wall(batched, max(10, steps))
    # every slice compared bit for bit (FTZ: the identity on randn's bit patterns), on the device
    ok = bool(torch.equal(torch.stack(xs).view(torch.int32), torch.stack(ys).view(torch.int32)))
    # per-launch durations: a second pass with HIP events around each launch on the launch stream
    reps = max(10, steps)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
    for e in evs:
        e[0].record(stream)
        efl.lib.encode_batched_into(enc_t, 1, False, sh)
        e[1].record(stream)
        efl.lib.decode_batched_into(dec_t, 1, flags, sh)
        e[2].record(stream)
    torch.cuda.synchronize(dev)
    k_enc = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    k_dec = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    kbytes = BYTES_PER_ELEM_KERNEL * slices * elems
    nbytes = slices * elems * 4
    out = {"workload": f"config 3: 4096 x 64 KiB fp32 slices [128,128] ({layout}), batched encode+decode",
           "GiBs": round(nbytes / GIB / t_b, 2), "ms": round(t_b * 1e3, 4),
           "hbm_frac": round(2 * kbytes / t_b / 1e9 / PEAK_HBM_GBS, 4),
           "kernels_ms": {"encode": round(k_enc, 4), "decode": round(k_dec, 4)},
           "kernels_hbm_frac": {"encode": round(kbytes / (k_enc * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                                "decode": round(kbytes / (k_dec * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)},
           "tile_lanes_pairs": {"encode": list(efl.lib.batched_tile("encode")),
                                "decode": list(efl.lib.batched_tile("decode"))},
           "table_entries": {"encode": enc_t.count, "decode": dec_t.count},
           "launches": {"batched": 2}, "roundtrip_ok": ok, "roundtrip_checked": "every slice, bit for bit"}
    if layout == "separate":
        t_n = wall(naive, 3)
        out.update({"naive_per_slice_ms": round(t_n * 1e3, 3), "naive_GiBs": round(nbytes / GIB / t_n, 3)})
        out["launches"]["naive"] = 2 * slices
    return out


def pinned_path(efl, dev, x_dev, reps=3):
    """The north_star's rate including copies: the tensor starts and ends in pinned host memory
    (the communicator's send/recv buffers). Encrypt leg: pinned fp32 -> H2D -> encode -> D2H ->
    pinned M, E; decrypt leg: pinned M, E -> H2D -> decode -> D2H -> pinned fp32, each a chunked
    pipeline over three streams (efl.framework.host_pipeline)."""
    from efl.framework.host_pipeline import PinnedCodecPipeline
    pipe = PinnedCodecPipeline(dev)
    x = x_dev.reshape(-1).cpu().pin_memory()
    n = x.numel()
    M = torch.empty(n, dtype=torch.int64, pin_memory=True)
    E = torch.empty(n, dtype=torch.int64, pin_memory=True)
    y = torch.empty(n, dtype=torch.float32, pin_memory=True)
    t_enc, t_dec = [], []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        pipe.encode(x, out=(M, E))
        t1 = time.perf_counter()
        pipe.decode(M, E, torch.float32, out=y)
        t2 = time.perf_counter()
        if r:
            t_enc.append(t1 - t0)
            t_dec.append(t2 - t1)
    ok = bool(torch.equal(x.view(torch.int32), y.view(torch.int32)))
    te, td = float(np.median(t_enc)), float(np.median(t_dec))
    gib = n * 4 / GIB
    return {"encrypt_GiBs": round(gib / te, 3), "decrypt_GiBs": round(gib / td, 3),
            "encrypt_decrypt_GiBs": round(gib / (te + td), 3),
            "encrypt_ms": round(te * 1e3, 2), "decrypt_ms": round(td * 1e3, 2),
            "pcie_bytes_per_leg": {"encrypt": {"h2d": n * 4, "d2h": n * 16},
                                   "decrypt": {"h2d": n * 16, "d2h": n * 4}},
            "chunk_elems": pipe.chunk, "buffers": pipe.nbuf, "roundtrip_bit_exact": ok,
            "how": "pinned host in/out, H2D | codec | D2H on three HIP streams, median of 3"}


# ------------------------------------------------------------------------------------ Stage P
# v_mad_u64_u32 issue rate measured on MI355X with every CU busy, in the shape of a Montgomery row
# (24 64-bit accumulators, one uniform multiplier): 3.17e13 lane-ops/s (tools/valu_probe.hip ->
# profiles/r01/valu_probe.jsonl). Every limb product of a Montgomery multiplication is one such
# instruction. `achieved` counts the algorithm's 32x32-bit limb products (radix-independent work),
# `limb_products_per_s` the instructions the kernel really issues (radix-2^28 decryption issues
# (32/28)^2 more, smaller ones).
MAD_U64_U32_PEAK = 3.1722e13
# (label, n_bytes, a_bytes, group_size, elements): the paillier_mnist example key
# (efls-train/python/efl/example/paillier_mnist/follower_dense.py:39, a_bytes = n_bytes/2 as
# paillier.py:175-176) and the reference default key (paillier.cc:799-805 / paillier.py:173-176)
STAGE_P_KEYS = [("example 1024-bit n, group_size 10", 128, 64, 10, 262144),
                ("example 1024-bit n, group_size 10, MNIST activation [256, 392]", 128, 64, 10, 256 * 392),
                ("default 4096-bit n, group_size 1", 512, 256, 1, 65536)]


def _mont_macs(L, squarings, multiplies, cios_squarings=False):
    """Limb MACs of Montgomery products over L limbs: 2 L^2 per multiply; a squaring forms each cross
    product once (L (L + 1) / 2) plus the L^2 of the reduction, as the one-lane kernels do (sliced28.h
    sqr_fips1). cios_squarings counts 2 L^2 per squaring instead: what the multi-lane families issue."""
    sq = 2 * L * L if cios_squarings else L * (L + 1) // 2 + L * L
    return 2 * L * L * multiplies + sq * squarings


DEC_WINDOW = 5     # csrc/paillier_sliced.hip kDecWin (efl_pl_tune(ln, 2, 1), the default)


def window_products(e: int, w: int = DEC_WINDOW):
    """(squarings, multiplies) of the sliced decryption's sliding-window exponentiation by e
    (windows of up to w bits ending in a 1 bit, left to right) including its odd-power table
    (1 squaring + 2^(w-1) - 1 multiplies), walked exactly as m_func does."""
    def bit(i):
        return (e >> i) & 1
    b = e.bit_length() - 1
    j = max(b - w + 1, 0)
    while not bit(j):
        j += 1
    b = j - 1
    sq, mul = 1, (1 << (w - 1)) - 1
    while b >= 0:
        if not bit(b):
            sq += 1
            b -= 1
            continue
        j = max(b - w + 1, 0)
        while not bit(j):
            j += 1
        sq += b - j + 1
        mul += 1
        b = j - 1
    return sq, mul


def stage_p(args):
    import random
    import efl
    from efl.privacy import paillier_cipher as pc
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    cpu_keys = {}
    # In production the key owner (sender: CRT sub-tables) and the public-key holder (receiver: the
    # n^2 table) are different processes, each under its own 4 GiB process-wide table budget. This
    # report measures both paths of one key in one process, so it gives the process the sum: each
    # path then runs with the table its own process would build.
    pc.table_budget(2 * pc.TABLE_MAX_BYTES)
    for label, n_bytes, a_bytes, g, N in STAGE_P_KEYS:
        n, hs, p, q = pc.generate_keypair_ints(n_bytes, 24, random.Random(n_bytes))
        kp = efl.paillier.Keypair(seed=7)
        torch.cuda.synchronize(dev)
        t_key = time.perf_counter()
        kp.set_keys_ints(n, hs, a_bytes, g, p, q, n_bytes)     # key block (the owner's n^2 table deferred)
        torch.cuda.synchronize(dev)
        t_key = time.perf_counter() - t_key
        k = kp.key
        t_tab = time.perf_counter()
        k.ensure_table()          # the n^2 table the public-key path walks (the "encrypt" row)
        torch.cuda.synchronize(dev)
        t_tab = time.perf_counter() - t_tab
        W = k.table_window
        gen = torch.Generator(device=dev).manual_seed(0)
        m = torch.randint(-2**40, 2**40, (N,), dtype=torch.int64, device=dev, generator=gen)
        ct = torch.empty((N, k.lc), dtype=torch.int32, device=dev)
        mag = torch.empty((N, k.ln), dtype=torch.int32, device=dev)
        neg = torch.empty(N, dtype=torch.int8, device=dev)

        def enc():
            efl.lib.check(lib.efl_pl_encrypt(*k.args(), m.data_ptr(), None, ct.data_ptr(), N, 7, 0, sh))

        def dec():
            efl.lib.check(lib.efl_pl_decrypt(*k.args(), ct.data_ptr(), mag.data_ptr(), neg.data_ptr(), N, sh))

        # the key owner's encryption (KeyBlock.crt_keys): hs^(a') mod p^2 and mod q^2 through their
        # own fixed-base tables, Garner join (efl_pl_crt_join), then g(m) hsa mod n^2
        torch.cuda.synchronize(dev)
        t_crt = time.perf_counter()
        subs = k.crt_keys()
        torch.cuda.synchronize(dev)
        t_crt = time.perf_counter() - t_crt
        fns = [("encrypt", enc), ("decrypt", dec)]
        if subs:
            ct_crt = torch.empty_like(ct)

            def enc_crt():
                # the key context's route for the owner (efl_pl_ctx_encrypt): both walks start from
                # each element's (y^2)^-1 g(m) and the CRT join is the ciphertext (round 5)
                efl.lib.check(lib.efl_pl_ctx_encrypt(k.ctx, m.data_ptr(), None, ct_crt.data_ptr(), N, 7, 0, 0, sh))
            fns.append(("encrypt_crt", enc_crt))
        times = {}
        for name, fn in fns:
            for _ in range(max(1, args.warmup // 5)):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 3
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            e1.synchronize()
            times[name] = e0.elapsed_time(e1) / reps * 1e-3
        got = kp.decrypt(pc.CipherTensor(ct[:512], (512,), k), dtype=torch.int64)
        if not torch.equal(got, m[:512]):
            raise SystemExit("bench: Paillier round trip is wrong")
        if subs and not torch.equal(ct_crt, ct):
            raise SystemExit("bench: CRT encryption differs from the public-key path")
        # work per element (exact for decrypt's uniform exponents; expected value for the table)
        pm1, qm1 = p - 1, q - 1
        dec_window = lib.efl_pl_tune(k.ln, 2, -1) == 1 and pc.kernel_slicing(k.ln, True) > 0
        dec_ops = [window_products(e) if dec_window else (e.bit_length() - 1, bin(e).count("1") - 1)
                   for e in (pm1, qm1)]
        dec_macs = sum(_mont_macs(k.ln, sq, mul) for sq, mul in dec_ops)
        # encryption: one table product per non-zero W-bit window of a' (expected count), + g(m)
        rows = -(-8 * a_bytes // W)
        enc_macs = _mont_macs(k.lc, 0, rows * (1 - 2.0 ** -W) + 1)
        res = {}
        if subs:
            res["encrypt_crt"] = stage_p_crt(k, subs, a_bytes, N, times["encrypt_crt"], times["encrypt"], t_crt)
        for name, macs in (("encrypt", enc_macs), ("decrypt", dec_macs)):
            per_s = N / times[name]
            fam = pc.kernel_slicing(k.ln, name == "decrypt")
            issued = macs
            if name == "decrypt" and fam:     # sliced decryption exponentiates in radix 2^28
                G = k.ln // fam               # lanes per number: one-lane numbers square by product scanning
                L28 = pc.limbs28_total(k.ln, G)
                issued = sum(_mont_macs(L28, sq, mul, cios_squarings=G > 1) for sq, mul in dec_ops)
            if name == "encrypt" and k.desc.off_table28 >= 0:   # the radix-2^28 table serves encryption
                issued = _mont_macs(k.desc.n2_28_len, 0, rows * (1 - 2.0 ** -W) + 1)
            res[name] = {"elements_per_s": round(per_s), "ms": round(times[name] * 1e3, 3),
                         "macs_per_element": int(macs),
                         "method": ("sliding window w=%d" % DEC_WINDOW if dec_window else "binary")
                         if name == "decrypt" else "fixed-base table, W=%d" % W,
                         "roofline": {"bound": "valu", "achieved": round(per_s * macs / 1e12, 3),
                                      "peak": round(MAD_U64_U32_PEAK / 1e12, 3), "unit": "TMAC/s",
                                      "frac": round(per_s * macs / MAD_U64_U32_PEAK, 4),
                                      "limb_products_per_s": round(per_s * issued / 1e12, 3),
                                      "issue_frac": round(per_s * issued / MAD_U64_U32_PEAK, 4)},
                         "kernel_family": fam}
        out = {"metric": "Paillier elements/s on 1 GPU (encrypt with fresh randomness, CRT decrypt)",
               "stage": "P", "config": {"key": label, "n_bits": 8 * n_bytes, "a_bits": 8 * a_bytes,
                                        "group_size": g, "table_window": W, "elements": N},
               "key_setup_ms": round(t_key * 1e3, 1), "public_table_setup_ms": round(t_tab * 1e3, 1),
               "table": {"rows": k.desc.table_rows, "cols": k.desc.table_cols,
                         "MiB": round(k.block_bytes / 2**20, 1)},
               "unit": "elements/s", "higher_is_better": True, "dtype": "u32 limbs",
               "data": "synthetic int64 mantissas in [-2^40, 2^40), deterministic key", **res,
               "library": efl.lib.version(), "cpu_baseline": None}
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = stage_p_cpu(n_bytes, a_bytes, g, p, q, hs, args.cpu_threads, cpu_keys)
            for name in ("encrypt", "decrypt"):
                out[name]["vs_cpu"] = round(out[name]["elements_per_s"] / out["cpu_baseline"][name], 1)
            if "encrypt_crt" in out:      # the same op (PaillierEncrypt) for the key owner
                out["encrypt_crt"]["vs_cpu"] = round(out["encrypt_crt"]["elements_per_s"] /
                                                     out["cpu_baseline"]["encrypt"], 1)
        if "MNIST" in label:
            out["matmul"] = stage_p_matmul(args, efl, pc, kp, lib, sh, stream, dev)
        out["table_budget"] = dict(zip(("budget", "in_use"), pc.table_budget()))
        print(json.dumps(out), flush=True)
        k.close()      # the next key's tables are sized against the process-wide budget


def stage_p_crt(k, subs, a_bytes, N, t, t_public, t_setup):
    """The key owner's encryption by CRT (efl_pl_ctx_encrypt): algorithmic limb MACs = the two
    half-length fixed-base walks (one product per non-zero window of each sub-table), each walk's
    start (y^2)^-1 g(m) (one product mod x^2, plus three Montgomery steps for |m| (n mod x^2)) and the
    join (the plain products q^2 yp and p^2 yq). Round 4's route multiplied g(m) into the join's
    hsa R by one product mod n^2 instead of the two start products."""
    macs = sum(_mont_macs(sk.lc, 0, -(-8 * a_bytes // sk.table_window) * (1 - 2.0 ** -sk.table_window))
               + _mont_macs(sk.lc, 0, 1) + 3 * 2 * sk.lc for sk in subs) + 2 * k.ln * k.ln
    issued = sum(_mont_macs(sk.desc.n2_28_len if sk.desc.off_table28 >= 0 else sk.lc, 0,
                            -(-8 * a_bytes // sk.table_window) * (1 - 2.0 ** -sk.table_window)) for sk in subs)
    per_s = N / t
    from efl import lib as _l
    paired = (subs[0].ln == 16 and pc_family(subs[0].ln) == 32 and _l.raw().efl_pl_tune(16, 5, -1) != 1)
    route = ("an element's two walks in one wave, start and CRT join in the kernel, last round split"
             if paired else "a walk launch per sub-key, then the CRT join launch")
    return {"elements_per_s": round(per_s), "ms": round(t * 1e3, 3), "vs_public_path": round(t_public / t, 3),
            "macs_per_element": int(macs),
            "method": "(y^2)^-1 g(m) hs^a' mod p^2 and mod q^2 (W=%d/%d), CRT join = the ciphertext; %s"
                      % (subs[0].table_window, subs[1].table_window, route),
            "roofline": {"bound": "valu", "achieved": round(per_s * macs / 1e12, 3),
                         "peak": round(MAD_U64_U32_PEAK / 1e12, 3), "unit": "TMAC/s",
                         "frac": round(per_s * macs / MAD_U64_U32_PEAK, 4),
                         "issue_frac_walks": round(per_s * issued / MAD_U64_U32_PEAK, 4)},
            "sub_key_setup_ms": round(t_setup * 1e3, 1),
            "sub_tables_MiB": round(sum(sk.block_bytes for sk in subs) / 2**20, 1),
            "kernel_family": pc_family(subs[0].ln)}


def pc_family(ln):
    from efl.privacy import paillier_cipher as pc
    return pc.kernel_slicing(ln, False)


# the receiver's forward product of the paillier_mnist example (paillier_layer.py:136:
# x @ fixedpoint_encode(w, decrease_precision=True)): x [256, 28*14] encrypted by the sender
# (leader_dense.py:44 / follower_dense.py:23 batch 256), w [392, 128] glorot-uniform
STAGE_P_MATMUL = (256, 392, 128)
MATMUL_WINDOW = 5   # csrc/paillier_sliced.hip kMatWin


def stage_p_matmul(args, efl, pc, kp, lib, sh, stream, dev):
    """PaillierMatmul (paillier.cc:941-1051) on the MNIST receiver shape: the efl_pl_matmul kernel
    (all u*w outputs, every term's x^|y| and 2^(exponent - min) squarings, both sign products) timed
    with HIP events; the plaintext of the first outputs checked exactly after the caller's
    invert + add finish."""
    u, v, w = STAGE_P_MATMUL
    k = kp.key
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    e0.record(stream)
    for _ in range(reps):
        mm()
    e1.record(stream)
    e1.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    # Montgomery products the kernel executes, counted from the data (per group, ignoring lanes a
    # wave masks off): x R once per x element; per output and sign, Straus over the terms of that
    # sign: (top level - 1) shared squarings, popcount(|y|) multiplies per term less the first (a
    # copy), one conversion out. `per_term_products` is one square-and-multiply per term instead
    # (bits-1 + popcount-1 + d, a conversion in and a multiply into the product), the schedule the
    # reference's powm-per-term loop (paillier.cc:1015-1032) has.
    xe_h, ym_h, ye_h = (a.cpu().numpy().astype(np.int64) for a in (xe, ym, ye))
    ex = xe_h[:, :, None] + ye_h[None, :, :]                  # [u, v, w]
    d = ex - ex.min(axis=1, keepdims=True)
    nz = ym_h != 0
    ay = np.abs(ym_h)
    bits = np.zeros(ym_h.shape, dtype=np.int64)
    pop = np.zeros(ym_h.shape, dtype=np.int64)
    for q in range(63):
        hit = (ay >> q) & 1
        pop += hit
        bits = np.where(hit == 1, q + 1, bits)
    # multiplies per term: one per right-to-left window of MATMUL_WINDOW bits starting at a 1 bit
    # (csrc/paillier_sliced.hip k_wmask / kMatWin), not one per set bit
    nwin = np.zeros(ym_h.shape, dtype=np.int64)
    rest = ay.copy()
    while rest.any():
        low = rest & -rest                                     # lowest set bit
        has = rest != 0
        nwin += has
        rest = np.where(has, rest & ~((low << MATMUL_WINDOW) - 1), 0)
    L = k.lc
    fam = pc.kernel_slicing(k.ln, False)
    # the term split of run_matmul28 (csrc/paillier_sliced.hip): each split squares on its own
    S, G = 1, (L // fam if fam else 1)
    fixed = lib.efl_pl_tune(k.ln, 3, -1)       # efl_pl_tune(ln, 3, S): a fixed split, 0 = per launch
    if fixed > 0:
        while 2 * S <= fixed and 2 * S <= v:
            S *= 2
    else:
        waves = 2 if fam >= 32 else 4                    # k_matmul28's waves per SIMD
        while 2 * S <= 8 and 2 * S <= v and u * w * G * S < 256 * 4 * 64 * waves:
            S *= 2
    # x R and its odd powers (1 squaring + 2^(w-1) - 1 products); combining the partials + conversion out
    products = u * v * (1 + (1 << (MATMUL_WINDOW - 1))) + (2 * S * u * w if S > 1 else 0)
    squarings = u * v                          # of `products`: the x^2 of each odd-power table, the levels below
    for sp in range(S):
        j0, j1 = v * sp // S, v * (sp + 1) // S
        for sgn in (1, -1):
            mask = np.zeros_like(nz)
            mask[j0:j1] = nz[j0:j1] & (np.sign(ym_h[j0:j1]) == sgn)
            top = np.where(mask[None, :, :], d + bits[None, :, :], 0).max(axis=1)    # [u, w]
            started = mask.any(axis=0)[None, :].repeat(u, axis=0)
            # squarings below the top level, multiplies less the first (a copy), one conversion out
            lv = int(np.maximum(top - 1, 0)[started].sum())
            squarings += lv
            products += lv + u * int(nwin[mask].sum()) - int(started.sum())
            if S == 1:
                products += int(started.sum())
    per_term = u * int((bits + pop)[nz].sum()) + int((d * nz[None, :, :]).sum()) + 2 * u * w
    L_issued = k.desc.n2_28_len if (fam and k.desc.off_table28 >= 0) else L
    macs = _mont_macs(L, squarings, products - squarings)
    issued = _mont_macs(L_issued, squarings, products - squarings, cios_squarings=G > 1)
    # the whole op as the layer calls it (kernel + z_neg^-1 + z_pos * z_neg^-1), then a plaintext
    # check of the first outputs: sum_j xm*ym*2^(xe+ye-min), exactly
    xct = pc.CipherTensor(X, (u, v), k)
    kp.matmul(xct, xe, ym, ye)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    zm, zexp = kp.matmul(xct, xe, ym, ye)
    torch.cuda.synchronize(dev)
    t_op = time.perf_counter() - t0
    n_chk = 64
    dec = kp.decrypt(pc.CipherTensor(zm.limbs[:n_chk], (n_chk,), k), dtype="string").to_ints()
    xm_h = xm.cpu().numpy()
    ze_h = zexp.cpu().numpy().reshape(-1)
    for o in range(n_chk):
        i, q = divmod(o, w)
        want = sum((int(xm_h[i, j]) * int(ym_h[j, q])) << int(ex[i, j, q] - ze_h[o]) for j in range(v))
        if dec[o] != want:
            raise SystemExit(f"bench: PaillierMatmul output {o} is wrong")
    res = {"shape": [u, v, w], "outputs_per_s": round(u * w / t, 1), "ms": round(t * 1e3, 3),
           "op_ms": round(t_op * 1e3, 3), "op_outputs_per_s": round(u * w / t_op, 1),
           "term_splits": S, "montgomery_products_per_output": round(products / (u * w), 1),
           "per_term_products_per_output": round(per_term / (u * w), 1),
           "roofline": {"bound": "valu", "achieved": round(macs / t / 1e12, 3),
                        "peak": round(MAD_U64_U32_PEAK / 1e12, 3), "unit": "TMAC/s",
                        "frac": round(macs / t / MAD_U64_U32_PEAK, 4),
                        "limb_products_per_s": round(issued / t / 1e12, 3),
                        "issue_frac": round(issued / t / MAD_U64_U32_PEAK, 4)},
           "kernel_family": fam, "cpu_baseline": None}
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = stage_p_matmul_cpu(kp, xe_h, ym_h, ye_h, v, w, args.cpu_threads)
        res["vs_cpu"] = round(res["op_outputs_per_s"] / res["cpu_baseline"]["value"], 1)   # whole op vs whole op
    return res


def stage_p_matmul_cpu(kp, xe, ym, ye, v, w, threads):
    """The reference's PaillierMatmul compute (oracle/paillier_gmp.c pl_gmp_matmul_bench) on the
    first rows of the same exponents and weights, sized for a few seconds on `threads` threads."""
    import ctypes
    from oracle import fxp, paillier as P
    L = fxp.lib()
    L.pl_gmp_matmul_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + \
        [ctypes.POINTER(ctypes.c_double)]
    n_hex = P.hx(kp.key.n).encode()
    t = (ctypes.c_double * 2)()
    ym_c, ye_c = np.ascontiguousarray(ym), np.ascontiguousarray(ye)
    rows = 1
    while True:
        xe_c = np.ascontiguousarray(xe[:rows])
        L.pl_gmp_matmul_bench(n_hex, xe_c.ctypes.data, ym_c.ctypes.data, ye_c.ctypes.data, rows, v, w, threads, t)
        if t[0] + t[1] > 2.0 or rows >= xe.shape[0]:
            break
        rows = min(xe.shape[0], rows * max(2, int(3.0 / max(t[0] + t[1], 1e-3))))
    return {"value": round(rows * w / (t[0] + t[1]), 1), "unit": "outputs/s", "cores": threads, "kind": "port",
            "sample": f"{rows} rows x {w} outputs ({rows * v} ciphertext inversions, serial as paillier.cc:994-999, "
                      f"then GMP powm per term over {threads} threads)"}


def stage_p_cpu(n_bytes, a_bytes, g, p, q, hs, threads, cache):
    """The reference's GMP path (oracle/paillier_gmp.c pl_gmp_bench) on a bounded sample sized for
    a few seconds per op on `threads` host threads."""
    import ctypes
    from oracle import fxp, paillier as P
    L = fxp.lib()
    L.pl_gmp_bench.argtypes = [ctypes.c_char_p] * 3 + [ctypes.c_uint, ctypes.c_uint, ctypes.c_longlong,
                                                        ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    key = (n_bytes, a_bytes, g)
    if key in cache:
        return cache[key]
    t = (ctypes.c_double * 2)()
    count = threads * 4
    while True:
        L.pl_gmp_bench(P.hx(p).encode(), P.hx(q).encode(), P.hx(hs).encode(), 8 * a_bytes, g, count, threads, t)
        if t[1] > 2.0 or count >= 1 << 20:
            break
        count = min(1 << 20, int(count * min(16.0, max(2.0, 4.0 / max(t[1], 1e-3)))))
    cache[key] = {"encrypt": round(count / t[0], 1), "decrypt": round(count / t[1], 1), "unit": "elements/s",
                  "cores": threads, "kind": "port",
                  "sample": f"{count} elements, GMP mpz path of paillier.cc:103-131 / :296-312 with the "
                            f"fbpowm table of gmp_utils.cc:56-144 built once, {threads} threads"}
    return cache[key]


def config5(timeout_s=240):
    """BASELINE config 5 (tools/bench_e2e.py): two processes on this box, 256 MiB fp32 from pinned
    host memory through the pipelined FixedPointHook encode leg, gRPC loopback (2 x 512 MiB messages),
    the pipelined decode leg, back to host; rate including every copy. Run as a child process so a
    failure there cannot take the headline line with it (the error is reported instead)."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_e2e.py")], capture_output=True,
                           text=True, timeout=timeout_s)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return {"error": f"rc {r.returncode}: {r.stderr.strip()[-300:]}"}
        return json.loads(lines[-1])
    except (subprocess.TimeoutExpired, OSError, ValueError) as e:
        return {"error": repr(e)[:300]}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`bench.py --gpus N` run without a torchrun environment: start the N ranks as children
    (torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1) and relay rank 0's JSON
    line. This process never touches the GPU (torch.cuda.device_count() does not initialise it on
    this image) and never execs: the children are fresh processes. Exit status: the children's, or
    3 when the world that ran is not the one asked for."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for ln in proc.stdout:                     # progress lines pass through; the JSON line is held
        if ln.startswith("{") and '"metric"' in ln:
            line = ln.strip()
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if rc:
        return rc
    if line is None:
        print("bench: rank 0 printed no result line", file=sys.stderr)
        return 3
    out = json.loads(line)
    out["launcher"] = f"bench.py --gpus {args.gpus}: torch.distributed.run children, rendezvous 127.0.0.1"
    print(json.dumps(out), flush=True)
    if out.get("n_gpus") != args.gpus:
        print(f"bench: asked for {args.gpus} ranks, {out.get('n_gpus')} ran", file=sys.stderr)
        return 3
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.stage == "p":
        if args.cpu_threads is None:
            args.cpu_threads = usable_cores()[0]
        return stage_p(args)
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args, argv)
    if int(env_world or 1) != args.gpus:
        # checked before any GPU or process-group call: a run labelled N must be N ranks
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        return 3
    from efl import distributed as edist
    world, rank, local, dev_index, backend = edist.init_from_env(args.backend)
    import efl
    dev = efl.lib.require_gpu()
    lib = efl.lib.raw()
    for kv in filter(None, args.tune.split(",")):
        k, v = (int(s) for s in kv.split("="))
        efl.lib.check(min(0, lib.efl_fxp_tune(k, v)))

    seed, bcast_us = broadcast_seed(world, rank)
    n = args.rows * COLS
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(args.rows, COLS, device=dev, generator=g)
    M = torch.empty(x.shape, dtype=torch.int64, device=dev)
    E = torch.empty(x.shape, dtype=torch.int64, device=dev)
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    ftz = efl.lib.flush_denormal()
    flags = 1 if ftz else 0
    xp, Mp, Ep, yp = x.data_ptr(), M.data_ptr(), E.data_ptr(), y.data_ptr()
    enc, dec = lib.efl_fxp_encode, lib.efl_fxp_decode

    def step():
        rc = enc(xp, 1, Mp, Ep, n, 0, sh) or dec(Mp, Ep, yp, 1, n, n, flags, sh)
        if rc:
            efl.lib.check(rc)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness gate before timing: with FTZ the round trip is the identity on every bit
    # pattern torch.randn makes (no denormals; +-0.0 -> +-0.0)
    if not torch.equal(y.view(torch.int32), x.view(torch.int32)) if ftz else \
            not torch.equal(y[x != 0], x[x != 0]):
        raise SystemExit("bench: encode/decode round trip is wrong")

    # ---- timed region: K steps, nothing else -------------------------------------------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # ---- per-kernel durations: a second pass of K steps with HIP events on the launch stream -
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for k in range(args.steps):
        evs[k][0].record(stream)
        efl.lib.check(enc(xp, 1, Mp, Ep, n, 0, sh))
        evs[k][1].record(stream)
        efl.lib.check(dec(Mp, Ep, yp, 1, n, n, flags, sh))
        evs[k][2].record(stream)
    torch.cuda.synchronize()
    t_enc = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))   # ms
    t_dec = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    # this rank's own kernel times and roofline fractions, before the max over ranks
    own = edist.rank_kernel_report(t_enc, t_dec, elapsed / args.steps * 1e3, n, BYTES_PER_ELEM_KERNEL,
                                   PEAK_HBM_GBS)
    if world > 1:
        elapsed, t_enc, t_dec = edist.all_reduce_max([elapsed, t_enc, t_dec])

    ms_per_step = elapsed / args.steps * 1e3
    value = world * (n * 4) / GIB / (elapsed / args.steps)
    # every rank reports the device it really ran on (PCI location) and its own kernel times,
    # gathered after the timed region
    rank_devices = edist.gather_rank_devices({**edist.rank_device_info(rank, dev), **own})

    # practical peak: device-to-device copy of the same byte volume as one kernel
    copy_gbs = None
    if rank == 0:
        buf_a = torch.empty(n * 5 // 4, dtype=torch.float64, device=dev)
        buf_b = torch.empty_like(buf_a)
        for _ in range(3):
            buf_b.copy_(buf_a)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for _ in range(10):
            buf_b.copy_(buf_a)
        c1.record(stream)
        torch.cuda.synchronize()
        copy_gbs = 2 * buf_a.numel() * 8 / (c0.elapsed_time(c1) / 10 * 1e-3) / 1e9
        del buf_a, buf_b

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    dominant = "encode" if t_enc >= t_dec else "decode"
    t_dom = max(t_enc, t_dec) * 1e-3
    achieved = BYTES_PER_ELEM_KERNEL * n / t_dom / 1e9
    traffic, traffic_source = None, None
    tr = load_traffic()
    if tr and tr.get("elements") == n and dominant in tr.get("kernels", {}):
        traffic = tr["kernels"][dominant].get("hbm_bytes_per_launch")
        # a recorded measurement, not one of this run: say which
        traffic_source = ("profiles/pmc_traffic.json (not measured in this run): " +
                          tr.get("command", "rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py") +
                          (f"; {tr['profile_dir']}" if tr.get("profile_dir") else "") +
                          (f"; library {tr['library']}" if tr.get("library") else ""))
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic: torch.randn fp32 on device, generator seed = rank",
        "config": {"workload": "config 2: single 256 MiB fp32 tensor [65536,1024] per GPU, "
                               "device-resident ConvertToFixedPoint + FixedPointToFloatPoint",
                   "elements_per_gpu": n, "decrease_precision": False, "decode_ftz": ftz,
                   "parallelism": f"element-wise shard, {world} x 256 MiB, {backend if world > 1 else 'no'} "
                                  f"seed broadcast"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_source, "kernel": dominant,
                     "algorithmic_bytes_per_launch": BYTES_PER_ELEM_KERNEL * n,
                     "timing": "HIP events around each launch, second pass of K steps after the timed region"},
        "kernels_ms": {"encode": round(t_enc, 4), "decode": round(t_dec, 4)},
        "step_roofline_frac": round(2 * BYTES_PER_ELEM_KERNEL * n / (ms_per_step * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
        "d2d_copy_GBs": round(copy_gbs, 1) if copy_gbs else None,
        "seed_broadcast_us": round(bcast_us, 2),
        "backend": backend if world > 1 else None,
        "devices_used": edist.distinct_devices(rank_devices),
        "devices_visible": torch.cuda.device_count(),
        "rank_devices": rank_devices,
        "library": efl.lib.version(),
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_extras:
        del M, E, y
        out["config3"] = config3(efl, dev, args.steps)
        out["config3"]["views"] = config3(efl, dev, args.steps, layout="views")
        out["pinned_path"] = pinned_path(efl, dev, x)
        out["config5"] = config5()
    if world == 1 and not args.no_cpu_baseline:
        threads, how = (args.cpu_threads, "--cpu-threads") if args.cpu_threads else usable_cores()
        out["cpu_baseline"] = cpu_baseline(x, threads, how, ftz)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
