#!/usr/bin/env python3
"""The gRPC leg of BASELINE config 5 alone (no GPU): the follower sends two int64 tensors of
`--mib` MiB each (the hook's mantissa and exponent) per step through efl.Communicator, the leader
receives both (payload views, as FixedPointHook reads them); wall per step from the follower's
first send to the leader's second recv. `--channels` sets the client connections (EFL_CHANNELS).
Prints one JSON line.

    python tools/grpc_probe.py [--mib 512] [--reps 3] [--channels 1 2 4]
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def party(role, my, peer, mib, reps, channels, q):
    import torch
    from efl.framework.communicator import Communicator
    c = Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}", default_timeout_milliseconds=600000,
                     connect_retry_seconds=0.2, channels=channels)
    c.initialize()
    n = mib * (1 << 20) // 8
    M = torch.arange(n, dtype=torch.int64)
    E = torch.full((n,), -7, dtype=torch.int64)
    times = []
    for r in range(reps + 1):
        if role == "follower":
            t0 = time.monotonic()
            hs = [c.send("x_mantissa", M), c.send("x_exponent", E)]
            for h in hs:
                h.result()
            times.append(t0)
        else:
            a = c._recv_raw("x_mantissa", readonly=True)
            b = c._recv_raw("x_exponent", readonly=True)
            times.append(time.monotonic())
            assert a.numel() == n and int(a[-1]) == n - 1 and int(b[0]) == -7
        c.add_step()
    q.put((role, times[1:]))
    c.shutdown()


def run(mib, reps, channels):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    ps = [ctx.Process(target=party, args=("leader", pl, pf, mib, reps, channels, q)),
          ctx.Process(target=party, args=("follower", pf, pl, mib, reps, channels, q))]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=900) for _ in ps)
    for p in ps:
        p.join(60)
    walls = sorted(e - s for s, e in zip(res["follower"], res["leader"]))
    return walls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--channels", type=int, nargs="+", default=[1, 2])
    a = ap.parse_args()
    for ch in a.channels:
        walls = run(a.mib, a.reps, ch)
        med = walls[len(walls) // 2]
        print(json.dumps({"probe": "gRPC leg of config 5 (two int64 messages per step)", "mib_per_message": a.mib,
                          "channels": ch, "wall_ms": [round(w * 1e3, 1) for w in walls],
                          "GBs": round(2 * a.mib * (1 << 20) / med / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
