#!/usr/bin/env python3
"""The paillier_mnist example's Paillier dense layer as two federated parties: one training step
(forward + backward) of efl.paillier.sender.dense / efl.paillier.recver.dense at the example shape
(activations [256, 392] -> 128 units, 1024-bit key: efls-train/python/efl/privacy/paillier_layer.py,
the protocol of §5's call sites) over efl.Communicator on loopback. Each party is its own process on
this box, sharing its GPU; the key travels by efl.paillier.Hook.

Per party: the mean wall of `--steps` timed steps after `--warmup`, then ONE extra step with every
cipher op and communicator call synchronised and timed (exclusive times: a matmul's inner invert and
add count under invert / add, a send's hex formatting under send), and how many elements each op
processed. Prints one JSON line per party.

    python tools/bench_layer.py [--steps 3] [--warmup 1] [--kind dense|weight]

--kind weight runs efl.paillier.{sender,recver}.weight instead (paillier_layer.py:209-360): an
element-wise [256, 128] kernel, whose receiver reduces the gradient over rows (one matmul launch).
"""
import argparse
import collections
import functools
import json
import multiprocessing as mp
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

ROWS, FEATURES, UNITS, N_BYTES = 256, 392, 128, 128


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OpTimer:
    """Exclusive wall time per wrapped call (device synchronised on entry and exit)."""

    def __init__(self, sync):
        self.sync = sync
        self.total = collections.defaultdict(float)
        self.calls = collections.Counter()
        self.elems = collections.Counter()
        self.stack = []
        self.on = False

    def wrap(self, obj, attr, name, count=None):
        fn = getattr(obj, attr)

        @functools.wraps(fn)
        def timed(*a, **kw):
            if not self.on:
                return fn(*a, **kw)
            self.sync()
            t0 = time.perf_counter()
            self.stack.append(0.0)
            try:
                return fn(*a, **kw)
            finally:
                self.sync()
                dt = time.perf_counter() - t0
                child = self.stack.pop()
                self.total[name] += dt - child
                if self.stack:
                    self.stack[-1] += dt
                self.calls[name] += 1
                if count is not None:
                    self.elems[name] += count(*a, **kw)
        setattr(obj, attr, timed)


def _numel(x):
    try:
        import math
        if hasattr(x, "numel"):
            return int(x.numel())
        if hasattr(x, "shape"):
            return int(math.prod(x.shape))
    except Exception:
        pass
    return 0


def party(role, my, peer, q, steps, warmup, kind):
    try:
        import torch
        import efl
        from efl.privacy.paillier_cipher import PaillierKeypair
        torch.cuda.init()
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}",
                             default_timeout_milliseconds=600000, connect_retry_seconds=0.2)
        c.initialize()
        kp = efl.paillier.Keypair()
        Role = efl.privacy.Role
        efl.paillier.Hook(kp, c, Role.SENDER if role == "follower" else Role.RECEIVER, "k",
                          n_bytes=N_BYTES).after_create_session()
        g = torch.Generator().manual_seed(0)
        feats = FEATURES if kind == "dense" else UNITS
        x = torch.randn(ROWS, feats, generator=g).cuda()
        dy = torch.randn(ROWS, UNITS, generator=g).cuda()

        def step():
            if role == "follower":     # sender: owns the key and the activations
                xi = x.clone().requires_grad_(True)
                if kind == "dense":
                    out, _ = efl.paillier.sender.dense(xi, kp, c, "l1", UNITS, seed=1)
                else:
                    out, _ = efl.paillier.sender.weight(xi, kp, c, "l1", UNITS, seed=1)
                out.backward(dy)
            else:                      # receiver: holds W
                if kind == "dense":
                    y, _ = efl.paillier.recver.dense(None, kp, c, "l1", (ROWS, FEATURES), UNITS, seed=2)
                else:
                    y, _ = efl.paillier.recver.weight(None, kp, c, "l1", UNITS, seed=2)
                y.backward(dy)
            torch.cuda.synchronize()
            c.add_step()

        for _ in range(warmup):
            step()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        wall = (time.perf_counter() - t0) / steps

        timer = OpTimer(torch.cuda.synchronize)
        cls = PaillierKeypair
        for attr in ("encrypt", "decrypt", "matmul", "add", "invert", "mul_scalar", "mul_exp2", "shift_add",
                     "_cipher"):
            if hasattr(cls, attr):
                timer.wrap(cls, attr, attr if attr != "_cipher" else "hex parse (_cipher)",
                           (lambda self, v, *a, **k: _numel(v)) if attr != "matmul" else
                           (lambda self, xm, xe, ym, ye: int(xe.shape[0]) * int(ym.shape[1])))
        from efl.privacy import paillier as fxp_api
        for attr in ("fixedpoint_encode", "fixedpoint_decode"):
            timer.wrap(fxp_api, attr, attr)
        from efl.privacy import paillier_layer as layer_mod
        timer.wrap(layer_mod, "fixedpoint_encode", "fixedpoint_encode")
        timer.wrap(layer_mod, "_decrypt_decode", "decrypt+decode")
        timer.wrap(c, "_send_raw", "send (serialise, hex)", lambda name, t: _numel(t))
        from efl.framework.communicator import SendHandle
        timer.wrap(SendHandle, "result", "send (wait for the peer's recv)")
        # the pieces of a ciphertext send (exclusive: what is left under "send" is the gRPC hand-off)
        from efl.privacy.paillier_cipher import CipherTensor
        from efl.privacy.hex_tensor import HexTensor
        from efl.framework import wire
        timer.wrap(CipherTensor, "to_hex", "send: hex text (GPU)")
        timer.wrap(HexTensor, "wire_parts", "send: varint lengths")
        timer.wrap(wire, "message_request", "send: request assembly (text D2H into it)")
        sent = [0, 0]                  # serialised request bytes and messages this party sends
        assemble = wire.message_request

        def counted(*a, **kw):
            r = assemble(*a, **kw)
            sent[0] += len(r)
            sent[1] += 1
            return r
        wire.message_request = counted
        timer.wrap(c, "_recv_raw", "recv (wait, parse)")
        timer.on = True
        t1 = time.perf_counter()
        step()
        inst = time.perf_counter() - t1
        timer.on = False
        c.shutdown()
        q.put((role, {"party": "sender (key owner, x)" if role == "follower" else "receiver (W)",
                      "step_ms": round(wall * 1e3, 1), "instrumented_step_ms": round(inst * 1e3, 1),
                      "ops_ms": {k: round(v * 1e3, 2) for k, v in sorted(timer.total.items(), key=lambda kv: -kv[1])},
                      "attributed_frac": round(sum(timer.total.values()) / inst, 3),
                      "calls": dict(timer.calls), "elements": dict(timer.elems),
                      "wire": {"bytes_sent": sent[0], "messages_sent": sent[1]}}, None))
    except BaseException as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((role, None, traceback.format_exc()[-2000:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--kind", choices=("dense", "weight"), default="dense")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    ps = [ctx.Process(target=party, args=("leader", pl, pf, q, a.steps, a.warmup, a.kind)),
          ctx.Process(target=party, args=("follower", pf, pl, q, a.steps, a.warmup, a.kind))]
    for p in ps:
        p.start()
    out, err = {}, None
    for _ in ps:
        role, res, e = q.get(timeout=1200)
        if e:
            err = (role, e)
        out[role] = res
    for p in ps:
        p.join(timeout=60)
    if err:
        raise SystemExit(f"{err[0]} failed:\n{err[1]}")
    # both directions' request bytes of the instrumented step against the slower party's step: the
    # rate the step would need from the transport if nothing else took time
    total = sum(out[r]["wire"]["bytes_sent"] for r in out)
    step_s = max(out[r]["step_ms"] for r in out) / 1e3
    for r in out:
        out[r]["wire"]["both_directions_bytes"] = total
        out[r]["wire"]["both_directions_GBs_over_step"] = round(total / step_s / 1e9, 3)
    for role in ("follower", "leader"):
        print(json.dumps({"bench": f"paillier_mnist {a.kind} layer step, two processes, 1024-bit key",
                          "shape": {"activations": [ROWS, FEATURES if a.kind == "dense" else UNITS], "units": UNITS},
                          **out[role]}), flush=True)


if __name__ == "__main__":
    main()
