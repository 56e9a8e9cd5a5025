"""Multi-GPU layout of the forward-encryption path (one process per GPU, torch.distributed).

The path is element-wise: a tensor is cut into contiguous, 256-byte-aligned
element ranges, one per rank, and every rank transforms its range with no payload exchange. The
only collective is a broadcast from rank 0 of the key material every rank needs — the 32-byte seed
of the per-element randomness counter stream and, once a Paillier key exists, the public key —
RCCL over xGMI on MI355X (`nccl` backend), gloo on CPU.

Each rank's counter base is the global element offset of its range, so results do not depend on
the number of GPUs (tests/test_distributed.py checks that invariant).
"""
from __future__ import annotations

import json
import os

import torch
import torch.distributed as dist

ALIGN_BYTES = 256


def shard_range(n: int, world: int, rank: int, elem_bytes: int = 4):
    """[start, end) of `rank`'s contiguous share of n elements; boundaries are multiples of
    256 bytes so every shard keeps 16-byte-per-lane vector access."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    quantum = max(1, ALIGN_BYTES // elem_bytes)
    units = (n + quantum - 1) // quantum
    per = units // world
    extra = units % world
    s_units = rank * per + min(rank, extra)
    e_units = s_units + per + (1 if rank < extra else 0)
    return min(n, s_units * quantum), min(n, e_units * quantum)


def _device_for(group=None):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_key_material(seed: bytes | None = None, public_key: dict | None = None, src: int = 0,
                           group=None):
    """Broadcast {seed (32 B), public key} from `src`; returns (seed, public_key) on every rank.
    One length broadcast + one payload broadcast (a few KB; off the critical path)."""
    rank = dist.get_rank(group)
    dev = _device_for(group)
    if rank == src:
        if seed is None:
            seed = os.urandom(32)
        blob = json.dumps({"seed": seed.hex(), "public_key": public_key}).encode()
        n = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    else:
        n = torch.zeros(1, dtype=torch.int64, device=dev)
    dist.broadcast(n, src, group=group)
    buf = torch.zeros(int(n.item()), dtype=torch.uint8, device=dev)
    if rank == src:
        buf.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    dist.broadcast(buf, src, group=group)
    msg = json.loads(bytes(buf.cpu().numpy()).decode())
    return bytes.fromhex(msg["seed"]), msg["public_key"]
