"""Multi-GPU layout of the forward-encryption path (one process per GPU, torch.distributed).

The path is element-wise: a tensor is cut into contiguous, 256-byte-aligned
element ranges, one per rank, and every rank transforms its range with no payload exchange. The
only collective is a broadcast from rank 0 of the key material every rank needs — the 32-byte seed
of the per-element randomness counter stream and, once a Paillier key exists, the public key —
RCCL over xGMI on MI355X (`nccl` backend), gloo when ranks share one GPU or run on CPU.

Each rank's counter base is the global element offset of its range, so results do not depend on
the number of GPUs (tests/test_distributed.py and tests/test_distributed_gpu.py check that
invariant, the latter with the HIP kernels under two ranks).
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


def choose_backend(world: int, backend: str | None = None) -> str:
    """RCCL (`nccl`) when every rank has a GPU of its own; gloo when ranks must share a device
    (RCCL refuses two ranks on one GPU) or there is no GPU."""
    if backend:
        return backend
    ndev = torch.cuda.device_count()          # does not initialise the GPU on this image
    return "nccl" if ndev >= max(1, world) else "gloo"


def init_from_env(backend: str | None = None):
    """Join the process group torchrun describes (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*).
    Returns (world, rank, local_rank, device index or None, backend)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev_index = (local % ndev) if ndev else None
    be = choose_backend(world, backend)
    if world > 1:
        if be == "nccl":
            torch.cuda.set_device(dev_index)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            if dev_index is not None:
                torch.cuda.set_device(dev_index)
            dist.init_process_group("gloo")
    return world, rank, local, dev_index, be


def _device_for(group=None):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_max(values, group=None):
    """Element-wise max over ranks of a list of floats (on the backend's device)."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_device_for(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.tolist()


def rank_device_info(rank: int, dev=None) -> dict:
    """What this rank really runs on, observed rather than inferred: host name, the current HIP
    device index and its PCI location (domain:bus:device) and UUID from the device properties.
    dev None (a CPU rank): device fields are None."""
    import socket
    info = {"rank": int(rank), "host": socket.gethostname(), "device": None, "pci": None, "uuid": None,
            "name": None}
    if dev is None:
        return info
    idx = torch.device(dev).index
    idx = torch.cuda.current_device() if idx is None else idx
    prop = torch.cuda.get_device_properties(idx)
    info["device"] = int(idx)
    info["name"] = prop.name
    bus = getattr(prop, "pci_bus_id", None)
    if bus is not None:
        info["pci"] = "%04x:%02x:%02x" % (int(getattr(prop, "pci_domain_id", 0)), int(bus),
                                          int(getattr(prop, "pci_device_id", 0)))
    u = getattr(prop, "uuid", None)
    info["uuid"] = str(u) if u is not None else None
    return info


def rank_kernel_report(t_enc_ms: float, t_dec_ms: float, step_ms: float, elements: int,
                       bytes_per_elem_kernel: int, peak_gbs: float) -> dict:
    """This rank's OWN measurements, before any max over ranks: the per-launch encode / decode
    durations (HIP events on its launch stream), its step time, and the HBM roofline fraction of
    each kernel (algorithmic bytes = bytes_per_elem_kernel x elements per launch) and of its step.
    Merged into its rank_device_info, so a multi-GPU line shows every GPU's own HBM fraction beside
    the max-over-ranks step."""
    kb = bytes_per_elem_kernel * elements

    def frac(ms, nbytes):
        return round(nbytes / (ms * 1e-3) / 1e9 / peak_gbs, 4) if ms > 0 else None
    return {"kernels_ms": {"encode": round(t_enc_ms, 4), "decode": round(t_dec_ms, 4)},
            "step_ms": round(step_ms, 4),
            "roofline_frac": {"encode": frac(t_enc_ms, kb), "decode": frac(t_dec_ms, kb),
                              "step": frac(step_ms, 2 * kb)}}


def gather_rank_devices(info: dict, group=None) -> list:
    """Every rank's rank_device_info, in rank order, on every rank (all_gather_object; a single
    process returns [info])."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [info]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, info, group=group)
    return sorted(out, key=lambda d: d["rank"])


def distinct_devices(rank_devices) -> int:
    """Number of distinct GPUs the ranks ran on: (host, PCI location) when the PCI location is
    known, else (host, UUID), else (host, device index). CPU ranks count none."""
    keys = set()
    for d in rank_devices:
        if d.get("device") is None:
            continue
        ident = d.get("pci") or d.get("uuid") or ("index", d["device"])
        keys.add((d.get("host"), ident))
    return len(keys)


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


def shard_keypair(seed: bytes, public_key: dict, n: int, world: int, rank: int, private_key=None):
    """The Paillier keypair one rank encrypts its shard of an n-element tensor with: the broadcast
    public key {n, hs, a_bytes, group_size[, n_bytes]} (hex ints), randomness keyed by the
    broadcast seed, and the running counter started at the shard's global element offset, so
    rank r's ciphertexts equal elements [start, end) of a single-GPU encryption under the same
    seed (Philox counter = global element index). Returns (keypair, (start, end))."""
    from efl.privacy.paillier_cipher import PaillierKeypair
    start, end = shard_range(n, world, rank, elem_bytes=8)
    kp = PaillierKeypair(seed=seed)
    pk = public_key
    p = q = None
    if private_key is not None:
        p, q = int(private_key["p"], 16), int(private_key["q"], 16)
    kp.set_keys_ints(int(pk["n"], 16), int(pk["hs"], 16), int(pk["a_bytes"]), int(pk.get("group_size", 1)),
                     p, q, pk.get("n_bytes"))
    kp.counter = start
    return kp, (start, end)
