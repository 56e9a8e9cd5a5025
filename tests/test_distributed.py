"""CPU, world_size 2 and 4 (gloo): the multi-GPU layout — shard ranges, key-material broadcast, and the
invariant that sharded results equal the single-process result (the codec is the CPU oracle here;
on MI355X the same code runs over RCCL with the HIP ops)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from efl import distributed as edist


def test_shard_range_partition():
    for n in (0, 1, 63, 64, 1000, 67108864, 12345679):
        for world in (1, 2, 3, 8):
            rs = [edist.shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (s0, e0), (s1, e1) in zip(rs, rs[1:]):
                assert e0 == s1
            assert all((s * 4) % 256 == 0 for s, _ in rs if s < n)
    with pytest.raises(ValueError):
        edist.shard_range(10, 2, 2)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import fxp
    seed, pk = edist.broadcast_key_material(b"\x07" * 32 if rank == 0 else None,
                                            {"n": "abc", "hs": "12"} if rank == 0 else None)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(100003, generator=g)
    s, e = edist.shard_range(x.numel(), world, rank)
    M, E = fxp.encode(x[s:e].numpy())
    gathered = [None] * world
    dist.all_gather_object(gathered, (s, e, M, E))
    # bench.py's max-over-ranks of (elapsed, t_enc, t_dec)
    mx = edist.all_reduce_max([float(rank), -float(rank), 1.5])
    assert mx == [float(world - 1), 0.0, 1.5]
    if rank == 0:
        Mfull = np.concatenate([g_[2] for g_ in gathered])
        Efull = np.concatenate([g_[3] for g_ in gathered])
        M1, E1 = fxp.encode(x.numpy())
        out.put((seed, pk, bool(np.array_equal(Mfull, M1) and np.array_equal(Efull, E1))))
    else:
        out.put((seed, pk, None))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_multi_rank_gloo(world):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    tmp.start_processes(_worker, args=(world, port, q), nprocs=world, join=True, start_method="spawn")
    res = [q.get(timeout=60) for _ in range(world)]
    assert all(r[0] == b"\x07" * 32 and r[1] == {"n": "abc", "hs": "12"} for r in res)
    assert any(r[2] is True for r in res)


def test_choose_backend(monkeypatch):
    """RCCL when every rank has its own GPU (the driver's 8-GPU node), gloo when ranks would share
    one (RCCL refuses two ranks on a device) or there is none; an explicit choice wins."""
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert edist.choose_backend(8) == "nccl" and edist.choose_backend(2) == "nccl"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert edist.choose_backend(2) == "gloo" and edist.choose_backend(1) == "nccl"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert edist.choose_backend(1) == "gloo"
    assert edist.choose_backend(4, "nccl") == "nccl"


def test_shard_range_paillier_counters():
    """shard_keypair starts each rank's Philox counter at its shard's global offset (8-byte
    elements: 32-element quanta), so the ranks' counter ranges tile [0, n) exactly."""
    for n in (1, 31, 32, 300, 1000003):
        for world in (1, 2, 3, 8):
            rs = [edist.shard_range(n, world, r, elem_bytes=8) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(e0 == s1 for (_, e0), (s1, _) in zip(rs, rs[1:]))
            assert all(s % 32 == 0 for s, _ in rs if s < n)
