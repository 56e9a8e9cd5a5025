"""GPU, world sizes 2 and 4: the multi-GPU layout of §8(e) run with the HIP kernels under several ranks.

The driver's 1-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so both
ranks share cuda:0 over gloo (efl.distributed.choose_backend) — the same code path an 8-GPU node
runs over RCCL, minus the transport. Checked:

* Stage F: each rank encodes / decodes its shard_range of one tensor with libefl_hip.so; the
  gathered mantissas, exponents and decoded floats equal the single-rank HIP result and the oracle
  bit for bit.
* Stage P: rank 0 broadcasts the 32-byte seed and the public key; each rank encrypts its shard with
  efl.distributed.shard_keypair (Philox counter = global element index); the gathered ciphertext
  hex equals a single-rank encryption of the whole tensor under the same seed, and decrypts to the
  plaintext ("1-GPU and N-GPU ciphertexts are byte-identical").
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as tmp

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

N_F = 1_000_003          # ragged: shards end off the 256-B grid only at the tail
N_P = 300


def _key():
    with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
        kat = json.load(f)
    return next(k for k in kat["keys"] if k["n_bytes"] == 128)      # the examples' 1024-bit n


def _plain():
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N_F, generator=g)
    x[:4] = torch.tensor([0.0, -0.0, 8388608.0, 1e-40])
    x[1000:2000] = 0.0                                           # ReLU-style zeros
    m = torch.randint(-2**62, 2**62, (N_P,), generator=g, dtype=torch.int64)
    return x, m


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from efl import distributed as edist
    _, _, _, dev_index, backend = edist.init_from_env()
    import torch.distributed as dist
    import efl
    dev = efl.lib.require_gpu()
    x, m = _plain()
    s, e = edist.shard_range(N_F, world, rank)
    M, E = efl.lib.convert_to_fixed_point(x[s:e].to(dev))
    y = efl.lib.fixed_point_to_float_point(M, E, torch.float32)
    torch.cuda.synchronize()
    k = _key()
    pk = {"n": k["n"], "hs": k["hs"], "a_bytes": k["a_bits"] // 8, "group_size": 1, "n_bytes": k["n_bytes"]}
    seed, pk_b = edist.broadcast_key_material(b"\x5a" * 32 if rank == 0 else None, pk if rank == 0 else None)
    kp, (ps, pe) = edist.shard_keypair(seed, pk_b, N_P, world, rank)
    ct = kp.encrypt(m[ps:pe]).tensor.to_hex().strings()
    parts = [None] * world
    dist.all_gather_object(parts, dict(rank=rank, backend=backend, dev=dev_index, s=s, e=e,
                                        M=M.cpu().numpy(), E=E.cpu().numpy(),
                                        y=y.cpu().numpy().view(np.uint32), ps=ps, pe=pe, ct=ct,
                                        seed=seed, counter=kp.counter))
    if rank == 0:
        q.put(parts)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_share_cuda0_bit_identical(world):
    import efl
    from oracle import fxp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    procs = tmp.start_processes(_worker, args=(world, port, q), nprocs=world, join=False, start_method="spawn")
    try:
        parts = q.get(timeout=100)
    except Exception:
        procs.join(timeout=5)          # re-raises a rank's own traceback if one failed
        raise
    while not procs.join(timeout=30):
        pass
    assert [p["backend"] for p in parts] == ["gloo"] * world
    # contiguous shards that tile [0, N_F) in rank order
    assert parts[0]["s"] == 0 and parts[-1]["e"] == N_F
    assert all(parts[r]["e"] == parts[r + 1]["s"] for r in range(world - 1))

    x, m = _plain()
    Mg = np.concatenate([p["M"] for p in parts])
    Eg = np.concatenate([p["E"] for p in parts])
    yg = np.concatenate([p["y"] for p in parts])
    # single-rank HIP result on the same device
    dev = efl.lib.require_gpu()
    M1, E1 = efl.lib.convert_to_fixed_point(x.to(dev))
    y1 = efl.lib.fixed_point_to_float_point(M1, E1, torch.float32)
    assert np.array_equal(Mg, M1.cpu().numpy()) and np.array_equal(Eg, E1.cpu().numpy())
    assert np.array_equal(yg, y1.cpu().numpy().view(np.uint32))
    # and the oracle
    Mo, Eo = fxp.encode(x.numpy())
    assert np.array_equal(Mg, Mo) and np.array_equal(Eg, Eo)
    assert np.array_equal(yg, fxp.decode(Mo, Eo, np.float32, ftz=True).view(np.uint32))

    # Stage P: sharded ciphertexts == one-rank encryption under the broadcast seed
    seed = parts[0]["seed"]
    assert all(p["seed"] == seed for p in parts)
    k = _key()
    pk = {"n": k["n"], "hs": k["hs"], "a_bytes": k["a_bits"] // 8, "group_size": 1, "n_bytes": k["n_bytes"]}
    from efl import distributed as edist
    kp1, rng1 = edist.shard_keypair(seed, pk, N_P, 1, 0, private_key={"p": k["p"], "q": k["q"]})
    assert rng1 == (0, N_P)
    whole = kp1.encrypt(m)
    cg = [c for p in parts for c in p["ct"]]
    assert cg == whole.tensor.to_hex().strings()
    assert [p["counter"] for p in parts] == [p["pe"] for p in parts] and parts[-1]["pe"] == N_P
    assert torch.equal(kp1.decrypt(efl.HexTensor.from_strings(cg), dtype=torch.int64).cpu(), m)


def _rccl_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as dist
    from efl import distributed as edist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    seed, pk = edist.broadcast_key_material(b"\x01" * 32, {"n": "ab", "hs": "cd"})
    mx = edist.all_reduce_max([1.5, -2.5, 3.0])
    dist.barrier()
    q.put((seed, pk, mx, dist.get_backend()))
    dist.destroy_process_group()


def test_rccl_collectives_of_the_multi_gpu_path():
    """The collectives bench.py and efl.distributed run over RCCL on an 8-GPU node (key material
    broadcast, max over ranks, barrier) exercised on this box's one GPU in a single-rank RCCL group:
    the same device placement of the tensors (_device_for) and the same communicator setup."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    q = tmp.get_context("spawn").Queue()
    procs = tmp.start_processes(_rccl_worker, args=(port, q), nprocs=1, join=False, start_method="spawn")
    try:
        seed, pk, mx, backend = q.get(timeout=100)
    except Exception:
        procs.join(timeout=5)
        raise
    while not procs.join(timeout=30):
        pass
    assert backend == "nccl" and seed == b"\x01" * 32 and pk == {"n": "ab", "hs": "cd"}
    assert mx == [1.5, -2.5, 3.0]
