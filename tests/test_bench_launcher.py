"""bench.py's own N-rank launch (`bench.py --gpus N` with no torchrun environment) and its world
checks. The driver's scaling run calls `bench.py --gpus N`; a run labelled N must have been N ranks.

CPU: a mismatched --gpus / WORLD_SIZE exits non-zero before any GPU or process-group call, and the
launcher propagates a failing rank's exit status.
GPU: `--gpus 2` on the one-GPU box starts two ranks (gloo, both on cuda:0) and relays rank 0's line.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env,
                          timeout=timeout, cwd=ROOT)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "4", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 3, r.stderr
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_single_rank_env_with_gpus_gt_1_exits_nonzero():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 3, r.stderr


def test_gpus_zero_rejected():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0


def test_launcher_propagates_rank_failure():
    """On a host without a GPU every rank fails in efl.lib.require_gpu(); the launcher must not
    print a result line and must exit non-zero."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("needs a host without a GPU")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-extras", "--no-cpu-baseline"])
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_devices_used_is_the_distinct_observed_count():
    """bench.py's devices_used = efl.distributed.distinct_devices(rank_devices): distinct (host,
    PCI location) pairs the ranks reported, never min(world, device_count)."""
    sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
    from efl import distributed as edist

    def rd(rank, dev, pci, host="h0", uuid=None):
        return {"rank": rank, "host": host, "device": dev, "pci": pci, "uuid": uuid, "name": "x"}
    eight = [rd(r, r, "0000:%02x:00" % (0x10 + r)) for r in range(8)]
    assert edist.distinct_devices(eight) == 8
    shared = [rd(0, 0, "0000:11:00"), rd(1, 0, "0000:11:00")]
    assert edist.distinct_devices(shared) == 1
    # the same index on two hosts is two devices; no PCI falls back to UUID, then to the index
    assert edist.distinct_devices([rd(0, 0, "0000:11:00", "a"), rd(1, 0, "0000:11:00", "b")]) == 2
    assert edist.distinct_devices([rd(0, 0, None, uuid="u1"), rd(1, 1, None, uuid="u1")]) == 1
    assert edist.distinct_devices([rd(0, 0, None), rd(1, 1, None)]) == 2
    assert edist.distinct_devices([rd(0, None, None)]) == 0
    # and bench.py reports exactly that function of what it gathered
    src = open(BENCH).read()
    assert '"devices_used": edist.distinct_devices(rank_devices)' in src
    assert "min(world, torch.cuda.device_count())" not in src


def test_rank_devices_gathered_over_gloo():
    """gather_rank_devices under a world-2 gloo group (CPU ranks): rank order, every rank's entry."""
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=90) for _ in range(2)]
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    for r, got in res:
        assert [d["rank"] for d in got] == [0, 1]
        assert all(d["device"] is None for d in got)
        # every rank's own kernel times and roofline fractions travel with its entry (VERDICT r5
        # item 6): rank 1 was given kernels twice as slow, and its fractions are its own
        r0, r1 = got
        assert r1["kernels_ms"]["encode"] == 2 * r0["kernels_ms"]["encode"]
        assert abs(r0["roofline_frac"]["encode"] - 2 * r1["roofline_frac"]["encode"]) < 1e-3
        for d in got:
            assert set(d["roofline_frac"]) == {"encode", "decode", "step"}
            assert d["step_ms"] > 0


def test_rank_kernel_report_contract():
    """rank_kernel_report: per-kernel fraction = bytes_per_elem x elements / kernel time / peak, the
    step's = twice the bytes / step time; the field names bench.py and the SCALE reader rely on."""
    sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
    from efl import distributed as edist
    n = 65536 * 1024
    r = edist.rank_kernel_report(0.2, 0.25, 0.45, n, 20, 8000.0)
    assert r["kernels_ms"] == {"encode": 0.2, "decode": 0.25} and r["step_ms"] == 0.45
    assert abs(r["roofline_frac"]["encode"] - 20 * n / 0.2e-3 / 8e12) < 1e-4
    assert abs(r["roofline_frac"]["decode"] - 20 * n / 0.25e-3 / 8e12) < 1e-4
    assert abs(r["roofline_frac"]["step"] - 40 * n / 0.45e-3 / 8e12) < 1e-4
    assert edist.rank_kernel_report(0.0, 0.1, 0.1, n, 20, 8000.0)["roofline_frac"]["encode"] is None
    src = open(BENCH).read()
    assert "edist.gather_rank_devices({**edist.rank_device_info(rank, dev), **own})" in src
    # the report is taken before the max over ranks overwrites this rank's times
    assert src.index("own = edist.rank_kernel_report(") < src.index("edist.all_reduce_max([elapsed, t_enc, t_dec])")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gather_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))
    import torch.distributed as dist
    from efl import distributed as edist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        own = edist.rank_kernel_report(0.2 * (rank + 1), 0.2 * (rank + 1), 0.4 * (rank + 1), 1 << 26, 20, 8000.0)
        q.put((rank, edist.gather_rank_devices({**edist.rank_device_info(rank, None), **own})))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpus2_launches_two_ranks_on_one_gpu():
    t0 = time.perf_counter()
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--no-extras", "--no-cpu-baseline"], timeout=110)
    wall = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["backend"] == "gloo"
    assert out["seed_broadcast_us"] > 0
    assert out["devices_used"] == 1
    # both ranks report what they observed: two entries, one device (same PCI location)
    rd = out["rank_devices"]
    assert [d["rank"] for d in rd] == [0, 1]
    assert all(d["device"] == 0 and d["pci"] for d in rd)
    assert len({(d["host"], d["pci"]) for d in rd}) == 1
    # each rank's own kernel times and HBM fractions (two ranks share the card, so each is slower
    # than alone, but each ran its kernels and reports them)
    for d in rd:
        assert d["kernels_ms"]["encode"] > 0 and d["kernels_ms"]["decode"] > 0 and d["step_ms"] > 0
        assert 0 < d["roofline_frac"]["encode"] < 1 and 0 < d["roofline_frac"]["step"] < 1
    # value = 2 x 0.25 GiB per step / max-over-ranks step time; the K timed steps fit in the wall
    assert out["value"] > 0 and out["steps"] * out["ms_per_step"] * 1e-3 < wall
    assert abs(out["value"] - 2 * 0.25 / (out["ms_per_step"] * 1e-3)) / out["value"] < 0.01
