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
    # value = 2 x 0.25 GiB per step / max-over-ranks step time; the K timed steps fit in the wall
    assert out["value"] > 0 and out["steps"] * out["ms_per_step"] * 1e-3 < wall
    assert abs(out["value"] - 2 * 0.25 / (out["ms_per_step"] * 1e-3)) / out["value"] < 0.01
