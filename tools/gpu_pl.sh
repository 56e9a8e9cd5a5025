#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_paillier_gpu.py -x -q > $O/pytest_pl.log 2>&1 &&
PL_SIZES=${PL_SIZES:-16384} PL_KEYS=${PL_KEYS:-64:1,128:1,128:10} timeout -k 10 900 python tools/bench_paillier.py > $O/bench_pl.jsonl 2> $O/bench_pl.err
echo "gpu_pl rc=$?"
