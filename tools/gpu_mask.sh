set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_mask_gpu.py tests/test_secret_sharing_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_mask.log 2>&1 &&
timeout -k 10 200 python tools/bench_mask.py > $O/bench_mask.jsonl 2> $O/bench_mask.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_mask -o run --output-format csv -- python3 tools/bench_mask.py --steps 20 --no-cpu-baseline > $O/prof_mask.log 2>&1
