# host-tensor ops through the pinned pipeline: Stage-F GPU parity, then the host-op A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fxp_gpu.py tests/test_hook_gpu.py tests/test_e2e_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_hostops.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_host_ops.py > gpurun_out/host_ops.jsonl 2> gpurun_out/host_ops.err
