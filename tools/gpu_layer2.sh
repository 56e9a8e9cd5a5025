# hex wire codec change: GPU tests touching DT_STRING payloads, then the layer bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_paillier_layer_gpu.py tests/test_hook_gpu.py tests/test_e2e_gpu.py tests/test_paillier_gpu.py tests/test_secret_sharing_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_layer.log 2>&1 &&
timeout -k 10 600 python -u tools/bench_layer.py --steps 3 --warmup 1 > gpurun_out/bench_layer.jsonl 2> gpurun_out/bench_layer.err
