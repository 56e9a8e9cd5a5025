#!/bin/bash
# round 3: device-side MulExp2/MulScalar/fxp_add parity, then the two layer benches
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_paillier_scalar_gpu.py tests/test_paillier_gpu.py tests/test_paillier_layer_gpu.py tests/test_hook_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_scalar_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 > gpurun_out/r03_layer_dense.jsonl 2> gpurun_out/r03_layer_dense.err || exit $?
timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 --kind weight > gpurun_out/r03_layer_weight.jsonl 2> gpurun_out/r03_layer_weight.err || exit $?
