#!/bin/bash
# round 3: FederalModel two-party training + config 5 at full size
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_federal_model_gpu.py tests/test_e2e_full_gpu.py tests/test_paillier_layer_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r03_model_tests.log 2>&1
