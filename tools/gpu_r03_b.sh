#!/bin/bash
# round 3: FederalModel + config-5 full-size tests, batched tile-order A/B, gRPC leg probe
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_federal_model_gpu.py tests/test_e2e_full_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r03_model_tests.log 2>&1 || exit $?
BATCH_ARMS="base:256,2,256,4,0,0;flat:256,2,256,4,1,1;xcd:256,2,256,4,2,2;xcd_d128:256,2,128,1,2,2;stream_shapes:512,1,128,1,2,2;enc0_dec2:256,2,256,4,0,2;enc2_dec0:256,2,256,4,2,0;xcd_d128k2:256,2,128,2,2,2" timeout -k 10 300 python -u tools/batched_probe.py > gpurun_out/r03_batched_probe.json 2> gpurun_out/r03_batched_probe.err || exit $?
timeout -k 10 400 python -u tools/grpc_probe.py --mib 512 --reps 3 --channels 1 2 4 > gpurun_out/r03_grpc_probe.jsonl 2>&1 || exit $?
EFL_GRPC_MAX_FRAME_SIZE=16777215 timeout -k 10 300 python -u tools/grpc_probe.py --mib 512 --reps 3 --channels 1 2 >> gpurun_out/r03_grpc_probe.jsonl 2>&1 || exit $?
