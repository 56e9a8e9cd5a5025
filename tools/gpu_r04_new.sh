#!/bin/bash
# round-4 new GPU tests (launcher, reference cases at 4096-bit, matmul oracle at every key, rotation)
# then the config-3 coalescing probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_bench_launcher.py tests/test_paillier_reference_cases_gpu.py tests/test_paillier_crt_gpu.py \
  tests/test_federal_model_gpu.py tests/test_fxp_gpu.py \
  "tests/test_paillier_gpu.py::test_matmul_vs_oracle" "tests/test_paillier_gpu.py::test_matmul_schedule_paths_every_key" \
  > gpurun_out/r04_new.log 2>&1
rc=$?
tail -30 gpurun_out/r04_new.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/config3_coalesce_probe.py > gpurun_out/c3_coalesce.jsonl 2> gpurun_out/c3_coalesce.err
rc=$?
cat gpurun_out/c3_coalesce.jsonl; tail -5 gpurun_out/c3_coalesce.err
[ $rc -eq 0 ] || exit $rc
for lib in libefl_hip.so libefl_hip_wprobe.so libefl_hip.so; do
  EFL_HIP_LIB=$PWD/elastic-federated-learning-solution_amd/efl/$lib timeout -k 10 200 python -u tools/walk_probe.py \
    >> gpurun_out/walk_probe.jsonl 2>> gpurun_out/walk_probe.err || exit $?
done
cat gpurun_out/walk_probe.jsonl
