# matmul event-list check: parity tests of the matmul, timing probe, kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/mmprobe.jsonl
timeout -k 10 400 python -u -m pytest tests/test_paillier_gpu.py tests/test_paillier_layer_gpu.py -m gpu -x -q -k "matmul or Matmul or dense or Dense" \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_mm.log 2>&1 &&
timeout -k 10 240 python -u tools/matmul_probe.py >> gpurun_out/mmprobe.jsonl 2>> gpurun_out/mmprobe.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mm -o run --output-format csv -- python3 tools/matmul_probe.py > gpurun_out/prof_mm.log 2>&1 &&
[ "$MMSWEEP" = 1 ] && timeout -k 10 400 python -u tools/matmul_sweep.py 0 1 2 4 8 > gpurun_out/matmul_sweep.jsonl 2> gpurun_out/matmul_sweep.err
true
