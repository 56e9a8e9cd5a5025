# matmul schedule paths: parity of every event-list path, then the matmul probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_paillier_gpu.py -m gpu -x -q -k "matmul" \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_mm3.log 2>&1 &&
timeout -k 10 240 python -u tools/matmul_probe.py > gpurun_out/mmprobe3.jsonl 2>> gpurun_out/mmprobe.err
