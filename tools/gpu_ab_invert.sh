# k_invert with u, v in registers: invert parity tests, then the invert bench for the current library
# and the previous one (libefl_hip_invold.so), alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/elastic-federated-learning-solution_amd/efl
rm -f gpurun_out/invert_ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_paillier_gpu.py -m gpu -x -q -k "invert or matmul or negative" --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_inv.log 2>&1 || exit 1
for v in "" _invold "" _invold; do
  EFL_HIP_LIB=$L/libefl_hip$v.so timeout -k 10 300 python -u tools/bench_invert.py >> gpurun_out/invert_ab.jsonl \
    2>> gpurun_out/invert_ab.err || exit 1
done
