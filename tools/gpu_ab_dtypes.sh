# fp64 / integer launch shapes: Stage-F GPU parity, then the dtype bench for the current library and
# the previous one (libefl_hip_fxpold.so), alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/elastic-federated-learning-solution_amd/efl
rm -f gpurun_out/fxp_dtypes.jsonl
timeout -k 10 600 python -u -m pytest tests/test_fxp_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_fxp.log 2>&1 || exit 1
for v in "" _fxpold "" _fxpold; do
  EFL_HIP_LIB=$L/libefl_hip$v.so timeout -k 10 200 python -u tools/bench_fxp_dtypes.py >> gpurun_out/fxp_dtypes.jsonl \
    2>> gpurun_out/fxp_dtypes.err || exit 1
done
