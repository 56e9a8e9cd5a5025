# matmul: operand prefetch one event ahead (EFL_MAT_PREFETCH=1 build) against the default, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/elastic-federated-learning-solution_amd/efl
rm -f gpurun_out/mmpf.jsonl
for v in "" _mmpf "" _mmpf; do
  EFL_HIP_LIB=$L/libefl_hip$v.so timeout -k 10 240 python -u tools/matmul_probe.py >> gpurun_out/mmpf.jsonl 2>> gpurun_out/mmpf.err || exit 1
done
