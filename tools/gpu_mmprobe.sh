set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/elastic-federated-learning-solution_amd/efl
for v in "" _mmscan _mmhot; do
  EFL_HIP_LIB=$L/libefl_hip$v.so timeout -k 10 240 python -u tools/matmul_probe.py >> gpurun_out/mmprobe.jsonl 2>> gpurun_out/mmprobe.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mm -o run --output-format csv -- python3 tools/matmul_probe.py > gpurun_out/prof_mm.log 2>&1
