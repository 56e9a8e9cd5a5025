# A/B of the CIOS step loop unrolled by 2 (libefl_hip_mu2.so)
# (libefl_hip_mu2.so), alternating, same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/elastic-federated-learning-solution_amd/efl
rm -f gpurun_out/ab_mu2.jsonl
for v in "" _mu2 "" _mu2; do
  EFL_HIP_LIB=$L/libefl_hip$v.so timeout -k 10 300 python -u bench.py --stage p --no-cpu-baseline \
    | sed "s|^{|{\"lib\": \"libefl_hip$v.so\", |" >> gpurun_out/ab_mu2.jsonl 2>> gpurun_out/ab_mu2.err || exit 1
done
