# A/B of the encrypt tail: the current library against the previous commit's k_encrypt28
# (libefl_hip_oldtail.so), alternating, same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/elastic-federated-learning-solution_amd/efl
rm -f gpurun_out/ab_tail.jsonl
for v in "" _oldtail "" _oldtail; do
  EFL_HIP_LIB=$L/libefl_hip$v.so timeout -k 10 300 python -u bench.py --stage p --no-cpu-baseline \
    | sed "s|^{|{\"lib\": \"libefl_hip$v.so\", |" >> gpurun_out/ab_tail.jsonl 2>> gpurun_out/ab_tail.err || exit 1
done
