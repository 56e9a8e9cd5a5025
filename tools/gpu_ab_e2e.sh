# A/B of config 5: post_recv reading the gRPC payloads in place vs private copies, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab_e2e.jsonl
for c in 0 1 0 1; do
  EFL_E2E_COPY_RECV=$c timeout -k 10 300 python -u tools/bench_e2e.py >> gpurun_out/ab_e2e.jsonl 2>> gpurun_out/ab_e2e.err || exit 1
done
