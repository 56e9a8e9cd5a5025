# kernel stats of the two-party layer bench (both processes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_layer -o run --output-format csv \
  -- python3 tools/bench_layer.py --steps 2 --warmup 1 > gpurun_out/prof_layer.log 2>&1
