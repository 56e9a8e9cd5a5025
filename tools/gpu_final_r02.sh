# end-of-session check: every GPU test, smoke, the driver's bench, kernel stats and PMC passes of
# the same bench, the two-party layer step
set -o pipefail
bash tools/gpu_r02.sh tests smoke bench prof pmc || exit 1
timeout -k 10 600 python -u tools/bench_layer.py --steps 3 --warmup 1 > gpurun_out/bench_layer.jsonl 2> gpurun_out/bench_layer.err
