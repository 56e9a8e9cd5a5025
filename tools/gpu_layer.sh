# the paillier_mnist dense layer step, two processes on one GPU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_layer.py --steps 3 --warmup 1 > gpurun_out/bench_layer.jsonl 2> gpurun_out/bench_layer.err
