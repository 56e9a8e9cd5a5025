#!/bin/bash
# Round-2 GPU session script: each GPU step under its own time limit, chained with &&, output
# under gpurun_out/. Usage: bash tools/gpu_r02.sh <step>...  (steps: tests, probe, bench, bench2,
# prof, pmc)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
run() {
  case "$1" in
    tests)  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
              > gpurun_out/pytest.log 2>&1 ;;
    dist)   timeout -k 10 200 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -v --timeout 150 \
              --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 ;;
    probe)  timeout -k 10 240 python -u tools/step_probe.py > gpurun_out/step_probe.json 2> gpurun_out/step_probe.err ;;
    bench)  timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
    bench2) timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
              --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 \
              > gpurun_out/bench2.json 2> gpurun_out/bench2.err ;;
    pl)     timeout -k 10 600 python -u -m pytest tests/test_paillier_gpu.py tests/test_distributed_gpu.py \
              tests/test_paillier_layer_gpu.py -m gpu -x -q \
              --timeout 300 --timeout-method thread > gpurun_out/pytest_pl.log 2>&1 ;;
    stagep) timeout -k 10 900 python -u bench.py --stage p --no-cpu-baseline > gpurun_out/stage_p.jsonl 2> gpurun_out/stage_p.err ;;
    hex)    timeout -k 10 240 python -u tools/bench_hex.py > gpurun_out/bench_hex.json 2> gpurun_out/bench_hex.err ;;
    hexprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hexprof -o run -- \
              python3 tools/bench_hex.py > gpurun_out/bench_hex_prof.json 2> gpurun_out/hexprof.err ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv \
              -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/prof_trace.log 2>&1 ;;
    pmc)    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_fetch.log 2>&1 && \
            timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_write.log 2>&1 ;;
    exh)    timeout -k 10 900 python -u tools/exhaustive_fxp.py > gpurun_out/exhaustive.json 2> gpurun_out/exhaustive.err ;;
    fxp)    timeout -k 10 600 python -u -m pytest tests/test_fxp_gpu.py -m gpu -x -q --timeout 120 \
              --timeout-method thread > gpurun_out/pytest_fxp.log 2>&1 ;;
    e2e)    timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py tests/test_hook_gpu.py -m gpu -x -v --timeout 150 \
              --timeout-method thread > gpurun_out/pytest_e2e.log 2>&1 ;;
    e2ebench) timeout -k 10 600 python -u tools/bench_e2e.py > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err ;;
    bprobe) timeout -k 10 300 python -u tools/batched_probe.py > gpurun_out/batched_probe.json 2> gpurun_out/batched_probe.err ;;
    stagepc) timeout -k 10 1100 python -u bench.py --stage p > gpurun_out/stage_p_cpu.jsonl 2> gpurun_out/stage_p_cpu.err ;;
    mmsweep) timeout -k 10 600 python -u tools/matmul_sweep.py > gpurun_out/matmul_sweep.jsonl 2> gpurun_out/matmul_sweep.err ;;
    mmvar)  for v in "" _mmC; do
              EFL_HIP_LIB=$PWD/elastic-federated-learning-solution_amd/efl/libefl_hip$v.so timeout -k 10 300 \
                python -u tools/matmul_sweep.py --families 16,32 0 1 2 4 8 >> gpurun_out/matmul_var.jsonl \
                2>> gpurun_out/matmul_var.err || return 1
            done ;;
    mask)   timeout -k 10 300 python -u tools/bench_mask.py > gpurun_out/bench_mask.jsonl 2> gpurun_out/bench_mask.err ;;
    profmask) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mask -o run --output-format csv \
              -- python3 tools/bench_mask.py --steps 20 --no-cpu-baseline > gpurun_out/prof_mask.log 2>&1 ;;
    plfam)  timeout -k 10 600 python -u tools/sweep_pl_family.py > gpurun_out/sweep_pl_family.jsonl 2> gpurun_out/sweep_pl_family.err ;;
    profp)  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p -o run --output-format csv \
              -- python3 bench.py --stage p --no-cpu-baseline > gpurun_out/prof_p.log 2>&1 ;;
    profhex) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hex -o run --output-format csv \
              -- python3 tools/bench_hex.py > gpurun_out/prof_hex.log 2>&1 ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s $(date +%T)"
  run "$s" || { rc=$?; echo "step $s failed rc=$rc"; exit $rc; }
done
echo "== done $(date +%T)"
