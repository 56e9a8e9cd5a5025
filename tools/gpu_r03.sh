#!/bin/bash
# Round-3 GPU session script: each GPU step under its own time limit, chained, output under
# gpurun_out/. Usage: bash tools/gpu_r03.sh <step>...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
run() {
  case "$1" in
    tests)  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
              > gpurun_out/r03_pytest.log 2>&1 ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 ;;
    bench)  timeout -k 10 300 python -u bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_trace -o run --output-format csv \
              -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03_prof_trace.log 2>&1 ;;
    pmc)    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03_prof_fetch -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r03_prof_fetch.log 2>&1 && \
            timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r03_prof_write -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r03_prof_write.log 2>&1 ;;
    spillkt) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_spill_kt -o run --output-format csv \
              -- python3 tools/spill_probe.py > gpurun_out/r03_spill_kt.log 2>&1 ;;
    spillpmc) timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_WAVE_CYCLES SQ_INSTS \
              -d gpurun_out/r03_spill_pmc -o run --output-format csv \
              -- python3 tools/spill_probe.py > gpurun_out/r03_spill_pmc.log 2>&1 ;;
    stagep) timeout -k 10 900 python -u bench.py --stage p --no-cpu-baseline > gpurun_out/r03_stage_p.jsonl 2> gpurun_out/r03_stage_p.err ;;
    layer)  timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 > gpurun_out/r03_layer_dense.jsonl 2> gpurun_out/r03_layer_dense.err && \
            timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 --kind weight > gpurun_out/r03_layer_weight.jsonl 2> gpurun_out/r03_layer_weight.err ;;
    e2ebench) timeout -k 10 600 python -u tools/bench_e2e.py > gpurun_out/r03_bench_e2e.json 2> gpurun_out/r03_bench_e2e.err ;;
    bprobe) timeout -k 10 300 python -u tools/batched_probe.py > gpurun_out/r03_batched_probe.json 2> gpurun_out/r03_batched_probe.err ;;
    decfam) timeout -k 10 600 python -u tools/sweep_dec_family.py > gpurun_out/r03_dec_family.jsonl 2> gpurun_out/r03_dec_family.err ;;
    mask)   timeout -k 10 300 python -u tools/bench_mask.py > gpurun_out/r03_bench_mask.jsonl 2> gpurun_out/r03_bench_mask.err ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s $(date +%T)"
  run "$s" || { rc=$?; echo "step $s failed rc=$rc"; exit $rc; }
done
echo "== done $(date +%T)"
