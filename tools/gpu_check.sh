#!/bin/bash
# One GPU session: parity tests, smoke, bench, variant sweep, rocprofv3 kernel-trace + PMC passes.
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
STAGE=${1:-all}
run_tests() { timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; }
run_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; }
run_bench() { timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err && timeout -k 10 300 python tools/bench_batched.py > $O/bench_batched.json 2> $O/bench_batched.err && timeout -k 10 600 python tools/bench_e2e.py > $O/bench_e2e.json 2> $O/bench_e2e.err; }
run_sweep() { timeout -k 10 300 python tools/sweep_fxp.py > $O/sweep.jsonl 2> $O/sweep.err; }
# traffic-mix HBM ceilings and VALU issue rates (tools/*.hip, built on the CPU side beforehand)
run_probes() {
  timeout -k 10 120 tools/stream_probe > $O/stream_probe.json 2> $O/stream_probe.err &&
  timeout -k 10 120 tools/valu_probe > $O/valu_probe.jsonl 2> $O/valu_probe.err
}
run_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trace -o run --output-format csv \
      -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_trace.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch -o run --output-format csv \
      -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_fetch.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write -o run --output-format csv \
      -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_write.log 2>&1
}
case $STAGE in
  all) run_tests && run_smoke && run_bench && run_sweep && run_prof ;;
  round) run_tests && run_smoke && run_probes && run_bench && run_prof ;;
  probes) run_probes ;;
  tests) run_tests ;;
  bench) run_bench && run_sweep ;;
  prof) run_prof ;;
  *) echo "unknown stage $STAGE"; exit 2 ;;
esac
rc=$?
echo "gpu_check $STAGE rc=$rc"
exit $rc
