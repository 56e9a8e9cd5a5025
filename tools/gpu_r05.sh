#!/bin/bash
# Round-5 GPU session script: each GPU step under its own time limit, chained, output under
# gpurun_out/. Usage: bash tools/gpu_r05.sh <step>...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
LIBDIR=$PWD/elastic-federated-learning-solution_amd/efl
run() {
  case "$1" in
    tests)  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
              > gpurun_out/r05_pytest.log 2>&1 ;;
    pltests) timeout -k 10 900 python -u -m pytest tests/test_paillier_gpu.py tests/test_paillier_crt_gpu.py \
              tests/test_federal_model_gpu.py tests/test_paillier_reference_cases_gpu.py tests/test_paillier_layer_gpu.py \
              -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_pltests.log 2>&1 ;;
    dist)   timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_bench_launcher.py tests/test_fxp_gpu.py \
              -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_dist.log 2>&1 ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 ;;
    bench)  timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err ;;
    bench2) timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 3 --no-extras --no-cpu-baseline \
              > gpurun_out/r05_bench_gpus2.json 2> gpurun_out/r05_bench_gpus2.err ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_trace -o run --output-format csv \
              -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/r05_prof_trace.log 2>&1 ;;
    pmc)    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r05_prof_fetch -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r05_prof_fetch.log 2>&1 && \
            timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r05_prof_write -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r05_prof_write.log 2>&1 ;;
    stagep) timeout -k 10 1000 python -u bench.py --stage p > gpurun_out/r05_stage_p.jsonl 2> gpurun_out/r05_stage_p.err ;;
    stagepq) timeout -k 10 600 python -u bench.py --stage p --no-cpu-baseline > gpurun_out/r05_stage_p.jsonl 2> gpurun_out/r05_stage_p.err ;;
    layer)  timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 > gpurun_out/r05_layer_dense.jsonl 2> gpurun_out/r05_layer_dense.err && \
            timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 --kind weight > gpurun_out/r05_layer_weight.jsonl 2> gpurun_out/r05_layer_weight.err ;;
    c3co)   timeout -k 10 300 python -u tools/config3_coalesce_probe.py > gpurun_out/r05_c3_coalesce.jsonl 2> gpurun_out/r05_c3_coalesce.err ;;
    c3kt)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_c3_kt -o run --output-format csv \
              -- python3 tools/config3_probe.py --reps 20 > gpurun_out/r05_c3_kt.log 2>&1 && \
            cp /tmp/r05_c3_kt/run_kernel_stats.csv gpurun_out/r05_c3_kernel_stats.csv ;;
    walk)   for lib in ${WALK_LIBS:-libefl_hip.so}; do
              EFL_HIP_LIB=$LIBDIR/$lib timeout -k 10 200 python -u tools/walk_probe.py >> gpurun_out/r05_walk_probe.jsonl \
                2>> gpurun_out/r05_walk_probe.err || return $?
            done ;;
    rekey)  timeout -k 10 300 python -u tools/rekey_probe.py > gpurun_out/r05_rekey.jsonl 2> gpurun_out/r05_rekey.err ;;
    keysize) timeout -k 10 300 python -u tools/keysize_probe.py > gpurun_out/r05_keysize.jsonl 2> gpurun_out/r05_keysize.err ;;
    keytests) timeout -k 10 900 python -u -m pytest tests/test_paillier_key_sizes_gpu.py tests/test_paillier_long_shift_gpu.py \
              -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r05_keysizes.log 2>&1 ;;
    tblw)   timeout -k 10 600 python -u tools/table_window_probe.py --crt 16 18 20 \
              > gpurun_out/r05_table_window_1024.jsonl 2> gpurun_out/r05_table_window_1024.err && \
            timeout -k 10 600 python -u tools/table_window_probe.py --crt --n-bytes 512 --a-bytes 256 --group 1 --sizes 65536 12 14 15 \
              > gpurun_out/r05_table_window_4096.jsonl 2> gpurun_out/r05_table_window_4096.err ;;
    decfam) timeout -k 10 600 python -u tools/sweep_dec_family.py > gpurun_out/r05_dec_family.jsonl 2> gpurun_out/r05_dec_family.err ;;
    fipst)  timeout -k 10 900 python -u -m pytest tests/test_paillier_gpu.py tests/test_paillier_crt_gpu.py \
              tests/test_paillier_key_sizes_gpu.py tests/test_paillier_scalar_gpu.py -m gpu -x -q --timeout 300 \
              --timeout-method thread > gpurun_out/r05_fips_tests.log 2>&1 ;;
    fipsab) for nb in 128; do
              for lib in ${AB_LIBS:-libefl_hip.so libefl_hip_nofips.so}; do
                WP_NBYTES=$nb EFL_HIP_LIB=$LIBDIR/$lib timeout -k 10 300 python -u tools/walk_probe.py \
                  >> gpurun_out/r05_fips_walk.jsonl 2>> gpurun_out/r05_fips_walk.err || exit 1
              done
            done
            for lib in ${AB_LIBS:-libefl_hip.so libefl_hip_nofips.so}; do
              EFL_HIP_LIB=$LIBDIR/$lib timeout -k 10 600 python -u bench.py --stage p --no-cpu-baseline \
                >> gpurun_out/r05_fips_stagep.jsonl 2>> gpurun_out/r05_fips_stagep.err || exit 1
            done ;;
    fp64)   timeout -k 10 300 python -u tools/fp64_shape_probe.py > gpurun_out/r05_fp64_shape.jsonl 2> gpurun_out/r05_fp64_shape.err ;;
    ctx)    timeout -k 10 600 python -u -m pytest tests/test_ctx_abi_gpu.py tests/test_paillier_crt_gpu.py -m gpu -x -q \
              --timeout 300 --timeout-method thread > gpurun_out/r05_ctx.log 2>&1 ;;
    split)  timeout -k 10 400 python -u tools/walk_split_probe.py > gpurun_out/r05_walk_split.jsonl 2> gpurun_out/r05_walk_split.err ;;
    splitt) timeout -k 10 600 python -u -m pytest tests/test_walk_split_gpu.py -m gpu -x -q --timeout 300 \
              --timeout-method thread > gpurun_out/r05_walk_split_tests.log 2>&1 ;;
    crtkt)  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_crtkt -o run --output-format csv \
              -- python3 tools/crt_mnist_probe.py --parts 1 > gpurun_out/r05_crtkt.log 2>&1 ;;
    crtkt3) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_crtkt3 -o run --output-format csv \
              -- python3 tools/crt_mnist_probe.py --parts 3 > gpurun_out/r05_crtkt3.log 2>&1 ;;
    dpchk)  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I elastic-federated-learning-solution_amd/csrc \
              tools/dp_fastmath_check.hip -o /tmp/dp_fastmath_check && \
            timeout -k 10 60 /tmp/dp_fastmath_check > gpurun_out/r05_dp_fastmath.json 2>&1 ;;
    mask)   timeout -k 10 300 python -u tools/bench_mask.py > gpurun_out/r05_bench_mask.jsonl 2> gpurun_out/r05_bench_mask.err ;;
    masktests) timeout -k 10 600 python -u -m pytest tests/test_mask_gpu.py tests/test_secret_sharing_gpu.py tests/test_dp_gpu.py \
              -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_mask_tests.log 2>&1 ;;
    bprobe) BATCH_ARMS="base:512,2,512,2;k1:512,1,512,1;xcd:512,2,512,2,2,2;flat:512,2,512,2,1,1;persist:512,2,512,2,3,3,2048;persist4k:512,2,512,2,3,3,4096;b256k4:256,4,256,4;again:512,2,512,2" \
              timeout -k 10 300 python -u tools/batched_probe.py > gpurun_out/r05_batched_probe.jsonl 2> gpurun_out/r05_batched_probe.err ;;
    crtt)   timeout -k 10 600 python -u -m pytest tests/test_crt_walks_gpu.py tests/test_walk_split_gpu.py tests/test_paillier_crt_gpu.py \
              tests/test_ctx_abi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_crt_tests.log 2>&1 ;;
    crtfp)  timeout -k 10 300 python -u tools/crt_fused_probe.py > gpurun_out/r05_crt_fused.jsonl 2> gpurun_out/r05_crt_fused.err ;;
    crtkt2) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_crtkt2 -o run --output-format csv \
              -- python3 tools/crt_mnist_probe.py --n 262144 > gpurun_out/r05_crtkt2.log 2>&1 ;;
    profp)  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_p -o run --output-format csv \
              -- python3 bench.py --stage p --no-cpu-baseline > gpurun_out/r05_prof_p.log 2>&1 ;;
    spillkt) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_spill_kt -o run --output-format csv \
              -- python3 tools/spill_probe.py > gpurun_out/r05_spill_kt.log 2>&1 ;;
    spillpmc) timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_WAVE_CYCLES SQ_INSTS \
              -d gpurun_out/r05_spill_pmc -o run --output-format csv \
              -- python3 tools/spill_probe.py > gpurun_out/r05_spill_pmc.log 2>&1 ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s $(date +%T)"
  run "$s" || { rc=$?; echo "step $s failed rc=$rc"; exit $rc; }
done
echo "== done $(date +%T)"
