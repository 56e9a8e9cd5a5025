#!/bin/bash
# Round-6 GPU session script: each GPU step under its own time limit, chained, output under
# gpurun_out/. Usage: bash tools/gpu_r06.sh <step>...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
LIBDIR=$PWD/elastic-federated-learning-solution_amd/efl
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
# config-3 PMC passes: one rocprofv3 run per counter group (TCP <= 4, TA <= 2, TD <= 2, GRBM <= 2)
C3PMC_1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum"
C3PMC_2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
C3PMC_3="TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum"
C3PMC_4="FETCH_SIZE"
C3PMC_5="WRITE_SIZE"
C3PMC_6="TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum"
run() {
  case "$1" in
    tests)  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
              > gpurun_out/r06_pytest.log 2>&1 ;;
    fxpt)   timeout -k 10 600 $PT tests/test_fxp_gpu.py tests/test_bench_launcher.py > gpurun_out/r06_fxp_tests.log 2>&1 ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 ;;
    bench)  timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err ;;
    benchq) timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06_benchq.json 2> gpurun_out/r06_benchq.err ;;
    bench2) timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 3 --no-extras --no-cpu-baseline \
              > gpurun_out/r06_bench_gpus2.json 2> gpurun_out/r06_bench_gpus2.err ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof_trace -o run --output-format csv \
              -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/r06_prof_trace.log 2>&1 ;;
    pmc)    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r06_prof_fetch -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r06_prof_fetch.log 2>&1 && \
            timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r06_prof_write -o run --output-format csv \
              -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r06_prof_write.log 2>&1 ;;
    c3co)   C3_SHAPES="${C3_SHAPES:-e2:512,2,512,2;d1:512,1,512,1;e256:256,1,512,2;d256:512,1,256,2;d128:512,1,128,1}" \
              timeout -k 10 300 python -u tools/config3_coalesce_probe.py >> gpurun_out/r06_c3_shapes.jsonl 2> gpurun_out/r06_c3_shapes.err ;;
    c3kt)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_c3_kt -o run --output-format csv \
              -- python3 tools/config3_probe.py --reps 20 > gpurun_out/r06_c3_kt.log 2>&1 ;;
    c3pmc)  for i in ${C3PMC_PASSES:-4 5 2 6 1 3}; do
              v="C3PMC_$i"
              timeout -s KILL 120 rocprofv3 --pmc ${!v} --kernel-include-regex 'k_batched|k_stream' \
                -d gpurun_out/r06_c3_pmc$i -o run --output-format csv \
                -- python3 tools/config3_probe.py --reps 10 > gpurun_out/r06_c3_pmc$i.log 2>&1 || return $?
              python3 tools/pmc_reduce.py gpurun_out/r06_c3_pmc$i --match batched k_stream --prune \
                > gpurun_out/r06_c3_pmc$i.json || return $?
            done ;;
    c3pmct) for i in ${C3PMC_PASSES:-3 1}; do
              v="C3PMC_$i"
              timeout -s KILL 120 rocprofv3 --pmc ${!v} --kernel-include-regex 'k_batched|k_stream' \
                -d gpurun_out/r06_c3_pmct$i -o run --output-format csv \
                -- python3 tools/config3_probe.py --reps 10 --shapes "default;512,1,512,2,0,0,1,2;512,1,512,2,0,0,1,4;512,1,512,2,0,0,2,1" \
                > gpurun_out/r06_c3_pmct$i.log 2>&1 || return $?
              python3 tools/pmc_reduce.py gpurun_out/r06_c3_pmct$i --match batched k_stream --prune \
                > gpurun_out/r06_c3_pmct$i.json || return $?
            done ;;
    stagep) timeout -k 10 1000 python -u bench.py --stage p > gpurun_out/r06_stage_p${RUN:-}.jsonl 2> gpurun_out/r06_stage_p.err ;;
    stagepq) timeout -k 10 600 python -u bench.py --stage p --no-cpu-baseline > gpurun_out/r06_stage_pq.jsonl 2> gpurun_out/r06_stage_pq.err ;;
    profp)  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof_p -o run --output-format csv \
              -- python3 bench.py --stage p --no-cpu-baseline > gpurun_out/r06_prof_p.log 2>&1 ;;
    mask)   timeout -k 10 300 python -u tools/bench_mask.py > gpurun_out/r06_bench_mask.jsonl 2> gpurun_out/r06_bench_mask.err ;;
    masktests) timeout -k 10 600 $PT tests/test_mask_gpu.py tests/test_secret_sharing_gpu.py tests/test_dp_gpu.py \
              > gpurun_out/r06_mask_tests.log 2>&1 ;;
    pltests) timeout -k 10 900 $PT tests/test_paillier_gpu.py tests/test_paillier_crt_gpu.py tests/test_ctx_abi_gpu.py \
              tests/test_crt_walks_gpu.py tests/test_walk_split_gpu.py > gpurun_out/r06_pltests.log 2>&1 ;;
    c3dec)  C3_LAYOUTS=separate C3_SHAPES="d1:512,1,512,1;d128:512,1,128,1;d256x4:512,1,256,4;d512x4:512,1,512,4;o1:512,1,512,2,0,1;o2:512,1,512,2,0,2;d128o2:512,1,128,1,0,2;e2:512,2,512,2;e2o2:512,2,512,2,2,0;e256:256,2,512,2" \
              timeout -k 10 300 python -u tools/config3_coalesce_probe.py >> gpurun_out/r06_c3_dec.jsonl 2> gpurun_out/r06_c3_dec.err ;;
    c3t)    C3_LAYOUTS=separate C3_SHAPES="e1t2:512,1,512,2,0,0,2,1;e1t4:512,1,512,2,0,0,4,1;e1t8:512,1,512,2,0,0,8,1;d2t2:512,1,512,2,0,0,1,2;d2t4:512,1,512,2,0,0,1,4;d2t8:512,1,512,2,0,0,1,8;e2t4:512,2,512,2,0,0,4,1;d1t8:512,1,512,1,0,0,1,8;both4:512,1,512,2,0,0,4,4;both8:512,1,512,2,0,0,8,4" \
              timeout -k 10 300 python -u tools/config3_coalesce_probe.py >> gpurun_out/r06_c3_tiles.jsonl 2> gpurun_out/r06_c3_tiles.err ;;
    mask9)  timeout -k 10 400 python -u tools/bench_mask.py --rounds 9 --no-cpu-baseline > gpurun_out/r06_bench_mask9.jsonl 2> gpurun_out/r06_bench_mask9.err ;;
    crtt)   timeout -k 10 900 $PT tests/test_crt_walks_gpu.py tests/test_walk_split_gpu.py tests/test_paillier_crt_gpu.py \
              tests/test_ctx_abi_gpu.py > gpurun_out/r06_crt_tests.log 2>&1 ;;
    decab)  for r in 1 2; do
              for v in "" _nofold; do
                EFL_HIP_LIB=$LIBDIR/libefl_hip$v.so timeout -k 10 300 python -u tools/dec_ab.py --label "lib$v" \
                  >> gpurun_out/r06_dec_ab.jsonl 2>> gpurun_out/r06_dec_ab.err || return $?
              done
            done ;;
    dect)   timeout -k 10 900 $PT tests/test_paillier_gpu.py tests/test_paillier_key_sizes_gpu.py -k "decrypt or round_trip" \
              > gpurun_out/r06_dec_tests.log 2>&1 ;;
    decsos) for r in 1 2; do
              for v in "" _ship; do
                EFL_HIP_LIB=$LIBDIR/libefl_hip$v.so timeout -k 10 300 python -u tools/dec_ab.py --label "lib$v" \
                  >> gpurun_out/r06_dec_sos.jsonl 2>> gpurun_out/r06_dec_sos.err || return $?
              done
            done ;;
    decpmc) for v in _fold _nofold; do
              EFL_HIP_LIB=$LIBDIR/libefl_hip$v.so timeout -s KILL 150 rocprofv3 \
                --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES \
                --kernel-include-regex 'k_decrypt' -d gpurun_out/r06_dec_pmc$v -o run --output-format csv \
                -- python3 tools/dec_ab.py --reps 1 --label "lib$v" > gpurun_out/r06_dec_pmc$v.log 2>&1 || return $?
              python3 tools/pmc_reduce.py gpurun_out/r06_dec_pmc$v --match k_decrypt > gpurun_out/r06_dec_pmc$v.json || return $?
            done ;;
    traffic) python3 tools/pmc_traffic.py gpurun_out/r06_prof_fetch/run_counter_collection.csv \
              gpurun_out/r06_prof_write/run_counter_collection.csv 67108864 profiles/r06 > gpurun_out/r06_pmc_traffic.json ;;
    maskpmc) for c in FETCH_SIZE WRITE_SIZE; do
              MASK_SWEEP=0 timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex 'k_mask|k_noise' \
                -d gpurun_out/r06_mask_pmc_$c -o run --output-format csv \
                -- python3 tools/bench_mask.py --steps 5 --rounds 1 --no-cpu-baseline > gpurun_out/r06_mask_pmc_$c.log 2>&1 || return $?
              python3 tools/pmc_reduce.py gpurun_out/r06_mask_pmc_$c --match k_mask k_noise --prune \
                > gpurun_out/r06_mask_pmc_$c.json || return $?
            done ;;
    masklay) timeout -k 10 300 python -u tools/mask_layout_probe.py ${MASKLAY_ARGS:-} >> gpurun_out/r06_mask_layout.jsonl 2> gpurun_out/r06_mask_layout.err ;;
    layer)  timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 > gpurun_out/r06_layer_dense.jsonl 2> gpurun_out/r06_layer_dense.err && \
            timeout -k 10 400 python -u tools/bench_layer.py --steps 3 --warmup 1 --kind weight > gpurun_out/r06_layer_weight.jsonl 2> gpurun_out/r06_layer_weight.err ;;
    spillpmc) timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_WAVE_CYCLES SQ_INSTS \
              -d gpurun_out/r06_spill_pmc -o run --output-format csv \
              -- python3 tools/spill_probe.py > gpurun_out/r06_spill_pmc.log 2>&1 ;;
    crtprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_crt_prof -o run --output-format csv \
              -- python3 tools/crt_tail_ab.py --modes 1,16,8 --rounds 2 > gpurun_out/r06_crt_prof.log 2>&1 ;;
    crtab)  timeout -k 10 400 python -u tools/crt_tail_ab.py >> gpurun_out/r06_crt_tail_ab.jsonl 2> gpurun_out/r06_crt_tail_ab.err ;;
    ab)     timeout -k 10 300 python -u tools/ab_fxp_libs.py r05=$LIBDIR/libefl_hip_r05.so cur=$LIBDIR/libefl_hip.so \
              pre=$LIBDIR/libefl_hip_pre.so >> gpurun_out/r06_ab_libs.jsonl 2> gpurun_out/r06_ab_libs.err ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s $(date +%T)"
  run "$s" || { rc=$?; echo "step $s failed rc=$rc"; exit $rc; }
done
echo "== done $(date +%T)"
