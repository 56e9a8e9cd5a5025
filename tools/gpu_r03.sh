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
    pltests) timeout -k 10 600 python -u -m pytest tests/test_paillier_gpu.py tests/test_paillier_scalar_gpu.py tests/test_paillier_layer_gpu.py \
              -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_pltests.log 2>&1 ;;
    crt)    timeout -k 10 600 python -u -m pytest tests/test_paillier_crt_gpu.py tests/test_paillier_gpu.py -m gpu -x -v --timeout 300 \
              --timeout-method thread > gpurun_out/r03_crt.log 2>&1 ;;
    crtp)   timeout -k 10 300 python -u tools/crt_probe.py > gpurun_out/r03_crt_probe.jsonl 2> gpurun_out/r03_crt_probe.err && \
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r03_crt_kt -o run --output-format csv \
              -- python3 tools/crt_probe.py --reps 3 > gpurun_out/r03_crt_kt.log 2>&1 && \
            cp /tmp/r03_crt_kt/run_kernel_stats.csv gpurun_out/r03_crt_kernel_stats.csv ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 ;;
    bench)  timeout -k 10 300 python -u bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_trace -o run --output-format csv \
              -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/r03_prof_trace.log 2>&1 ;;
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
    bprobe) BATCH_ARMS="base:256,2,256,4,0,0;flat:256,2,256,4,1,1;p2048:256,2,256,4,3,3,2048;p4096:256,2,256,4,3,3,4096;p1024:256,2,256,4,3,3,1024;p8192:256,2,256,4,3,3,8192;pe_d0:256,2,256,4,3,0,4096;pe512:512,1,256,4,3,3,4096;pd2:256,2,256,2,3,3,4096" \
            timeout -k 10 300 python -u tools/batched_probe.py > gpurun_out/r03_batched_probe.json 2> gpurun_out/r03_batched_probe.err ;;
    decfam) timeout -k 10 600 python -u tools/sweep_dec_family.py > gpurun_out/r03_dec_family.jsonl 2> gpurun_out/r03_dec_family.err ;;
    c3kt)   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r03_c3_kt -o run --output-format csv \
              -- python3 tools/config3_probe.py --reps 20 > gpurun_out/r03_c3_kt.log 2>&1 && \
            python tools/pmc_reduce.py /tmp/r03_c3_kt --match batched k_stream --prune > gpurun_out/r03_c3_kt.json && \
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r03_c3_kt_flat -o run --output-format csv \
              -- python3 tools/config3_probe.py --reps 20 --order 1 1 > gpurun_out/r03_c3_kt_flat.log 2>&1 && \
            python tools/pmc_reduce.py /tmp/r03_c3_kt_flat --match batched k_stream --prune > gpurun_out/r03_c3_kt_flat.json ;;
    c3pmc)  for pass in "FETCH_SIZE" "WRITE_SIZE" \
                        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM"; do
              tag=$(echo $pass | cut -d' ' -f1)
              timeout -s KILL 120 rocprofv3 --pmc $pass -d /tmp/r03_c3_$tag -o run --output-format csv \
                -- python3 tools/config3_probe.py --reps 3 > gpurun_out/r03_c3_$tag.log 2>&1 || return $?
              python tools/pmc_reduce.py /tmp/r03_c3_$tag --match batched k_stream --prune > gpurun_out/r03_c3_$tag.json || return $?
            done ;;
    grpc)   timeout -k 10 300 python -u tools/grpc_raw_probe.py > gpurun_out/r03_grpc_raw.json 2>&1 && \
            timeout -k 10 400 python -u tools/grpc_probe.py --mib 512 --reps 3 --channels 1 2 > gpurun_out/r03_grpc_probe2.jsonl 2>&1 ;;
    bprobe2) BATCH_ARMS="${BATCH_ARMS:-base:256,2,256,4,0,0;d128k1:256,2,128,1,0,0;d128k2:256,2,128,2,0,0;d256k1:256,2,256,1,0,0;d256k2:256,2,256,2,0,0;d512k1:256,2,512,1,0,0;d512k2:256,2,512,2,0,0;d512k4:256,2,512,4,0,0;base2:256,2,256,4,0,0}" \
            timeout -k 10 300 python -u tools/batched_probe.py > gpurun_out/r03_batched_probe2.json 2> gpurun_out/r03_batched_probe2.err ;;
    c3gap)  timeout -k 10 300 python -u tools/config3_probe.py --reps 50 > gpurun_out/r03_c3_wall.json 2>&1 && \
            timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r03_c3_gap -o run --output-format csv \
              -- python3 tools/config3_probe.py --reps 20 > gpurun_out/r03_c3_gap.log 2>&1 && \
            python tools/kernel_gaps.py /tmp/r03_c3_gap/run_kernel_trace.csv > gpurun_out/r03_c3_gaps.json ;;
    ovh)    timeout -k 10 300 python -u tools/op_overhead_probe.py > gpurun_out/r03_op_overhead.jsonl 2> gpurun_out/r03_op_overhead.err ;;
    grpcopt) timeout -k 10 600 python -u tools/grpc_options_probe.py > gpurun_out/r03_grpc_options.jsonl 2>&1 ;;
    c3lay)  timeout -k 10 300 python -u tools/config3_layout_probe.py > gpurun_out/r03_c3_layout.jsonl 2> gpurun_out/r03_c3_layout.err && \
            PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 300 python -u tools/config3_layout_probe.py \
              >> gpurun_out/r03_c3_layout.jsonl 2>> gpurun_out/r03_c3_layout.err ;;
    c3arms) C3_ARMS="${C3_ARMS:-e512k1:512,1,512,2,0,0;e256k2:256,2,512,2,0,0;d128k1:512,2,128,1,0,0;flat:512,2,512,2,1,1;xcd:512,2,512,2,2,2;e512k4:512,4,512,4,0,0}" \
            timeout -k 10 400 python -u tools/config3_layout_probe.py > gpurun_out/r03_c3_arms.jsonl 2> gpurun_out/r03_c3_arms.err ;;
    tblw)   timeout -k 10 500 python -u tools/table_window_probe.py > gpurun_out/r03_table_window.jsonl 2> gpurun_out/r03_table_window.err ;;
    tblw4)  timeout -k 10 500 python -u tools/table_window_probe.py --n-bytes 512 --a-bytes 256 --group 1 10 11 12 --sizes 65536 \
              > gpurun_out/r03_table_window4096.jsonl 2> gpurun_out/r03_table_window4096.err ;;
    mask)   timeout -k 10 300 python -u tools/bench_mask.py > gpurun_out/r03_bench_mask.jsonl 2> gpurun_out/r03_bench_mask.err ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s $(date +%T)"
  run "$s" || { rc=$?; echo "step $s failed rc=$rc"; exit $rc; }
done
echo "== done $(date +%T)"
