#!/bin/bash
# The one GPU session script (gpurun -- 'bash tools/gpu_session.sh STEPS'): STEPS is a comma list of
# the named steps below, run in that order.  Each GPU step has its own time limit; a crash / abort /
# timeout (any status other than 0 or pytest's "tests failed" = 1) ends the session there.
# Outputs under gpurun_out/ (TAG prefixes the file names: TAG=r5a tools/gpu_session.sh ...).
#
#   tests      product GPU suite (pytest -m gpu)          abtests   A/B-library bit-identity suites
#   subset     pytest -m gpu -k "$PYTEST_K" [$PYTEST_FILES]
#   smoke      __graft_entry__.smoke()                     bench     python bench.py (the driver's command)
#   marks      rocprofv3 --kernel-trace --stats of the default bench with --mark-file, cut per bench
#              region by tools/trace_sections.py (per-workload kernel averages beside bench's numbers)
#   prof       rocprofv3 --kernel-trace --stats of bench.py (whole run)
#   pmc        FETCH_SIZE / WRITE_SIZE passes of the 7B headline -> traffic.json (hash-stamped)
#   pmc70      the same for the 70B in-place launch -> traffic_70b.json
#   pmcsq      SQ counters of the 7B headline
#   single     tools/single_trace.py per variant in $SINGLE_VARIANTS (A/B library) + a kernel trace
#   abgemm     tools/ab_gemm.py $AB_GEMM_ARGS             abformats tools/ab_formats_lib.py $AB_FMT_ARGS
#   ablib      tools/ab_lib.py $AB_LIB_ARGS                gemvcold  tools/bench_gemv_cold.py $GEMV_ARGS
#   formats    tools/bench_formats.py                      ppl       tools/ppl_delta.py on random OPT-125M
#   b70        bench.py --model llama2-70b                 inplace   bench.py --inplace
#   dist2      2 ranks sharing cuda:0 over gloo (the multi-rank plumbing; not a scaling point)
#   gpmc       MFMA / VALU counters of tools/gemm_pmc.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
T=${TAG:+${TAG}_}
step() {  # step <name> <timeout> <cmd...>
  local name=$T$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local st=$?
  echo "=== $name exit $st"
  tail -n 4 "$OUT/$name.log" | cut -c1-600
  if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "ABORT session after $name (status $st)"; exit $st; fi
  return $st
}
PYT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread"
HEAD="--no-cpu-baseline --no-ppl --no-shapes --no-sections --ramp-seconds 0 --steps 3 --warmup 1"
IFS=',' read -ra STEPS <<< "${1:-tests,smoke,bench}"
for s in "${STEPS[@]}"; do
  case $s in
    tests) step pytest_gpu 1000 $PYT tests -m gpu ;;
    abtests) IWQ_AB=1 step pytest_gpu_ab 700 $PYT tests/test_gpu_parity.py tests/test_gpu_approx.py tests/test_gpu_fp_unpack.py -m gpu ;;
    subset) step pytest_subset 900 $PYT ${PYTEST_FILES:-tests} -m gpu -x -k "$PYTEST_K" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    marks)
      cd /tmp
      step prof_marks 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${T}prof_marks" -o run -- \
        python3 "$ROOT/bench.py" --mark-file "$OUT/${T}marks.jsonl"
      cd "$ROOT"
      step sections 120 python3 tools/trace_sections.py "$OUT/${T}prof_marks" "$OUT/${T}marks.jsonl" \
        -o "$OUT/${T}sections.json" ;;
    prof)
      cd /tmp
      step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${T}prof" -o run -- \
        python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2
      cd "$ROOT" ;;
    pmc)
      cd /tmp
      step pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/${T}pmc_fetch" -o run -- python3 "$ROOT/bench.py" $HEAD
      step pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/${T}pmc_write" -o run -- python3 "$ROOT/bench.py" $HEAD
      cd "$ROOT"
      step traffic 60 python3 tools/pmc_traffic.py "$OUT/${T}pmc_fetch" "$OUT/${T}pmc_write" --numel 6476005376 \
        --kernel "k_group<0, 128, false, 0, true, 4, false, true, true, true, false, false, 256>" -o "$OUT/${T}traffic.json" ;;
    pmc70)
      cd /tmp
      step pmc70_fetch 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/${T}pmc70_fetch" -o run -- python3 "$ROOT/bench.py" --model llama2-70b $HEAD
      step pmc70_write 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/${T}pmc70_write" -o run -- python3 "$ROOT/bench.py" --model llama2-70b $HEAD
      cd "$ROOT"
      step traffic70 60 python3 tools/pmc_traffic.py "$OUT/${T}pmc70_fetch" "$OUT/${T}pmc70_write" --numel 68451041280 \
        --kernel "k_group<0, 128, false, 0, true, 4, false, true, true, true, false, false, 256>" --placement in-place -o "$OUT/${T}traffic_70b.json" ;;
    pmcsq)
      cd /tmp
      step pmc_sq 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/${T}pmc_sq" -o run -- python3 "$ROOT/bench.py" $HEAD
      cd "$ROOT" ;;
    single)
      for v in ${SINGLE_VARIANTS:-0}; do
        IWQ_AB=1 step single_v$v 200 python tools/single_trace.py --variant $v ${SINGLE_ARGS:-}
      done
      cd /tmp
      step trace_single 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${T}trace_single" -o run -- python3 "$ROOT/tools/single_trace.py" ${SINGLE_ARGS:-}
      cd "$ROOT"
      step trace_gaps 60 python3 tools/trace_gaps.py "$OUT/${T}trace_single" ;;
    abgemm) step ab_gemm 600 python tools/ab_gemm.py $AB_GEMM_ARGS ;;
    abformats) step ab_formats 600 python tools/ab_formats_lib.py $AB_FMT_ARGS ;;
    ablib) step ab_lib 600 python tools/ab_lib.py $AB_LIB_ARGS ;;
    gemvcold) step gemv_cold 600 python tools/bench_gemv_cold.py ${GEMV_ARGS:-} ;;
    formats) step bench_formats 600 python tools/bench_formats.py ;;
    ppl)
      step ppl_opt125m 600 python tools/ppl_delta.py --random opt-125m --synthetic_tokens 65536 --w_bits 8 4 --w_group_size -2
      step ppl_opt125m_g128 600 python tools/ppl_delta.py --random opt-125m --synthetic_tokens 65536 --w_bits 4 3 --w_group_size 128 ;;
    b70) step bench70b 900 python bench.py --model llama2-70b --steps 5 --warmup 2 --cpu-seconds 8 ;;
    inplace) step bench_inplace 600 python bench.py --no-cpu-baseline --inplace ;;
    dist2)
      export IWQ_DIST_BACKEND=gloo
      step dist2_7b 600 python bench.py --gpus 2 --steps 5 --warmup 2
      step dist2_70b 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --model llama2-70b --steps 3 --warmup 1 --no-collectives
      unset IWQ_DIST_BACKEND ;;
    gpmc)
      cd /tmp
      step gemm_pmc 600 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$OUT/${T}gemm_pmc" -o run -- python3 "$ROOT/tools/gemm_pmc.py" ${GPMC_ARGS:-}
      cd "$ROOT" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== session done"
