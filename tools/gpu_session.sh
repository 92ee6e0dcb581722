#!/bin/bash
# One gpurun session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/abort/timeout (status >= 2 other than pytest's
# "tests failed" = 1) ends the session immediately.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local st=$?
  echo "=== $name exit $st"
  tail -n 5 "$OUT/$name.log"
  if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "ABORT session after $name (status $st)"; exit $st; fi
  return $st
}
WHAT=${1:-all}
if [[ $WHAT == all || $WHAT == *fulltests* ]]; then
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if [[ $WHAT == *newtests* ]]; then
  step pytest_new 900 python -u -m pytest ${NEWTESTS:-tests/test_gpu_quantize_model.py} -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if [[ $WHAT == all || $WHAT == *smoke* ]]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $WHAT == all || $WHAT == *bench* ]]; then
  step bench 600 python bench.py
fi
if [[ $WHAT == all || $WHAT == *prof* ]]; then
  cd /tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2
  cd "$ROOT"
fi
if [[ $WHAT == *inplace* ]]; then
  step bench_inplace 600 python bench.py --no-cpu-baseline --inplace
fi
if [[ $WHAT == *b70* ]]; then
  step bench70b 900 python bench.py --model llama2-70b --steps 5 --warmup 2 --cpu-seconds 8
fi
if [[ $WHAT == *gemvcold* ]]; then
  step gemv_cold 600 python tools/bench_gemv_cold.py ${GEMV_ARGS:-}
fi
if [[ $WHAT == *gemm* ]]; then
  step bench_gemm 600 python tools/bench_gemm.py ${GEMM_ARGS:-}
fi
if [[ $WHAT == *ppl* ]]; then
  step ppl_opt125m 600 python tools/ppl_delta.py --random opt-125m --synthetic_tokens 65536 --w_bits 8 4 --w_group_size -2
  step ppl_opt125m_g128 600 python tools/ppl_delta.py --random opt-125m --synthetic_tokens 65536 --w_bits 4 3 --w_group_size 128
fi
if [[ $WHAT == *formats* ]]; then
  step bench_formats 600 python tools/bench_formats.py
  cd /tmp
  step prof_formats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_formats" -o run -- python3 "$ROOT/tools/bench_formats.py" --reps 10
  cd "$ROOT"
fi
if [[ $WHAT == *gpmc* ]]; then
  cd /tmp
  step gemm_pmc 600 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$OUT/gemm_pmc" -o run -- python3 "$ROOT/tools/gemm_pmc.py"
  step gemm_pmc_dec 600 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$OUT/gemm_pmc_dec" -o run -- python3 "$ROOT/tools/gemm_pmc.py" --m 1 --n 28672 --k 8192
  cd "$ROOT"
fi
if [[ $WHAT == *ab* ]]; then
  step ab 600 python bench.py --no-cpu-baseline --variants "${AB_VARIANTS:-0,1,2,3,4,5,6,7,8}" --steps 10 --rounds 5
fi
if [[ $WHAT == *single* ]]; then
  step ab_single 600 python tools/ab_single.py ${SINGLE_ARGS:-}
  step ab_single_4096 600 python tools/ab_single.py --rows 4096 --cols 4096 --copies 64 ${SINGLE_ARGS:-}
fi
if [[ $WHAT == *dist2* ]]; then
  # rehearsal of the multi-rank bench on a 1-GPU box: 2 ranks share cuda:0 over gloo
  export IWQ_DIST_BACKEND=gloo
  # the driver's command form without torchrun: bench.py spawns its own ranks
  step dist2_7b 600 python bench.py --gpus 2 --steps 5 --warmup 2 --gather
  step dist2_70b 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --model llama2-70b --steps 3 --warmup 1
  step dist2_7b_sg 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --model llama2-7b --steps 3 --warmup 1 --scatter --gather --no-shapes
  unset IWQ_DIST_BACKEND
fi
if [[ $WHAT == *pmc* ]]; then
  cd /tmp
  B="python3 $ROOT/bench.py --no-cpu-baseline --no-ppl --no-shapes --no-sections --ramp-seconds 0 --steps 3 --warmup 1"
  step pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $B
  step pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $B
  step traffic 60 python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" --numel 6476005376 --kernel "k_group<0, 128, false, 0, true," -o "$OUT/traffic.json"
  step pmc_sq 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o run -- $B
  cd "$ROOT"
fi
echo "=== session done"
