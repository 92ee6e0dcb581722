#!/bin/bash
# Prefill GEMM diagnostics on one box: interleaved A/B timing, then PMC passes (one rocprofv3 run per
# counter set, kernel trace for durations) for each arm on q_proj and down_proj.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
VARS=${VARS:-0,45,47}
SHAPES=${SHAPES:-"4096x4096 4096x11008"}
GRPS=${GRPS:--2}   # weight groups to profile, e.g. "-2 128" (per channel and g128)
if [ -z "$NO_AB" ]; then
  timeout -k 10 300 python tools/ab_gemm.py --variants "$VARS" > "$OUT/ab_gemm_pc.jsonl" 2>&1 || exit $?
  timeout -k 10 300 python tools/ab_gemm.py --variants "$VARS" --group 128 > "$OUT/ab_gemm_g128.jsonl" 2>&1 || exit $?
fi
cd /tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
# issue back-pressure: LDS / TA FIFOs full, VMEM issue cycles, VALU + MFMA co-execution
P3="SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
PASSES=${PASSES:-"1 2"}
for shape in $SHAPES; do
  N=${shape%x*}; K=${shape#*x}
  for g in $GRPS; do
  for arm in ref $(echo $VARS | tr ',' ' '); do
    if [ $arm = ref ]; then A="--ref"; else A="--variant $arm"; fi
    for p in $PASSES; do
      eval C=\$P$p
      D=$OUT/pmc_${N}x${K}_g${g}_${arm}_p$p
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $D -o run -- python3 $ROOT/tools/gemm_pmc.py --n $N --k $K --group $g $A > $D.log 2>&1 || { echo "pmc fail $D"; exit 3; }
    done
  done
  done
done
cd $ROOT
for D in $OUT/pmc_*_p[0-9]; do echo "== $D"; python3 tools/pmc_kernels.py $D; done > $OUT/pmc_gemm_summary.txt 2>&1
echo ok
