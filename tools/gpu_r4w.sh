#!/bin/bash
# round-4 session W: grouped prefill without the per-K-step division and with packed-fp16 parameter
# offsets -- A/B of two product builds (grouped g128 default + NIB arms, per channel as the control)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "prefill or w4a16 or nib or fused or gemm" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_w.log 2>&1; rc=$?; tail -2 $OUT/t_w.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for pair in base=iron_weight_only_quant_amd/_lib/libiwq_base.so new=iron_weight_only_quant_amd/_lib/libiwq.so; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 200 python tools/ab_gemm.py --lib $lib --tag $tag --group 128 --variants 0,nib --rounds 5 >> $OUT/ab_w.jsonl 2>/dev/null || exit 3
  done
done
for pair in base=iron_weight_only_quant_amd/_lib/libiwq_base.so new=iron_weight_only_quant_amd/_lib/libiwq.so; do
  tag=${pair%%=*}; lib=${pair#*=}
  timeout -k 10 200 python tools/ab_gemm.py --lib $lib --tag pc_$tag --group -2 --variants 0,nib --rounds 5 >> $OUT/ab_w.jsonl 2>/dev/null || exit 3
done
