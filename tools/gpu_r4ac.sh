#!/bin/bash
# round-4 session AC: NIB codes on group-major parameters take the one-wave-per-SIMD form 165 -- A/B of two
# product builds (nibgm arm), parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "prefill or w4a16 or nib or fused or group_major or quantlinear" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_ac.log 2>&1; rc=$?; tail -2 $OUT/t_ac.log; [ $rc -eq 0 ] || exit $rc
IWQ_AB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "group_major or b32 or nib" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_ac_ab.log 2>&1; rc=$?; tail -2 $OUT/t_ac_ab.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for pair in base=iron_weight_only_quant_amd/_lib/libiwq_base.so new=iron_weight_only_quant_amd/_lib/libiwq.so; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 250 python tools/ab_gemm.py --lib $lib --tag $tag --group 128 --variants nibgm --shapes q_proj,gate_proj,down_proj,70b_q,70b_down --rounds 5 >> $OUT/ab_ac.jsonl 2>/dev/null || exit 3
  done
done
