#!/bin/bash
# round-4 session S: two AB-library builds (compiler-tracked v_and_or_b32 vs inline asm) alternated
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
export IWQ_AB=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill_b32 or nib_default or short_k or persistent" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_ab_s.log 2>&1 || { tail -20 $OUT/t_ab_s.log; exit 1; }
tail -1 $OUT/t_ab_s.log
for r in 1 2 3; do
  for pair in base=iron_weight_only_quant_amd/_lib/libiwq_ab_base.so new=iron_weight_only_quant_amd/_lib/libiwq_ab.so; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 200 python tools/ab_gemm.py --lib $lib --tag $tag --variants 151,153,172 --shapes q_proj,down_proj,70b_q --rounds 3 >> $OUT/ab_s.jsonl 2>/dev/null || exit 3
  done
done
