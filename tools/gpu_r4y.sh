#!/bin/bash
# round-4 session Y: the grouped 16x16x32 forms on group-major parameters (A/B library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 250 python tools/ab_gemm.py --lib iron_weight_only_quant_amd/_lib/libiwq_ab.so --group 128 --variants gm150,gm152,gm153,gm163,gm165,gm169,gm172 --shapes q_proj,down_proj,70b_q --rounds 5 --tag r$r >> $OUT/ab_y.jsonl 2>/dev/null || exit 3
done
