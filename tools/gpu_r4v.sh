#!/bin/bash
# round-4 session V: is the grouped prefill's gap clock (operand entropy) or work?  grouped 150 on
# data / power-of-two / unit scales, per channel 151 beside it, hipBLASLt on the matching weight
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for sc in data pow2 ones; do
  timeout -k 10 200 python tools/ab_gemm.py --group 128 --variants 0 --shapes q_proj,down_proj --scales $sc --tag g128_$sc >> $OUT/ab_v.jsonl || exit 3
  timeout -k 10 200 python tools/ab_gemm.py --group -2 --variants 0 --shapes q_proj,down_proj --scales $sc --tag pc_$sc >> $OUT/ab_v.jsonl || exit 3
done
