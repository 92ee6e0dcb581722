#!/bin/bash
# round-4 session AA: quant_dim 1 on the persistent LDS-staged column kernel (A/B variant 5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
export IWQ_AB=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "quant_dim1" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_aa.log 2>&1; rc=$?; tail -2 $OUT/t_aa.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for g in 128 64; do
    timeout -k 10 120 python tools/ab_col.py --group $g --variants 0,5,0,5 >> $OUT/ab_aa.jsonl 2>/dev/null || exit 3
  done
done
