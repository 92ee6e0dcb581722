#!/bin/bash
# round-4 session Z: single-call walk with the grid's two halves half an iteration apart (STG, A/B 16 / 17)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
export IWQ_AB=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "group_major or single or variants" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_z.log 2>&1; rc=$?; tail -2 $OUT/t_z.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in 0 16 17; do
    timeout -k 10 120 python tools/single_trace.py --variant $v >> $OUT/ab_z.jsonl 2>/dev/null || exit 3
  done
done
