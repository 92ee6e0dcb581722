#!/bin/bash
# round-4 session X: group-major parameter copies for the grouped prefill (IWQ_FLAG_GROUP_MAJOR):
# parity tests, then in-run A/B against the reference-order call and hipBLASLt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_quantize_model.py -k "group_major or nib or prefill_default or quantlinear or quantize_model" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_x.log 2>&1; rc=$?; tail -2 $OUT/t_x.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python tools/ab_gemm.py --group 128 --variants 0,nib,gm,nibgm --shapes q_proj,gate_proj,down_proj,70b_q,70b_down --rounds 5 --tag r$r >> $OUT/ab_x.jsonl 2>/dev/null || exit 3
done
