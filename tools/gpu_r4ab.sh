#!/bin/bash
# round-4 session AB: b16w epilogue as quad-transposed 8-B stores -- A/B of two product builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fused_proj.py -k "prefill or w4a16 or nib or fused or gemm or group_major or quantlinear" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_ab.log 2>&1; rc=$?; tail -2 $OUT/t_ab.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for pair in base=iron_weight_only_quant_amd/_lib/libiwq_base.so new=iron_weight_only_quant_amd/_lib/libiwq.so; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 200 python tools/ab_gemm.py --lib $lib --tag pc_$tag --group -2 --variants 0 --rounds 5 >> $OUT/ab_ab.jsonl 2>/dev/null || exit 3
    timeout -k 10 200 python tools/ab_gemm.py --lib $lib --tag $tag --group 128 --variants gm,nibgm --rounds 5 >> $OUT/ab_ab.jsonl 2>/dev/null || exit 3
  done
done
