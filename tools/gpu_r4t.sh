#!/bin/bash
# round-4 session T: FP unpack with hoisted parameter loads + prefetch, A/B of two product builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp_unpack.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_t.log 2>&1; tail -2 $OUT/t_t.log
for r in 1 2 3; do
  for pair in base=iron_weight_only_quant_amd/_lib/libiwq_base.so new=iron_weight_only_quant_amd/_lib/libiwq.so; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 200 python tools/ab_formats_lib.py --lib $lib --tag $tag >> $OUT/ab_t.jsonl 2>/dev/null || exit 3
  done
done
