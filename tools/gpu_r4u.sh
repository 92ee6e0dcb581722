#!/bin/bash
# round-4 session U: FP pack (k_fp_group_lut) with the next iteration's loads prefetched, A/B of two product builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp_dtypes.py tests/test_gpu_approx.py tests/test_gpu_random_sweep.py -k "fp or apx or approx or batched or sweep" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_u.log 2>&1; rc=$?; tail -2 $OUT/t_u.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for pair in base=iron_weight_only_quant_amd/_lib/libiwq_base.so new=iron_weight_only_quant_amd/_lib/libiwq.so; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 200 python tools/ab_formats_lib.py --lib $lib --tag $tag >> $OUT/ab_u.jsonl 2>/dev/null || exit 3
  done
done
