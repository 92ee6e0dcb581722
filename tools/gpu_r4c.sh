#!/bin/bash
# round-4 session C: prefill parity (16x16x32 forms, NIB twins, defaults), A/B of the stagger forms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local st=$?; tail -3 $OUT/$name.log; echo "=== $name exit $st"; return $st; }
run t_prefill_c 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill or nib or w4a16" --timeout 200 --timeout-method thread -p no:cacheprovider
st=$?; [ $st -le 1 ] || exit $st
run ab_c 400 python tools/ab_gemm.py --variants 74,150,151,153,154,155,156 --rounds 9
[ $? -eq 0 ] || exit 3
run ab_c_g128 300 python tools/ab_gemm.py --variants 0 --group 128 --rounds 5
run t_fp_dtypes 400 python -u -m pytest tests/test_gpu_fp_dtypes.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
