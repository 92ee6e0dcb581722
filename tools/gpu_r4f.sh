#!/bin/bash
# round-4 session F: one-wave-per-SIMD prefill (162 / 163) parity + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local st=$?; tail -3 $OUT/$name.log; echo "=== $name exit $st"; return $st; }
run t_prefill_f 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill_b32 or nib_default or short_k" --timeout 200 --timeout-method thread -p no:cacheprovider
st=$?; [ $st -le 1 ] || exit $st
[ $st -eq 0 ] || exit 1
run ab_f_pc 400 python tools/ab_gemm.py --variants 151,153,162,163 --rounds 7
[ $? -eq 0 ] || exit 3
run ab_f_pc70 400 python tools/ab_gemm.py --variants 151,153,162,163 --shapes 70b_q,70b_gate,70b_down --rounds 5
