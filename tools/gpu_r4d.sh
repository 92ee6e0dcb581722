#!/bin/bash
# round-4 session D: grouped 16x16x32 prefill parity + A/B (g128, 7B and 70B shapes), per-channel 70B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local st=$?; tail -3 $OUT/$name.log; echo "=== $name exit $st"; return $st; }
run t_prefill_d 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill_b32 or nib_default or short_k" --timeout 200 --timeout-method thread -p no:cacheprovider
st=$?; [ $st -le 1 ] || exit $st
run ab_d_g128 400 python tools/ab_gemm.py --group 128 --variants 74,150,151,157,153 --rounds 7
[ $? -eq 0 ] || exit 3
run ab_d_g128_70b 400 python tools/ab_gemm.py --group 128 --variants 74,151 --shapes 70b_q,70b_gate,70b_down --rounds 5
[ $? -eq 0 ] || exit 3
run ab_d_pc_70b 400 python tools/ab_gemm.py --variants 74,151,153 --shapes 70b_q,70b_gate,70b_down --rounds 5
