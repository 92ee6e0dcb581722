#!/bin/bash
# round-4 session E: grouped prefill with group-major parameters (A/B), per-channel epilogue diagnostic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local st=$?; tail -3 $OUT/$name.log; echo "=== $name exit $st"; return $st; }
run t_prefill_e 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill_b32 or nib_default or short_k" --timeout 200 --timeout-method thread -p no:cacheprovider
st=$?; [ $st -le 1 ] || exit $st
run ab_e_g128 400 python tools/ab_gemm.py --group 128 --variants 74,150,157,158,159,160 --rounds 7
[ $? -eq 0 ] || exit 3
run ab_e_g128_70b 400 python tools/ab_gemm.py --group 128 --variants 74,150,158,159 --shapes 70b_q,70b_down --rounds 5
[ $? -eq 0 ] || exit 3
run ab_e_pc 400 python tools/ab_gemm.py --variants 151,161 --shapes q_proj,down_proj,70b_q --rounds 7
