#!/bin/bash
# round-4 session B: the 16x16x32 prefill variants (parity, then interleaved A/B vs 74 and hipBLASLt),
# then the whole GPU suite and smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local st=$?; tail -3 $OUT/$name.log; echo "=== $name exit $st"; return $st; }
run t_prefill 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill_b32 or prefill_short_k" --timeout 120 --timeout-method thread -p no:cacheprovider
st=$?; [ $st -le 1 ] || exit $st
run ab_b16 300 python tools/ab_gemm.py --variants 0,150,151 --rounds 7
[ $? -eq 0 ] || exit 3
run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
st=$?; [ $st -le 1 ] || exit $st
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
