#!/bin/bash
# round-4 session Q: approx tests (both libraries), single-call walk at 8 waves / SIMD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 tmo=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1; local st=$?; echo "=== $name exit $st"; tail -n 3 "$OUT/$name.log"; if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "ABORT after $name ($st)"; exit $st; fi; return $st; }
step q_approx_prod 300 python -u -m pytest tests/test_gpu_approx.py -q -p no:cacheprovider --timeout 200 --timeout-method thread
IWQ_AB=1 step q_approx_ab 300 python -u -m pytest tests/test_gpu_approx.py -q -p no:cacheprovider --timeout 200 --timeout-method thread
export IWQ_AB=1
for v in 0 1 2 14 15 0 14 15; do
  step single_q_$v 200 python tools/single_trace.py --variant $v
done
cat $OUT/single_q_*.log | grep shape
