#!/bin/bash
# round-4 session M: product GPU suite, A/B-library parity suite, single-call walk variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 tmo=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1; local st=$?; echo "=== $name exit $st"; tail -n 4 "$OUT/$name.log"; if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "ABORT after $name ($st)"; exit $st; fi; return $st; }
step m_pytest_prod 1000 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
IWQ_AB=1 step m_pytest_ab 700 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
export IWQ_AB=1
for v in 0 9 10 11 12 13 0i 5i 9i; do
  case $v in *i) A="--inplace --variant ${v%i}";; *) A="--variant $v";; esac
  step single_l_$v 200 python tools/single_trace.py $A
done
