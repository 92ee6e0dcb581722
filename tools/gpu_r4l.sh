#!/bin/bash
# round-4 session L: single-call walk variants (9-13), in place
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
export IWQ_AB=1
for v in 0 9 10 11 12 13 0i 5i 9i; do
  case $v in *i) A="--inplace --variant ${v%i}";; *) A="--variant $v";; esac
  timeout -k 10 200 python tools/single_trace.py $A > $OUT/single_l_$v.log 2>&1 || exit 3
done
cat $OUT/single_l_*.log
