#!/bin/bash
# round-4 session A: the fail-safe per-tensor kernel's tests, then the default bench with the new
# configs[2]/[3]/[4] sections
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dropin_edges.py -x -q -k "tensor or onepass" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_onepass.log 2>&1
st=$?; tail -3 $OUT/t_onepass.log; [ $st -le 1 ] || exit $st
timeout -k 10 600 python bench.py > $OUT/bench_r4a.json 2> $OUT/bench_r4a.err
st=$?; tail -c 600 $OUT/bench_r4a.err; exit $st
