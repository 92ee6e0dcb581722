#!/bin/bash
# round-4 session K: b16r parity + A/B; single-call trace (kernel vs boundary) + single-walk A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local st=$?; tail -3 $OUT/$name.log; echo "=== $name exit $st"; return $st; }
export IWQ_AB=1
run t_ab_k 500 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill_b32 or nib_default or short_k" --timeout 200 --timeout-method thread -p no:cacheprovider
[ $? -eq 0 ] || exit 1
run ab_k_pc 400 python tools/ab_gemm.py --variants 165,168,169,170 --shapes q_proj,gate_proj,down_proj,70b_q --rounds 7
[ $? -eq 0 ] || exit 3
run ab_k_g128 400 python tools/ab_gemm.py --group 128 --variants 150,165,168,169,170 --rounds 5
[ $? -eq 0 ] || exit 3
for v in 0 3 4 5 6 7 8; do
  run single_v$v 200 python tools/single_trace.py --variant $v || exit 3
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_single -o run -- python3 $ROOT/tools/single_trace.py > $OUT/trace_single.log 2>&1 || exit 3
cd $ROOT && python3 tools/trace_gaps.py $OUT/trace_single > $OUT/trace_single_gaps.txt
