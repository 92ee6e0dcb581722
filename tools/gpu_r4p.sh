#!/bin/bash
# round-4 session P: persistent prefill v3 (saddr DMA) parity + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 tmo=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1; local st=$?; echo "=== $name exit $st"; tail -n 4 "$OUT/$name.log"; if [ $st -ne 0 ]; then echo "ABORT after $name ($st)"; exit $st; fi; return $st; }
export IWQ_AB=1
step t_ab_p 500 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefill_b32 or nib_default or short_k or persistent" --timeout 200 --timeout-method thread -p no:cacheprovider
step ab_p_pc 400 python tools/ab_gemm.py --variants 151,153,171,172 --shapes q_proj,gate_proj,down_proj,70b_q,70b_gate,70b_down --rounds 5
step ab_p_g128 400 python tools/ab_gemm.py --group 128 --variants 150,152,171,172 --shapes q_proj,gate_proj,down_proj,70b_q --rounds 5
