#!/bin/bash
# round-4 validation: product GPU suite, A/B-library parity suite, smoke, bench, rocprofv3 stats of bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 tmo=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1; local st=$?; echo "=== $name exit $st"; tail -n 3 "$OUT/$name.log" | cut -c1-400; if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "ABORT after $name ($st)"; exit $st; fi; return $st; }
step f_pytest_prod 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
IWQ_AB=1 step f_pytest_ab 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_approx.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
step f_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step f_bench 600 python bench.py
cd /tmp
step f_rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/f_prof" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2
cd "$ROOT"
echo "=== done"
