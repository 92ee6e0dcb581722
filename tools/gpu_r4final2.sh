#!/bin/bash
# round-4 closing validation: product GPU suite, A/B-library parity suite, smoke, PMC traffic of the
# headline kernel (FETCH_SIZE / WRITE_SIZE passes -> profiles/traffic.json on this tree), bench,
# rocprofv3 stats of bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 tmo=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1; local st=$?; echo "=== $name exit $st"; tail -n 3 "$OUT/$name.log" | cut -c1-400; if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "ABORT after $name ($st)"; exit $st; fi; return $st; }
step g_pytest_prod 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
IWQ_AB=1 step g_pytest_ab 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_approx.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
step g_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
cd /tmp
B="python3 $ROOT/bench.py --no-cpu-baseline --no-ppl --no-shapes --no-sections --ramp-seconds 0 --steps 3 --warmup 1"
step g_pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/g_pmc_fetch" -o run -- $B
step g_pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/g_pmc_write" -o run -- $B
step g_traffic 60 python3 "$ROOT/tools/pmc_traffic.py" "$OUT/g_pmc_fetch" "$OUT/g_pmc_write" --numel 6476005376 --kernel "k_group<0, 128, false, 0, true," -o "$OUT/traffic.json"
cp "$OUT/traffic.json" "$ROOT/profiles/traffic.json"
cd "$ROOT"
step g_bench 600 python bench.py
cd /tmp
step g_rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g_prof" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2
cd "$ROOT"
echo "=== done"
