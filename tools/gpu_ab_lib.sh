# A/B of library builds on one box (tools/ab_lib.py): GPU tests on the tree's libiwq.so, then the
# libraries named in AB_LIBS (tag=path pairs) alternated over AB_ROUNDS rounds, one process each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_ab.log
fi
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for pair in $AB_LIBS; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 120 python tools/ab_lib.py --lib "$lib" --tag "$tag" 2>/dev/null | tee -a gpurun_out/${AB_OUT:-ab_lib}.jsonl || exit 1
  done
done
