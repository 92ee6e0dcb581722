# A/B of library builds on the FP / format paths (tools/bench_formats.py --lib): FP GPU tests on the
# tree's libiwq.so, then AB_LIBS (tag=path pairs) alternated over AB_ROUNDS rounds, one process each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp_unpack.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fp or grid or unpack" > gpurun_out/pytest_abf.log 2>&1 || { tail -30 gpurun_out/pytest_abf.log; exit 1; }
tail -2 gpurun_out/pytest_abf.log
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for pair in $AB_LIBS; do
    tag=${pair%%=*}; lib=${pair#*=}
    timeout -k 10 180 python tools/bench_formats.py --lib "$lib" --tag "$tag" --only "$AB_ONLY" 2>/dev/null | tee -a gpurun_out/${AB_OUT:-ab_formats}.jsonl || exit 1
  done
done
