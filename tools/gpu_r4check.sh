#!/bin/bash
# round-4 last check of the libraries as committed: product GPU suite + smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/h_pytest_prod.log 2>&1; rc=$?; tail -2 $OUT/h_pytest_prod.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/h_smoke.log 2>&1; rc=$?; tail -1 $OUT/h_smoke.log; exit $rc
