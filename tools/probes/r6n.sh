set -o pipefail
# round 6 (session 2): FP pack tables with embedded codes + d16 reads -- product suite, A/B identity, A/B timing, bench
O=gpurun_out
PYT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu -x > $O/r6n_pytest_gpu.log 2>&1 || exit $?
IWQ_AB=1 timeout -k 10 600 $PYT tests/test_gpu_fp_unpack.py tests/test_gpu_parity.py -m gpu -x -k "fp or codes or grid or embedded" > $O/r6n_pytest_ab_fp.log 2>&1 || exit $?
IWQ_AB=1 timeout -k 10 600 python -u tools/ab_fp_variants.py --formats 2:1:asym,2:1:sym,4:3:asym,4:3:sym,3:2:asym --variants 0,7 --rounds 5 > $O/r6n_ab_fp_ec.jsonl 2> $O/r6n_ab_fp_ec.err || exit $?
timeout -k 10 600 python -u bench.py > $O/r6n_bench.json 2> $O/r6n_bench.err || exit $?
