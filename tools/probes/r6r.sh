set -o pipefail
# round 6 (session 2): FP table kernel addressed per iteration (imm offsets per unit) -- identity + timing
O=gpurun_out
PYT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread"
IWQ_AB=1 timeout -k 10 600 $PYT tests/test_gpu_fp_unpack.py tests/test_gpu_parity.py -m gpu -x -k "fp or codes or grid or embedded" > $O/r6r_pytest_ab_fp.log 2>&1 || exit $?
IWQ_AB=1 timeout -k 10 600 python -u tools/ab_fp_variants.py --formats 2:1:asym,4:3:asym,2:1:sym,4:3:sym,3:2:asym --variants 0,7 --rounds 5 > $O/r6r_ab_fp.jsonl 2> $O/r6r_ab_fp.err || exit $?
