set -o pipefail
# round 6 (session 2): per-tensor one pass with the publish acknowledgement moved behind the sweep
O=gpurun_out
PYT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu -x -k "tensor or onepass or per_tensor" > $O/r6q_pytest_tensor.log 2>&1 || exit $?
IWQ_AB=1 timeout -k 10 600 $PYT tests/test_gpu_parity.py -m gpu -x -k "tensor or onepass" > $O/r6q_pytest_ab_tensor.log 2>&1 || exit $?
IWQ_AB=1 timeout -k 10 600 python -u tools/ab_tensor.py --shapes 11008x4096,4096x11008,4096x4096 --variants 0,10,0,10,0,10,0,10 > $O/r6q_ab_tensor.jsonl 2> $O/r6q_ab_tensor.err || exit $?
