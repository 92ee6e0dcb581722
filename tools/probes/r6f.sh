set -o pipefail
O=gpurun_out
PYT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gpu_fullsize.py tests/test_gpu_quantize_model.py -m gpu -x > $O/r6f_pytest_full.log 2>&1 || exit $?
IWQ_AB=1 timeout -k 10 600 $PYT tests/test_gpu_parity.py -m gpu -x -k "gemv or ksplit or large_x or w4a16_gemm_vs" > $O/r6f_pytest_gemv.log 2>&1 || exit $?
IWQ_AB=1 timeout -k 10 500 python -u tools/bench_gemv_cold.py --shapes q_proj,down_proj,qkv_fused,gate_up_fused --m 8,16 --group -2 --variants 32,31 --layouts tiled --no-ref > $O/r6f_gemv_ks_pc.jsonl 2> $O/r6f_gemv_ks_pc.err || exit $?
IWQ_AB=1 timeout -k 10 500 python -u tools/bench_gemv_cold.py --shapes q_proj,down_proj,qkv_fused,gate_up_fused --m 8,16 --group 128 --variants 32,31 --layouts tiled --no-ref > $O/r6f_gemv_ks_g128.jsonl 2> $O/r6f_gemv_ks_g128.err || exit $?
timeout -k 10 600 python -u bench.py > $O/r6f_bench.json 2> $O/r6f_bench.err || exit $?
