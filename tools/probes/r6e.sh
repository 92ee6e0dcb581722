set -o pipefail
export IWQ_AB=1
O=gpurun_out
timeout -k 10 500 python -u tools/ab_outplace.py --variants 0,118,155,156,157,158,159,160,161 --shifts 0 --skews "" --out $O/r6e_walks.jsonl > $O/r6e_walks.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_gemv_cold.py --shapes q_proj,down_proj,qkv_fused,gate_up_fused --m 1,8,16 --group -2 --variants 0,29,30 --layouts tiled --no-ref > $O/r6e_gemv_pc.jsonl 2> $O/r6e_gemv_pc.err || exit $?
timeout -k 10 400 python -u tools/bench_gemv_cold.py --shapes q_proj,down_proj,qkv_fused,gate_up_fused --m 1,8,16 --group 128 --variants 0,29,30 --layouts tiled --no-ref > $O/r6e_gemv_g128.jsonl 2> $O/r6e_gemv_g128.err || exit $?
timeout -k 10 400 python -u tools/ab_fp_variants.py --formats 2:1:asym,4:3:asym,4:3:sym --variants 0,1,3,4 --out $O/r6e_fp.jsonl > $O/r6e_fp.log 2>&1 || exit $?
unset IWQ_AB
timeout -k 10 300 python -u tools/bench_tensor_dt.py --shapes 4096x4096,11008x4096 --dtypes float16 > $O/r6e_tensor.jsonl 2> $O/r6e_tensor.err || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "tensor or onepass or workspace or gemv or decode" > $O/r6e_pytest.log 2>&1
