set -o pipefail
O=gpurun_out
export IWQ_AB=1
for g in -2 128; do
timeout -k 10 400 python -u tools/bench_gemv_cold.py --shapes q_proj,down_proj,qkv_fused,gate_up_fused --m 1,8,16 --group $g --variants 0,200,201,203,207,221,223,227 --layouts tiled --no-ref >> $O/r6k_gemv_ksx.jsonl 2>> $O/r6k.err || exit $?
done
