set -o pipefail
O=gpurun_out
export IWQ_AB=1
for g in -2 128; do
timeout -k 10 400 python -u tools/bench_gemv_cold.py --shapes q_proj,down_proj,qkv_fused --m 1,16 --group $g --variants 0,203,241,243,247 --layouts tiled --no-ref >> $O/r6m_gemv_ksx_xcd.jsonl 2>> $O/r6m.err || exit $?
done
