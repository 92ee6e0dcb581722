set -o pipefail
O=gpurun_out
export IWQ_AB=1
for g in -2 128; do
timeout -k 10 300 python -u tools/bench_gemv_cold.py --shapes q_proj,down_proj --m 1,16 --group $g --variants 0,107,105,106 --layouts tiled --no-ref >> $O/r6j_gemv_xstream.jsonl 2>> $O/r6j.err || exit $?
done
