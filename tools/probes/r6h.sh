set -o pipefail
O=gpurun_out
R=$(pwd)
export IWQ_AB=1
timeout -k 10 300 python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -x -k "warp_specialised" > $O/r6h_pytest_ws.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/ab_gemm.py --variants 0,180,181,183 --shapes q_proj,gate_proj,down_proj --m 8192 > $O/r6h_ab_ws.jsonl 2> $O/r6h_ab_ws.err || exit $?
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for v in 181 183; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $R/$O/r6h_pmc_${v}_p1 -o run -- python3 $R/tools/gemm_pmc.py --n 4096 --k 11008 --variant $v > $R/$O/r6h_pmc_${v}_p1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $R/$O/r6h_pmc_${v}_p2 -o run -- python3 $R/tools/gemm_pmc.py --n 4096 --k 11008 --variant $v > $R/$O/r6h_pmc_${v}_p2.log 2>&1 || exit $?
done
