set -o pipefail
# round 6 (session 2): PMC passes over the FP pack kernels on the final tree (SQ issue counters, HBM bytes)
O=$(pwd)/gpurun_out
R=$(pwd)
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/r6t_pmc_sq -o run -- python3 $R/tools/fp_pack_run.py > $O/r6t_pmc_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/r6t_pmc_fetch -o run -- python3 $R/tools/fp_pack_run.py > $O/r6t_pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/r6t_pmc_write -o run -- python3 $R/tools/fp_pack_run.py > $O/r6t_pmc_write.log 2>&1 || exit $?
