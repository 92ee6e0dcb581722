cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/pmc_lds_74 -o run -- python3 $R/tools/gemm_pmc.py --n 4096 --k 11008 > $R/gpurun_out/pmc_lds_74.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/pmc_lds_ref -o run -- python3 $R/tools/gemm_pmc.py --n 4096 --k 11008 --ref > $R/gpurun_out/pmc_lds_ref.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/pmc_lds_74g -o run -- python3 $R/tools/gemm_pmc.py --n 11008 --k 4096 > $R/gpurun_out/pmc_lds_74g.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/pmc_lds_refg -o run -- python3 $R/tools/gemm_pmc.py --n 11008 --k 4096 --ref > $R/gpurun_out/pmc_lds_refg.log 2>&1
