cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/k2pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-trace -d $R/gpurun_out/k2pmc/p1 -o run --output-format csv -- python3 $R/tools/k2_only.py > $R/gpurun_out/k2pmc/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/k2pmc/p2 -o run --output-format csv -- python3 $R/tools/k2_only.py > $R/gpurun_out/k2pmc/p2.log 2>&1 || exit $?
cd $R && python tools/k2_pmc_summary.py gpurun_out/k2pmc k_scores2 > gpurun_out/k2pmc/summary.txt 2>&1
