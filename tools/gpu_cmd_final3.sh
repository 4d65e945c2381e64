# r3 final evidence, part 3: E in its three f32 modes, and the RONI kernels
cd $GRAFT_REPO_ROOT
bash tools/profile.sh E --workload E_4096x262144_fp32 --steps 10 --warmup 3 || exit $?
bash tools/profile.sh Emfma --workload E_4096x262144_fp32 --f32-mode mfma --steps 10 --warmup 3 || exit $?
bash tools/profile.sh Ecert --workload E_4096x262144_fp32 --f32-mode certified --steps 10 --warmup 3 || exit $?
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_roni
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_roni/trace -o run --output-format csv -- python3 $R/tools/roni_ab.py > $R/gpurun_out/prof_roni/trace.log 2>&1 || exit $?
echo part 3 done
