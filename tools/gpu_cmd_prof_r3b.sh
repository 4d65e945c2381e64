# round-3 rocprofv3 records, part 2: E in its three f32 modes
cd $GRAFT_REPO_ROOT
bash tools/profile.sh E --workload E_4096x262144_fp32 --steps 10 --warmup 3 || exit $?
bash tools/profile.sh Emfma --workload E_4096x262144_fp32 --f32-mode mfma --steps 10 --warmup 3 || exit $?
bash tools/profile.sh Ecert --workload E_4096x262144_fp32 --f32-mode certified --steps 10 --warmup 3 || exit $?
echo part 2 done
