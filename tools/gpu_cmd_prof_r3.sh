# round-3 rocprofv3 records (kernel trace + stats, then one PMC group per pass)
# for every driver-timed line: D (headline), C, E in its three modes, B.
cd $GRAFT_REPO_ROOT
bash tools/profile.sh D || exit $?
bash tools/profile.sh C --workload C_1024x131072 || exit $?
bash tools/profile.sh B --workload B_mnist --steps 500 --warmup 50 || exit $?
bash tools/profile.sh E --workload E_4096x262144_fp32 --steps 10 --warmup 3 || exit $?
bash tools/profile.sh Emfma --workload E_4096x262144_fp32 --f32-mode mfma --steps 10 --warmup 3 || exit $?
bash tools/profile.sh Ecert --workload E_4096x262144_fp32 --f32-mode certified --steps 10 --warmup 3 || exit $?
echo all profiles done
