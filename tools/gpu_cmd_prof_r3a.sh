# round-3 rocprofv3 records, part 1: D (headline), C, B
cd $GRAFT_REPO_ROOT
bash tools/profile.sh D || exit $?
bash tools/profile.sh C --workload C_1024x131072 || exit $?
bash tools/profile.sh B --workload B_mnist --steps 500 --warmup 50 || exit $?
echo part 1 done
