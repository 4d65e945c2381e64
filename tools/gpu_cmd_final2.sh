# r3 final evidence, part 2: rocprofv3 records (kernel trace + PMC passes) for D, C, B, A
cd $GRAFT_REPO_ROOT
bash tools/profile.sh D || exit $?
bash tools/profile.sh C --workload C_1024x131072 || exit $?
bash tools/profile.sh B --workload B_mnist --steps 500 --warmup 50 || exit $?
bash tools/profile.sh A --workload A_creditcard --steps 500 --warmup 50 || exit $?
echo part 2 done
