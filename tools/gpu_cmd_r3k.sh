cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "zc 120 ./tools/ubench_zc" "pytest_small 300 python -u -m pytest tests/test_gpu_small.py -m gpu -q -x --timeout 120 --timeout-method thread -k host_entry"
bash tools/profile.sh A --workload A_creditcard --steps 500 --warmup 50 || exit $?
bash tools/gpu_run.sh "bench 900 python bench.py"
