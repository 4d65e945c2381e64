cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread" "benchD 300 python bench.py" "benchB 200 python bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50" "benchE8 200 python bench.py --workload E_4096x262144_fp32 --emulate-ranks 8 --no-cpu-baseline --no-e2e --steps 10 --warmup 3" || exit $?
bash tools/profile.sh D
