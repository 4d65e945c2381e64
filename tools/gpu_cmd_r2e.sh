cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread" "benchD8 200 python bench.py --emulate-ranks 8 --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 40 --warmup 10" "benchB 200 python bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50"
