cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "benchDv 300 python bench.py --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 10 --warmup 3" "benchA 200 python bench.py --workload A_creditcard --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50"
