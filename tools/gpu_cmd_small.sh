cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_small 240 python -u -m pytest tests/test_gpu_small.py -m gpu -x -q --timeout 120 --timeout-method thread" "benchB 200 python bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50"
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profB2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/profB2.log 2>&1
