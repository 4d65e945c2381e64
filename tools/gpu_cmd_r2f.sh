cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread" "benchD 300 python bench.py" "benchB 200 python bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50" "smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
bash tools/profile.sh D || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profB -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50 > $GRAFT_REPO_ROOT/gpurun_out/profB.log 2>&1
