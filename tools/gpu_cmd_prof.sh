cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_run.sh "pytest_harness 200 python -u -m pytest tests/test_c_verifier_harness.py -m gpu -v --timeout 120 --timeout-method thread" || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profB -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/profB.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profE -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload E_4096x262144_fp32 --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/profE.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && timeout 100 python bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50 > gpurun_out/benchB.log 2>&1
cd $GRAFT_REPO_ROOT && timeout -k 10 200 python tools/ab_scores.py build_ab/libbk_base.so biscotti_amd/libbk.so > gpurun_out/ab_scores.log 2>&1
