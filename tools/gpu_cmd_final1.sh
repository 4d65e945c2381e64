# r3 final evidence, part 1: every GPU test, the smoke, the driver's bench command
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" "smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'" "bench 900 python bench.py"
