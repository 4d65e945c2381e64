cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" "smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'" "bench 900 python bench.py"
