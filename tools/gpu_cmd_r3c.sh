cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" "ubench 300 ./tools/ubench_fp64_data 2.5" "bench 900 python bench.py" "smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'"
