cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread"
