# r3 closing check on the final tree: every GPU test and the smoke
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" "smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'"
