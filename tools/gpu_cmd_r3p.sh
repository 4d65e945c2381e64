cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "probe_order 60 ./tools/probe_mfma_order" "pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread"
