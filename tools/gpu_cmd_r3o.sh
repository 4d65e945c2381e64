cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" "idle_i200 120 python tools/idle_probe.py" "idle_i001 120 env IDLE=0.001 python tools/idle_probe.py"
