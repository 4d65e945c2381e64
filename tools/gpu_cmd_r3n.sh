cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "idle_i200 120 python tools/idle_probe.py" "idle_i020 120 env IDLE=0.02 python tools/idle_probe.py" "idle_i005 120 env IDLE=0.005 python tools/idle_probe.py" "idle_i001 120 env IDLE=0.001 python tools/idle_probe.py"
