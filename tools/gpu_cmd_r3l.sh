cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "idle_poll 120 python tools/idle_probe.py" "idle_block0 120 env BK_SPIN_US=0 python tools/idle_probe.py" "idle_sched 120 env BK_SPIN_US=0 BK_SCHED=1 python tools/idle_probe.py" "idle_poll2 120 python tools/idle_probe.py" "idle_block02 120 env BK_SPIN_US=0 python tools/idle_probe.py"
