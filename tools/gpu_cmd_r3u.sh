cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "t8 120 python tools/roni_ab.py" "t2 120 env BK_RONI_TILES=2 python tools/roni_ab.py" "t4 120 env BK_RONI_TILES=4 python tools/roni_ab.py" "t16 120 env BK_RONI_TILES=16 python tools/roni_ab.py" "t8b 120 python tools/roni_ab.py"
