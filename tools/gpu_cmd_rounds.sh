cd $GRAFT_REPO_ROOT
L=biscotti_amd/libbk.so
bash tools/gpu_run.sh "rdD 300 env REPS=10 python tools/ab_libs.py def=$L r1=$L,BK_PLAN_ROUNDS=1 r2=$L,BK_PLAN_ROUNDS=2 r4=$L,BK_PLAN_ROUNDS=4 m1=$L,BK_PLAN_MODE=1 def2=$L" "rdC 300 env REPS=10 N=1024 D=131072 python tools/ab_libs.py def=$L r1=$L,BK_PLAN_ROUNDS=1 r2=$L,BK_PLAN_ROUNDS=2 r4=$L,BK_PLAN_ROUNDS=4 m1=$L,BK_PLAN_MODE=1 def2=$L"
