cd $GRAFT_REPO_ROOT
P="python tools/k1_probe.py"
bash tools/gpu_run.sh "p_base 120 $P base" "p_w16 120 env LIB=build_ab/libbk_l2w16.so $P w16" "p_m1r1 120 env BK_PLAN_MODE=1 BK_PLAN_ROUNDS=1 $P m1r1" "p_m1r2 120 env BK_PLAN_MODE=1 BK_PLAN_ROUNDS=2 $P m1r2" "p_m1r4 120 env BK_PLAN_MODE=1 BK_PLAN_ROUNDS=4 $P m1r4" "p_m1r8 120 env BK_PLAN_MODE=1 BK_PLAN_ROUNDS=8 $P m1r8" "p_m1r16 120 env BK_PLAN_MODE=1 BK_PLAN_ROUNDS=16 $P m1r16" "p_m2r4 120 env BK_PLAN_MODE=2 BK_PLAN_ROUNDS=4 $P m2r4" "p_base2 120 $P base2" "p_w64 120 env LIB=build_ab/libbk_l2w64.so $P w64"
