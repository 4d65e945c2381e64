# E's 8-rank shard on the fp32 MFMA under each K1 planner mode (the K1b slab count vs K1)
cd $GRAFT_REPO_ROOT
A="--workload E_4096x262144_fp32 --f32-mode mfma --emulate-ranks 8 --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --no-variants --steps 20 --warmup 5"
bash tools/gpu_run.sh "pm_def 300 python bench.py $A" "pm0 300 env BK_PLAN_MODE=0 python bench.py $A" "pm1 300 env BK_PLAN_MODE=1 python bench.py $A" "pm2 300 env BK_PLAN_MODE=2 python bench.py $A" "pm3 300 env BK_PLAN_MODE=3 python bench.py $A"
