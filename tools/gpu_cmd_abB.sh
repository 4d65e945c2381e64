cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "abB 300 env N=100 D=7850 F=30 REPS=40 python tools/ab_libs.py base=build_ab/libbk_base.so new=biscotti_amd/libbk.so base2=build_ab/libbk_base.so new2=biscotti_amd/libbk.so" "benchB 200 python bench.py --workload B_mnist --no-cpu-baseline --no-e2e --no-next-rows --no-graph-probe --steps 500 --warmup 50"
