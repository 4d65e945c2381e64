# K1 timing-only ablations on the final library: normal / no MFMA / no global loads (D and C)
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "ablD 300 python tools/ablate_gram.py" "ablC 300 env N=1024 D=131072 python tools/ablate_gram.py"
