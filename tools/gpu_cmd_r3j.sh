cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'" "bench 900 python bench.py"
