cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "ab_scores 200 python tools/ab_scores.py build_ab/libbk_base.so biscotti_amd/libbk.so" "ab_scores_kpt4 200 env BK_K2_KPT=4 python tools/ab_scores.py build_ab/libbk_base.so biscotti_amd/libbk.so" "k2modes 300 python tools/k2_modes.py" "pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread"
