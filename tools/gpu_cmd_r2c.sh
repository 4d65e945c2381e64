cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_nan 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k nan_and_inf --timeout 120 --timeout-method thread" "ab_scores 200 python tools/ab_scores.py build_ab/libbk_base.so biscotti_amd/libbk.so" "k2modes 300 python tools/k2_modes.py" || exit $?
bash tools/gpu_cmd_k2pmc.sh
