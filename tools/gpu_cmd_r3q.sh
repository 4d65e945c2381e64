cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_roni 300 python -u -m pytest tests/test_gpu_roni_softmax.py tests/test_gpu_roni.py -q -x --timeout 120 --timeout-method thread" "ab_mfma 120 python tools/roni_ab.py" "ab_valu 120 env BK_RONI_VALU=1 python tools/roni_ab.py" "ab_mfma2 120 python tools/roni_ab.py"
