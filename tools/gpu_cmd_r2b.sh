cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "trace_small 120 env BK_SMALL_TRACE=gpurun_out/small.bin python tools/trace_small.py run" "ab_scores 200 python tools/ab_scores.py build_ab/libbk_base.so biscotti_amd/libbk.so" "k2modes 300 python tools/k2_modes.py" "pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread"
