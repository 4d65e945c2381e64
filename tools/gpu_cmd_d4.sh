cd $GRAFT_REPO_ROOT
L=biscotti_amd/libbk.so
B=build_ab/libbk_d4off.so
bash tools/gpu_run.sh "d4D 300 env REPS=10 python tools/ab_libs.py off=$B on=$L off2=$B on2=$L" "d4D8 200 env REPS=20 D=131072 python tools/ab_libs.py off=$B on=$L off2=$B on2=$L" "d4C 300 env REPS=10 N=1024 D=131072 python tools/ab_libs.py off=$B on=$L off2=$B on2=$L" "pytest_par 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_margin.py tests/test_gpu_f32mfma.py tests/test_gpu_group.py tests/test_gpu_two_process.py -m gpu -q -x --timeout 200 --timeout-method thread"
