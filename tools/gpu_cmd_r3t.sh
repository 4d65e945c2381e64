cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_roni 300 python -u -m pytest tests/test_gpu_roni_softmax.py tests/test_gpu_roni.py -q -x --timeout 120 --timeout-method thread" "ab_mfma 120 python tools/roni_ab.py" "ab_valu 120 env BK_RONI_VALU=1 python tools/roni_ab.py" || exit $?
mkdir -p gpurun_out/prof_roni
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_roni/trace -o run --output-format csv -- python3 $R/tools/roni_ab.py > $R/gpurun_out/prof_roni/trace.log 2>&1
echo rc=$?
find $R/gpurun_out/prof_roni -name "*stats*" | head
