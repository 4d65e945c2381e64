cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_roni
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_roni/trace -o run --output-format csv -- python3 $R/tools/roni_ab.py > $R/gpurun_out/prof_roni/trace.log 2>&1
echo rc=$?
find $R/gpurun_out/prof_roni -name "*stats*" | head
