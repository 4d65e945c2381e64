# K8 at four waves per SIMD (build_ab/libbk_k8w4.so) against the shipped library
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "base1 120 python tools/roni_ab.py" "w4_1 120 env LIB=build_ab/libbk_k8w4.so python tools/roni_ab.py" "base2 120 python tools/roni_ab.py" "w4_2 120 env LIB=build_ab/libbk_k8w4.so python tools/roni_ab.py"
