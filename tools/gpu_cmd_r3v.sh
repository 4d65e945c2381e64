# A's host entry with the zero-copy k_tiny read, against the copy (BK_TINY_ZERO_COPY=0)
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "pytest_tiny 300 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_small.py tests/test_c_verifier_harness.py -q -x --timeout 120 --timeout-method thread" "hostA_zc 300 env WL=A_creditcard python tools/host_entry_ab.py zero_copy" "hostA_copy 300 env WL=A_creditcard BK_TINY_ZERO_COPY=0 python tools/host_entry_ab.py copy" "hostA_zc2 300 env WL=A_creditcard python tools/host_entry_ab.py zero_copy"
