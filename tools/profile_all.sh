#!/bin/bash
# rocprofv3 evidence for every BASELINE config on the current libbk.so: one
# tools/profile.sh run (kernel trace + stats of bench.py, then one --pmc pass
# per counter group) per config.  Summaries are made afterwards on the build
# host with tools/pmc_summary.py (it stamps the libbk.so hash bench.py checks):
#   tools/profile_all.sh [tag patterns...]    (on the GPU box, via gpurun; e.g. 'E_*')
#   then here, per tag: python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> \
#       profiles/r05/rocprof_<tag>_r05 <warmup> <steps>   (10 40; E: 5 10)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
# optional arguments: only the tags matching one of these shell patterns
ONLY=("$@")
run() {
  tag=$1; shift
  if [ ${#ONLY[@]} -gt 0 ]; then
    hit=0
    for p in "${ONLY[@]}"; do case "$tag" in $p) hit=1 ;; esac; done
    [ $hit = 1 ] || return 0
  fi
  echo "=== profile $tag: $*"
  "$R/tools/profile.sh" "$tag" "$@" || { echo "profile $tag failed rc=$?"; exit 1; }
}
run D_512x1M_f153
run D_512x1M_f153_i8_certified --f32-mode i8_certified
run D_512x1M_f153_i8x2_certified --f32-mode i8x2_certified
run C_1024x131072 --workload C_1024x131072
for m in exact mfma certified i8 i8_certified i8x2 i8x2_certified; do
  t=E_4096x262144_fp32; [ "$m" = exact ] || t="${t}_$m"
  run "$t" --workload E_4096x262144_fp32 --f32-mode "$m" --steps 10 --warmup 5
done
run B_mnist --workload B_mnist
run A_creditcard --workload A_creditcard
echo profile_all done
