#!/bin/bash
# rocprofv3 record of SURVEY §8(f) row 4's kernels (tools/roni_probe.py): one
# kernel-trace + stats pass, then one --pmc pass per counter group (never with
# other trace domains).  Summarised by tools/roni_pmc_summary.py.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/prof_roni"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/tools/roni_probe.py" 20 > "$OUT/trace.log" 2>&1 || exit $?
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmc$i" -o run --output-format csv -- python3 "$R/tools/roni_probe.py" 5 > "$OUT/pmc$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i ($grp) rc=$rc"; tail -3 "$OUT/pmc$i.log"; if [ $rc -ge 124 ]; then exit $rc; fi; fi
done
echo profile_roni done
