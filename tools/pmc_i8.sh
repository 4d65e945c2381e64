#!/bin/bash
# PMC passes over K1i8 alone (tools/ab_i8.py on one build; config E by default,
# DT=f64 for the headline batch): one rocprofv3 --pmc pass per counter group,
# --kernel-trace beside it only (never other trace domains).
#   tools/pmc_i8.sh <tag> [lib]
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1
LIB=${2:-$R/biscotti_amd/libbk.so}
OUT="$R/gpurun_out/pmci8_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export REPS=${REPS:-1} ROUNDS=${ROUNDS:-1}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmc$i" -o run --output-format csv -- python3 "$R/tools/ab_i8.py" "x=$LIB" > "$OUT/pmc$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i ($grp) rc=$rc"; tail -3 "$OUT/pmc$i.log"; exit $rc; fi
done
echo pmc_i8 done
