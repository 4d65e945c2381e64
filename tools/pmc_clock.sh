#!/bin/bash
# One rocprofv3 --pmc pass (MFMA busy + GRBM_GUI_ACTIVE, --kernel-trace beside
# it only) over K1i8 alone (tools/ab_i8.py) per build: the shader clock each
# build's Gram runs at (GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's duration).
#   tools/pmc_clock.sh <tag> <lib>...      (MODE / DT as for ab_i8.py)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
export REPS=${REPS:-3} ROUNDS=${ROUNDS:-1}
for LIB in "$@"; do
  case "$LIB" in /*) ;; *) LIB="$R/$LIB" ;; esac
  b=$(basename "$LIB" .so)
  OUT="$R/gpurun_out/pmcclk_${TAG}_$b"
  mkdir -p "$OUT"
  timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d "$OUT/pmc1" -o run --output-format csv -- python3 "$R/tools/ab_i8.py" "x=$LIB" > "$OUT/pmc1.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc $b rc=$rc"; tail -3 "$OUT/pmc1.log"; exit $rc; fi
done
echo pmc_clock done
