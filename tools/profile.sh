#!/bin/bash
# rocprofv3 passes over bench.py (kernel trace + stats, then one PMC counter
# group per pass -- never --pmc together with trace domains).
#   tools/profile.sh <tag> [bench args...]
# The trace pass runs bench.py with its default steps/warmup (the same command
# as the bench line, minus the CPU baseline), so the rocprof average of K1 over
# the timed window agrees with bench.py's HIP-event figure; the PMC passes use
# short runs (counters are per dispatch).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# --no-variants / --no-next-rows: only the workload's own dispatches (the
# summary picks K1 as the dispatches within 2x of the longest k_gram)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-graph-probe --no-variants --no-next-rows "$@" > "$OUT/trace.log" 2>&1 || exit $?
SHORT="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-graph-probe --no-variants --no-next-rows $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  # --kernel-trace beside --pmc (allowed; no other trace domains): each
  # dispatch's duration in the same pass gives the physical clock
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmc$i" -o run --output-format csv -- python3 $SHORT > "$OUT/pmc$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i ($grp) rc=$rc"; tail -3 "$OUT/pmc$i.log"; if [ $rc -ge 124 ]; then exit $rc; fi; fi
done
echo profile done
