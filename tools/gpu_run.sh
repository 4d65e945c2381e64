#!/bin/bash
# One GPU session: run steps in order, each under its own time limit; stop at
# the first step that crashed / timed out (exit >= 2 and not a plain test
# failure).  Usage: tools/gpu_run.sh "<label> <timeout_s> <cmd...>" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  label=${spec%% *}; rest=${spec#* }; to=${rest%% *}; cmd=${rest#* }
  echo "=== [$label] (timeout ${to}s) $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] exit $rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$label.log"
  # pytest steps may fail (rc 1) and the session goes on; any other step that
  # fails (a Python exception after a GPU fault is rc 1 too) ends the session
  case "$label" in
    pytest*) if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: step $label rc=$rc"; exit $rc; fi ;;
    *) if [ $rc -ne 0 ]; then echo "stopping: step $label rc=$rc"; exit $rc; fi ;;
  esac
done
