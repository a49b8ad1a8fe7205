#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first fault / abort / timeout.
# Usage: tools/gpu_session.sh "<label>::<timeout_s>::<command>" ...
# Exit statuses 0 and 1 (test failures) continue; anything else (134 abort, 139 segv,
# 124/137 timeout) ends the session so no further GPU work starts after a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  label="${spec%%::*}"; rest="${spec#*::}"; tmo="${rest%%::*}"; cmd="${rest#*::}"
  echo "=== [$label] (timeout ${tmo}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 15 "gpurun_out/$label.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $label ended with $rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
