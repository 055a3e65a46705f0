#!/bin/bash
# Run one gpurun call, waiting out "no box / slot free" answers (nothing ran, nothing charged):
# tools/gpurun_wait.sh <log> <timeout_s> <command>. Any other outcome (success or failure) ends it.
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -qE "retry in a few minutes|being prepared; retry" "$LOG" && [ $rc -ne 0 ]; then sleep 90; continue; fi
  exit $rc
done
