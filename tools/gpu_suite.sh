#!/bin/bash
# GPU parity suite in one process (GPU box), log under gpurun_out/<tag>_tests.log.
T=${1:-s}; shift
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "$@" > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/${T}_tests.log | tail -60 | cut -c1-150
tail -3 gpurun_out/${T}_tests.log
exit $rc
