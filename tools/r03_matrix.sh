#!/bin/bash
# GPU box: the SharedMatrix tests (vectors + cell ops), then the C2 / C3 / cold-load measurements.
T=${1:-mx}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matrix.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_matrix.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/${T}_matrix.log | head -40
[ $rc -eq 0 ] || { tail -60 gpurun_out/${T}_matrix.log; exit $rc; }
bash tools/r03_c23.sh ${T}
