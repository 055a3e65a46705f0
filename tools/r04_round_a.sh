#!/bin/bash
# GPU box: lone-document A/B, the row-engine GPU tests (k_solo + k_rows) and the matrix spec pins, then
# C2 / C5 bench lines with and without k_rows. Stops at the first failing step.
set -o pipefail
T=ab6 bash tools/r04_ab.sh base cur omm opath || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_reg.py \
  tests/test_matrix_spec.py > gpurun_out/ab6/tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab6/tests.log
[ $rc -eq 0 ] || exit $rc
T=bab1 TO=300 bash tools/r04_bench_ab.sh "C2:" "C2:rows_bulk=4" "C2:rows_bulk=8" "C5:rows_bulk=4" "C5:"
