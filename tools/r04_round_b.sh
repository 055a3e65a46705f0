#!/bin/bash
# GPU box: the new GPU tests (k_rows, matrix spec pins, marker-heavy re-run, full-size C4 and C2), then
# bench lines with and without k_rows. Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out/rb
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_reg.py \
  tests/test_matrix_spec.py tests/test_relative_pos.py tests/test_gpu_fullsize.py tests/test_gpu_c4.py \
  > gpurun_out/rb/tests.log 2>&1; rc=$?
tail -4 gpurun_out/rb/tests.log
[ $rc -eq 0 ] || exit $rc
T=rb TO=300 EXTRA="--no-cpu-baseline" bash tools/r04_bench_ab.sh "C2:" "C2:rows_bulk=4" "C2:rows_bulk=8" "C5:rows_bulk=4" "C4:" "C4:rows_bulk=4"
