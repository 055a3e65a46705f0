#!/bin/bash
# GPU box: lone-document A/B (round-3 build vs this tree), C4 with and without the XCD-aligned bulk
# grid (5 steps each), the row-engine / matrix / relative-position / C4 GPU tests. Fail-stop.
set -o pipefail
mkdir -p gpurun_out/rc
T=rc bash tools/r04_ab.sh base cur || exit 1
T=rc TO=400 EXTRA="--no-cpu-baseline --steps 5 --warmup 1" bash tools/r04_bench_ab.sh "C4:" "C4:xcd_align=0" || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_reg.py \
  tests/test_matrix_spec.py tests/test_matrix.py tests/test_relative_pos.py tests/test_gpu_c4.py \
  > gpurun_out/rc/tests.log 2>&1; rc=$?
tail -3 gpurun_out/rc/tests.log
exit $rc
