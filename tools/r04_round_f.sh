#!/bin/bash
# GPU box: k_rows on the shared row pool (PAGED engine): its GPU parity tests, then C2 (kind 2 and
# kind 5) on the LDS engine vs k_rows at 4, 8 and 12 waves per CU. Fail-stop.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rf
timeout -k 10 600 python -u -m pytest tests/test_gpu_reg.py -x -v --timeout 300 --timeout-method thread > gpurun_out/rf/reg_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/rf/reg_tests.log | tail -20; tail -3 gpurun_out/rf/reg_tests.log; exit 1; }
tail -1 gpurun_out/rf/reg_tests.log
T=rf EXTRA="--no-cpu-baseline" bash tools/r04_bench_ab.sh "C2:" "C2:rows_bulk=8" "C2:rows_bulk=12" "C2:rows_bulk=4" || exit 1
T=rf5 EXTRA="--no-cpu-baseline --kind 5" bash tools/r04_bench_ab.sh "C2:rows_bulk=8" "C2:rows_bulk=12" || exit 1
echo round f done
