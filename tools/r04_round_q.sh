#!/bin/bash
# GPU box: k_rows without the spare row per wave and a longer pool wait: the k_rows GPU
# tests, then C2 at 8 and 12 waves per CU (kind 2 and kind 5) and C3 at 8 (auto). Fail-stop.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rq
timeout -k 10 600 python -u -m pytest tests/test_gpu_reg.py -v --timeout 300 --timeout-method thread > gpurun_out/rq/tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rq/tests.log | tail -20; tail -1 gpurun_out/rq/tests.log
[ $rc -le 1 ] || exit 1
T=rq EXTRA="--no-cpu-baseline" bash tools/r04_bench_ab.sh "C2:rows_bulk=12" "C2:" "C3:rows_bulk=12" || exit 1
T=rq5 EXTRA="--no-cpu-baseline --kind 5" bash tools/r04_bench_ab.sh "C2:" "C2:rows_bulk=12" || exit 1
echo round q done
