#!/bin/bash
# GPU box: full GPU parity suite on the default build (255-entry LDS heap, split_insert removed),
# lone-document A/B against the round-start build, and C2 shapes on the LDS engine vs k_rows at
# 4 and 8 waves per CU (kind 2, and kind 5 whose documents fit 8 waves' rows). Fail-stop.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/re
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/re/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/re/gpu_tests.log | tail -20; tail -2 gpurun_out/re/gpu_tests.log
[ $rc -le 1 ] || exit 1  # a crash or time limit (not a failed assertion) ends the call
T=re bash tools/r04_ab.sh base cur || exit 1
T=re EXTRA="--no-cpu-baseline" bash tools/r04_bench_ab.sh "C2:" "C2:rows_bulk=4" || exit 1
T=re5 EXTRA="--no-cpu-baseline --kind 5" bash tools/r04_bench_ab.sh "C2:" "C2:rows_bulk=4" "C2:rows_bulk=8" || exit 1
echo round e done
