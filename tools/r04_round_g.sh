#!/bin/bash
# GPU box: full GPU parity suite (k_rows auto-routing for lean batches without solo documents), then
# the C2 and C5 bench lines at default options with cpu_baseline. Stops on a crash or time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rg
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rg/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rg/gpu_tests.log | tail -20; tail -1 gpurun_out/rg/gpu_tests.log
[ $rc -le 1 ] || exit 1
T=rg bash tools/r04_bench_ab.sh "C2:" "C5:" || exit 1
echo round g done
