#!/bin/bash
# GPU box, final build of the round: the full GPU suite, the lone-document A/B against the round-start
# build, the bench lines (C4 headline with cpu_baseline, then C2, C3, C5) and tools/profile.sh.
# Stops on a crash or time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rk
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rk/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rk/gpu_tests.log | tail -20; tail -1 gpurun_out/rk/gpu_tests.log
[ $rc -le 1 ] || exit 1
T=rk bash tools/r04_ab.sh base cur || exit 1
T=rk TO=600 bash tools/r04_bench_ab.sh "C4:" "C2:" "C3:" "C5:" || exit 1
bash tools/profile.sh r04k || exit 1
echo round k done
