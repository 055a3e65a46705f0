#!/bin/bash
# GPU box, final tree (12-wave k_rows default): the full GPU suite, smoke(), the C2 / C3 bench lines with
# cpu_baseline and their rocprof summaries + FETCH/WRITE passes. Stops on a crash or time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rr
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rr/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rr/gpu_tests.log | tail -20; tail -1 gpurun_out/rr/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rr/smoke.log 2>&1 || { tail -5 gpurun_out/rr/smoke.log; exit 1; }
tail -1 gpurun_out/rr/smoke.log
T=rr TO=600 bash tools/r04_bench_ab.sh "C2:" "C3:" || exit 1
bash tools/profile.sh r04c2 --config C2 --steps 2 --warmup 0 --no-cpu-baseline --verify-docs 2 || exit 1
bash tools/profile.sh r04c3 --config C3 --steps 2 --warmup 0 --no-cpu-baseline --verify-docs 2 || exit 1
echo round r done
