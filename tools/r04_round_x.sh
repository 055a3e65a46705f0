#!/bin/bash
# GPU box, final tree (12-wave k_rows default with the in-pass restart queue): the full GPU suite,
# smoke(), and the C2 / C3 lines at the default with cpu_baseline. Stops on a crash or time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rx
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rx/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rx/gpu_tests.log | tail -20; tail -1 gpurun_out/rx/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rx/smoke.log 2>&1 || { tail -5 gpurun_out/rx/smoke.log; exit 1; }
tail -1 gpurun_out/rx/smoke.log
T=rx TO=600 EXTRA="--steps 10" bash tools/r04_bench_ab.sh "C2:" || exit 1
T=rx TO=600 bash tools/r04_bench_ab.sh "C3:" || exit 1
echo round x done
