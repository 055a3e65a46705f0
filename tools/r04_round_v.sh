#!/bin/bash
# GPU box, final tree (k_rows auto: 12 waves with properties, 8 lean): the full GPU suite, smoke() and
# the C2 line at the default. Stops on a crash or time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rv
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rv/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rv/gpu_tests.log | tail -20; tail -1 gpurun_out/rv/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rv/smoke.log 2>&1 || { tail -5 gpurun_out/rv/smoke.log; exit 1; }
tail -1 gpurun_out/rv/smoke.log
T=rv TO=600 bash tools/r04_bench_ab.sh "C2:" || exit 1
echo round v done
