#!/bin/bash
# GPU box: the full GPU suite and smoke() on the final tree (WIDE row engine on k_solo's FULL
# instantiation). Stops on a crash or time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rl
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rl/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rl/gpu_tests.log | tail -20; tail -1 gpurun_out/rl/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rl/smoke.log 2>&1 || { tail -5 gpurun_out/rl/smoke.log; exit 1; }
tail -1 gpurun_out/rl/smoke.log
echo round l done
