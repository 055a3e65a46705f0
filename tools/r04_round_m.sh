#!/bin/bash
# GPU box: the full GPU suite, smoke() and a short C4 bench on the final tree. Stops on a crash or
# time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rm
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rm/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rm/gpu_tests.log | tail -20; tail -1 gpurun_out/rm/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rm/smoke.log 2>&1 || { tail -5 gpurun_out/rm/smoke.log; exit 1; }
tail -1 gpurun_out/rm/smoke.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rm/c4.json 2> gpurun_out/rm/c4.err || { tail -5 gpurun_out/rm/c4.err; exit 1; }
cat gpurun_out/rm/c4.json
echo round m done
