#!/bin/bash
# GPU box: the PROPS row engine -- k_rows / property GPU tests, C3 on k_rows (auto) vs the LDS engine
# (rows_bulk 0), and the lone-document A/B (the lean k_solo build after the PROPS template change).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ri
timeout -k 10 600 python -u -m pytest tests/test_gpu_reg.py tests/test_gpu_props.py -v --timeout 300 --timeout-method thread > gpurun_out/ri/tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/ri/tests.log | tail -20; tail -1 gpurun_out/ri/tests.log
[ $rc -le 1 ] || exit 1
T=ri EXTRA="--no-cpu-baseline" bash tools/r04_bench_ab.sh "C3:" "C3:rows_bulk=0" "C3:rows_bulk=4" || exit 1
T=ri bash tools/r04_ab.sh base cur || exit 1
bash tools/profile.sh r04b || exit 1
echo round i done
