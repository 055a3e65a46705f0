#!/bin/bash
# GPU box: C2 / C3 bench lines and the GPU suite on the current build.
set -e
T=${1:-h}
for C in C2 C3; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > gpurun_out/${T}_bench_${C}.json 2> gpurun_out/${T}_bench_${C}.err || { tail -20 gpurun_out/${T}_bench_${C}.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/${T}_bench_${C}.json')); print('$C', a['ms_per_step'], a['extra']['kernel_ms_steps'], a['extra']['docs_continued_hbm'])"
done
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
