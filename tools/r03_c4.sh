#!/bin/bash
# GPU box: default C4 bench line (+ LDS / HBM kernel times of the last step), then the GPU suite.
set -e
T=${1:-c4}
timeout -k 10 400 python bench.py --steps 4 > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err || { tail gpurun_out/${T}_bench_c4.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/${T}_bench_c4.json')); x=a['extra']; print(round(a['value']/1e6,2), x['kernel_ms_steps'], x['lds_ms_last_step'], x['hbm_wave_slots'])"
grep warmup gpurun_out/${T}_bench_c4.err
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
