#!/bin/bash
# GPU box: C4 bench lines at several HBM-wave shares (interference on the critical wave).
set -e
for hw in 0 4 8; do
  timeout -k 10 400 python bench.py --steps 4 --no-cpu-baseline --verify-docs 2 --opt hbm_waves_per_cu=$hw > gpurun_out/r03hw_$hw.json 2> gpurun_out/r03hw_$hw.err || { tail gpurun_out/r03hw_$hw.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/r03hw_$hw.json')); print('hw $hw', round(a['value']/1e6,2), a['extra']['kernel_ms_steps'])"
  grep warmup gpurun_out/r03hw_$hw.err
done
