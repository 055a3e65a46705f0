#!/bin/bash
# GPU box: HBM-wave priority A/B on C2 / C3, cold-load reps, GPU suite.
set -e
bash tools/r03_ab.sh main p1 p2 main p1 p2
timeout -k 10 300 python tools/pcie_rate.py --config C4 --reps 3 > gpurun_out/r03pa_pcie.json 2> gpurun_out/r03pa_pcie.err || { tail -5 gpurun_out/r03pa_pcie.err; exit 1; }
python -c "
import json; a=json.load(open('gpurun_out/r03pa_pcie.json'))
for r in a['reps']: print({k:r[k] for k in ('load_ms','h2d_ms','alloc_ms','stage_copy_ms','stage_wait_ms')})"
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r03pa_tests.log 2>&1 || { tail -30 gpurun_out/r03pa_tests.log; exit 1; }
tail -2 gpurun_out/r03pa_tests.log
