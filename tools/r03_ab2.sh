#!/bin/bash
# GPU box: sink-flag A/B on the critical path (lone 1M doc) and the C4 pass, then the GPU suite.
set -e
bash tools/ab_lone.sh cur nosink cur nosink
CFG=C4 REPS=2 bash tools/ab_cfg.sh main nosink
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r03s_tests.log 2>&1 || { tail -30 gpurun_out/r03s_tests.log; exit 1; }
tail -3 gpurun_out/r03s_tests.log
