#!/bin/bash
# Undistorted phase costs of the lone critical-path wave: one build per phase, each timing only that
# phase (engine.hpp MTE_PROF_ONLY). Usage (GPU box): bash tools/phase_only.sh [ops] po_total po_apply ...
N=${1:-100000}; shift
mkdir -p gpurun_out/po
for v in "$@"; do
  MTE_LIB=$v timeout -k 10 120 python tools/lone_doc.py --ops $N --reps 1 --verify 0 > gpurun_out/po/$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/po/$v.json')); c={k:v for k,v in a['cycles_per_op'].items() if v and not k.startswith('n_')}; print('$v', round(a['us_per_op'],3), c)"
done
