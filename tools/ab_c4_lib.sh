#!/bin/bash
# GPU box: C4 bench lines alternating between two library builds (MTE_LIB names, "cur" = default)
# with per-build engine options, interleaved REPS times, into gpurun_out/<tag>/.
# Usage: T=<tag> bash tools/ab_c4_lib.sh "cur:solo_xcd_quiet=1" "prev:"
set -o pipefail
T=${T:-abl}; mkdir -p gpurun_out/$T
for rep in $(seq 1 ${REPS:-2}); do
for spec in "$@"; do
  lib=${spec%%:*}; opts=${spec#*:}; v=$lib; [ "$lib" = cur ] && v=""
  args=""; for o in ${opts//,/ }; do args="$args --opt $o"; done
  name="${lib}_${opts//[=,]/}_$rep"
  MTE_LIB=$v timeout -k 10 ${TO:-400} python bench.py --config ${CFG:-C4} --no-cpu-baseline $args > gpurun_out/$T/$name.json 2> gpurun_out/$T/$name.err || { echo "$name failed"; tail -5 gpurun_out/$T/$name.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/$T/$name.json')); print('$name', round(a['ms_per_step'],1), a['extra']['kernel_ms_steps'], a['extra'].get('us_per_op_critical_path'))"
done
done
