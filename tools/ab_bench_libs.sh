#!/bin/bash
# GPU box: bench.py lines of library variants (MTE_LIB names, "cur" = the default build) on one box,
# interleaved: T=<tag> bash tools/ab_bench_libs.sh "<configs>" <lib>...  -> gpurun_out/<tag>/<cfg>_<lib>.json
set -o pipefail
T=${T:-abl}
CFGS=$1; shift
mkdir -p gpurun_out/$T
for lib in "$@"; do
  for cfg in $CFGS; do
    v=$lib; [ "$lib" = cur ] && v=""
    MTE_LIB=$v timeout -k 10 ${TO:-600} python bench.py --config $cfg --no-cpu-baseline > gpurun_out/$T/${cfg}_$lib.json 2> gpurun_out/$T/${cfg}_$lib.err || { echo "$cfg $lib failed"; tail -3 gpurun_out/$T/${cfg}_$lib.err; exit 1; }
    python -c "import json; a=json.load(open('gpurun_out/$T/${cfg}_$lib.json')); print('$cfg', '$lib', round(a['ms_per_step'],1), 'ms/step', a['extra']['kernel_ms_steps'])"
  done
done
