#!/bin/bash
# GPU box: bench.py lines for (config, option) pairs, one JSON line each into gpurun_out/<tag>/.
# Usage: T=<tag> bash tools/bench_ab.sh "C2:" "C2:rows_bulk=4" "C5:rows_bulk=4" ...
#   (config:opt[,opt...]; an empty opt list = the default engine options)
set -o pipefail
T=${T:-bab}
mkdir -p gpurun_out/$T
for spec in "$@"; do
  cfg=${spec%%:*}; opts=${spec#*:}
  args=""; name=$cfg
  if [ -n "$opts" ]; then
    for o in ${opts//,/ }; do args="$args --opt $o"; name="${name}_${o//=/}"; done
  fi
  timeout -k 10 ${TO:-600} python bench.py --config $cfg $args ${EXTRA:-} > gpurun_out/$T/$name.json 2> gpurun_out/$T/$name.err || { echo "$name failed"; tail -5 gpurun_out/$T/$name.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/$T/$name.json')); x=a['extra']; print('$name', round(a['ms_per_step'],1), 'ms/step', round(a['value']/1e6,1), 'Mops/s', 'steps', x['kernel_ms_steps'], 'cpu', (a.get('cpu_baseline') or {}).get('value'))"
done
