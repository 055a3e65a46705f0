#!/bin/bash
# A/B of engine variants on the critical-path workload (GPU box): for each name, the lone-document
# replay time of _build/<name>/libmte.so ("main" = the default build). Usage: bash tools/ab.sh main v1 v2 ...
N=${N:-100000}
mkdir -p gpurun_out/ab
for v in "$@"; do
  lib=$v; [ "$v" = main ] && lib=""
  MTE_LIB=$lib timeout -k 10 120 python tools/lone_doc.py --ops $N --reps 3 --verify ${VERIFY:-0} ${OPTS:-} > gpurun_out/ab/$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json,sys; a=json.load(open('gpurun_out/ab/$v.json')); print('$v', [round(a[f'kernel_ms_{i}']*1e3/a['ops'],3) for i in range(3)], 'us/op', a.get('verified'))"
done
