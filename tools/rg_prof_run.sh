#!/bin/bash
# GPU box: each single-scope profiling library (tools/rg_prof_only.sh) on the lone 200k-op document.
T=${1:-po}
mkdir -p gpurun_out/$T
for d in fluidframework_amd/_build/rp_*/; do
  v=$(basename $d); n=${v#rp_}
  MTE_LIB=$v timeout -k 10 120 python tools/lone_doc.py --ops 200000 --reps 1 --verify 0 > gpurun_out/$T/$n.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/$T/$n.json')); c=a['cycles_per_op']; print('$n', round(a['us_per_op'],3), c.get('$n'))"
done
