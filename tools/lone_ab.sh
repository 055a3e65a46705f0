#!/bin/bash
# GPU box: lone 1M-op document A/B over library variants (MTE_LIB names, "cur" = default build),
# interleaved twice; then the GPU row-engine parity tests on the default build.
set -o pipefail
T=${T:-ab}
mkdir -p gpurun_out/$T
for rep in 1 2; do
for lib in "$@"; do
  v=$lib; [ "$lib" = cur ] && v=""
  MTE_LIB=$v timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --reps 2 --verify $([ $rep = 1 ] && echo 1 || echo 0) > gpurun_out/$T/${lib}_$rep.json 2>gpurun_out/$T/${lib}_$rep.err || { echo "$lib failed"; tail -3 gpurun_out/$T/${lib}_$rep.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/$T/${lib}_$rep.json')); print('$lib', round(a['us_per_op'],4), a.get('verified'), a['doc0']['status'], a['doc0']['mode'])"
done
done
