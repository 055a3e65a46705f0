#!/bin/bash
# GPU box: the lone 10^6-op document on k_solo (default) and on k_rows at 4 waves per CU (option
# solo_max=0: the row engine alone in its kernel, fixed 20-row quarters), interleaved twice.
set -o pipefail
T=${T:-lr}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  v=$([ $rep = 1 ] && echo 1 || echo 0)
  for run in solo rows4; do
    o=""; [ $run = rows4 ] && o="--opt solo_max=0 --opt rows_bulk=4"
    timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --reps 2 --verify $v $o > gpurun_out/$T/${run}_$rep.json 2> gpurun_out/$T/${run}_$rep.err || { echo "$run failed"; tail -3 gpurun_out/$T/${run}_$rep.err; exit 1; }
    python -c "import json; a=json.load(open('gpurun_out/$T/${run}_$rep.json')); print('$run', round(a['us_per_op'],4), a.get('verified'), a['doc0']['status'], a['doc0']['mode'])"
  done
done
