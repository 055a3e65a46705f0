#!/bin/bash
# GPU box: the lone 10^6-op document with the heap-server wave (default), without it (option
# heap_server=0) and on the build before it (MTE_LIB=$1), interleaved twice -> gpurun_out/<tag>/.
set -o pipefail
T=${T:-hs}; BASE=${1:-r05h}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  v=$([ $rep = 1 ] && echo 1 || echo 0)
  for run in base srv nosrv; do
    case $run in
      base) env MTE_LIB=$BASE timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --reps 2 --verify $v > gpurun_out/$T/${run}_$rep.json 2> gpurun_out/$T/${run}_$rep.err ;;
      srv) timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --reps 2 --verify $v > gpurun_out/$T/${run}_$rep.json 2> gpurun_out/$T/${run}_$rep.err ;;
      nosrv) timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --reps 2 --verify $v --opt heap_server=0 > gpurun_out/$T/${run}_$rep.json 2> gpurun_out/$T/${run}_$rep.err ;;
    esac
    rc=$?; [ $rc -eq 0 ] || { echo "$run failed ($rc)"; tail -3 gpurun_out/$T/${run}_$rep.err; exit 1; }
    python -c "import json; a=json.load(open('gpurun_out/$T/${run}_$rep.json')); print('$run', round(a['us_per_op'],4), a.get('verified'), a['doc0']['status'], a['doc0']['mode'])"
  done
done
