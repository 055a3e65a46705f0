#!/bin/bash
# A/B of engine builds on a bench config (GPU box): replay_once per _build/<name>/libmte.so
# ("main" = default build). Usage: CFG=C2 bash tools/ab_cfg.sh main v1 v2 ...
CFG=${CFG:-C2}
mkdir -p gpurun_out/abc
for v in "$@"; do
  lib=$v; [ "$v" = main ] && lib=""
  MTE_LIB=$lib timeout -k 10 300 python tools/replay_once.py --config $CFG --replays ${REPS:-3} ${OPTS:-} > gpurun_out/abc/${CFG}_$v.json 2> gpurun_out/abc/${CFG}_$v.err || { echo "$v failed"; tail -3 gpurun_out/abc/${CFG}_$v.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/abc/${CFG}_$v.json')); print('$CFG $v', a['kernel_ms_all'], 'failed', a['failed_docs'], 'hbm_docs', a['hbm_docs'], 'cont', a['continued'])"
done
