#!/bin/bash
# GPU box: the round's measurement set at default options -- C4 (headline), C2, C3, C5 bench lines with
# cpu_baseline; the lone 10^6-op critical-path document; tools/profile.sh (C4 kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes). Fail-stop.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rh
timeout -k 10 300 python tools/lone_doc.py --ops 1000000 --reps 3 --verify 1 > gpurun_out/rh/lone1m.json 2> gpurun_out/rh/lone1m.err || { tail -5 gpurun_out/rh/lone1m.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/rh/lone1m.json')); print('lone', a['us_per_op'], a.get('verified'))"
T=rh TO=600 bash tools/r04_bench_ab.sh "C4:" "C2:" "C5:" "C3:" || exit 1
bash tools/profile.sh r04 || exit 1
echo round h done
