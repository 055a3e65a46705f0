#!/bin/bash
# One GPU call per row-engine change: the GPU parity suite, the lone 1M-op critical-path document
# (checked against the oracle) and the phase profile of a 200k-op lone document.
# Usage (GPU box): bash tools/reg_iter.sh <tag>
T=${1:-i}
mkdir -p gpurun_out
bash tools/gpu_suite.sh ${T} || exit 1
timeout -k 10 300 python tools/lone_doc.py --ops 1000000 > gpurun_out/${T}_lone1m.json 2> gpurun_out/${T}_lone.err || { echo lone1m failed; tail gpurun_out/${T}_lone.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/${T}_lone1m.json')); print('1M us/op', round(a['us_per_op'],3), 'verified', a.get('verified'), 'mode', a['doc0']['mode'])"
MTE_LIB=prof timeout -k 10 200 python tools/lone_doc.py --ops 200000 --reps 1 --verify 0 > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || { echo prof failed; tail gpurun_out/${T}_prof.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/${T}_prof.json')); print(round(a['us_per_op'],3), {k:v for k,v in a['cycles_per_op'].items() if v})"
