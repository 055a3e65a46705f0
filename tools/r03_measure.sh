#!/bin/bash
# One GPU call: the whole GPU parity suite, then the default C4 bench line and a rocprofv3 kernel
# trace of a short C4 run. Usage (GPU box): bash tools/r03_measure.sh <tag>
T=${1:-m}
mkdir -p gpurun_out
bash tools/gpu_suite.sh ${T} || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err || { tail -20 gpurun_out/${T}_bench_c4.err; exit 1; }
cat gpurun_out/${T}_bench_c4.json
export TMPDIR=/tmp; mkdir -p gpurun_out/prof_${T}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}/trace -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --verify-docs 2 > gpurun_out/prof_${T}/trace.log 2>&1 || { echo trace failed; exit 1; }

MTE_LIB=prof timeout -k 10 200 python tools/lone_doc.py --ops 200000 --reps 1 --verify 0 > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || { echo prof failed; tail gpurun_out/${T}_prof.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/${T}_prof.json')); print(a['us_per_op'], {k:v for k,v in a['cycles_per_op'].items() if v})"
echo measure ${T} done
