#!/bin/bash
# GPU box: GPU suite, lone 1M-op document, phase profile, C4 bench.
T=${1:-h}
bash tools/reg_iter.sh $T || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err || { tail gpurun_out/${T}_bench_c4.err; exit 1; }
grep -o "\"value\": [0-9.]*\|\"kernel_ms_steps.*solo_lead" gpurun_out/${T}_bench_c4.json
