#!/bin/bash
# GPU box: the lone-wave latency microbench, then the default C4 bench line.
T=${1:-b}
mkdir -p gpurun_out
timeout -k 5 60 ./tools/microbench/chains > gpurun_out/${T}_chains.txt 2>&1; cat gpurun_out/${T}_chains.txt
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err || { tail -20 gpurun_out/${T}_bench_c4.err; exit 1; }
cat gpurun_out/${T}_bench_c4.json
