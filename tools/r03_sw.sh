#!/bin/bash
# GPU box: HBM-wave share sweeps on C2 / C3 shapes, then a kernel trace of the C2 bench.
T=${1:-sw}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/sweep.py --kind 2 --ops 10000 --docs 4096 --modes lds --hw 0,4,8,12,16 > gpurun_out/${T}_c2.jsonl 2> gpurun_out/${T}_c2.err || { tail -5 gpurun_out/${T}_c2.err; exit 1; }
cut -c1-400 gpurun_out/${T}_c2.jsonl
timeout -k 10 300 python tools/sweep.py --kind 3 --ops 10000 --docs 65536 --modes lds --hw 0,4,12 > gpurun_out/${T}_c3.jsonl 2> gpurun_out/${T}_c3.err || { tail -5 gpurun_out/${T}_c3.err; exit 1; }
cut -c1-400 gpurun_out/${T}_c3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --verify-docs 2 > gpurun_out/${T}_trace.log 2>&1 || { tail -5 gpurun_out/${T}_trace.log; exit 1; }
find gpurun_out/${T}_trace -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
