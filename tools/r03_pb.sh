#!/bin/bash
# GPU box: C4 bench with torch initialised up front (first-step check), HBM-priority A/B, cold loads, suite.
set -e
timeout -k 10 400 python bench.py --steps 4 > gpurun_out/r03pb_bench_c4.json 2> gpurun_out/r03pb_bench_c4.err || { tail gpurun_out/r03pb_bench_c4.err; exit 1; }
grep -o "\"value\": [0-9.]*\|\"kernel_ms_steps[^]]*]" gpurun_out/r03pb_bench_c4.json; grep warmup gpurun_out/r03pb_bench_c4.err
bash tools/r03_pa.sh
