#!/bin/bash
# GPU box: cold-load split (4 reps), then the C2 and C3 bench lines (VERDICT r02 item 4 targets).
T=${1:-c23}
mkdir -p gpurun_out
timeout -k 10 300 python tools/pcie_rate.py --config C4 --reps 4 > gpurun_out/${T}_pcie.json 2> gpurun_out/${T}_pcie.err || { tail -5 gpurun_out/${T}_pcie.err; exit 1; }
cat gpurun_out/${T}_pcie.json
for C in C2 C3; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > gpurun_out/${T}_bench_${C}.json 2> gpurun_out/${T}_bench_${C}.err || { tail -20 gpurun_out/${T}_bench_${C}.err; exit 1; }
  cat gpurun_out/${T}_bench_${C}.json
done
