#!/bin/bash
# GPU box: the round's evidence on the current build -- GPU suite, lone 1M-op critical path, default
# C4 bench line, rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of a C4 replay, PCIe-inclusive
# (cold + warm) C4 load.
T=${1:-f}
mkdir -p gpurun_out
bash tools/gpu_suite.sh ${T} || exit 1
timeout -k 10 300 python tools/lone_doc.py --ops 1000000 > gpurun_out/${T}_lone1m.json 2> gpurun_out/${T}_lone.err || { echo lone failed; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/${T}_lone1m.json')); print('1M us/op', round(a['us_per_op'],3), 'verified', a.get('verified'))"
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err || { tail gpurun_out/${T}_bench_c4.err; exit 1; }
grep -o "\"value\": [0-9.]*\|\"kernel_ms_steps[^]]*]" gpurun_out/${T}_bench_c4.json
bash tools/profile.sh ${T} --steps 1 --warmup 0 --no-cpu-baseline --verify-docs 0 || exit 1
timeout -k 10 300 python tools/pcie_rate.py --config C4 --reps 2 > gpurun_out/${T}_pcie_c4.json 2> gpurun_out/${T}_pcie.err || { tail gpurun_out/${T}_pcie.err; exit 1; }
echo final ${T} done
