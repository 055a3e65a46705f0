#!/bin/bash
# GPU box, final tree (32-bit op numbers in the row engine's replay loop): the full GPU suite, smoke(),
# the lone-document A/B against the round-start build and the default bench line (C4 with cpu_baseline),
# then C2 / C3 / C5. Stops on a crash or time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rt2
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/rt2/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rt2/gpu_tests.log | tail -20; tail -1 gpurun_out/rt2/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rt2/smoke.log 2>&1 || { tail -5 gpurun_out/rt2/smoke.log; exit 1; }
tail -1 gpurun_out/rt2/smoke.log
T=rt2 bash tools/r04_ab.sh base cur || exit 1
timeout -k 10 600 python bench.py > gpurun_out/rt2/C4.json 2> gpurun_out/rt2/C4.err || { tail -5 gpurun_out/rt2/C4.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/rt2/C4.json')); print('C4', round(a['ms_per_step'],1), round(a['value']/1e6,2), a['extra']['kernel_ms_steps'])"
T=rt2 TO=600 bash tools/r04_bench_ab.sh "C2:" "C3:" "C5:" || exit 1
echo round t done
