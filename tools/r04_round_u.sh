#!/bin/bash
# GPU box: the longer bounded pool wait -- k_rows GPU tests and C2 twice (10 steps), watching for re-runs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ru
timeout -k 10 600 python -u -m pytest tests/test_gpu_reg.py -v --timeout 300 --timeout-method thread > gpurun_out/ru/tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/ru/tests.log | tail -20; tail -1 gpurun_out/ru/tests.log
[ $rc -le 1 ] || exit 1
T=ru EXTRA="--no-cpu-baseline --steps 10" bash tools/r04_bench_ab.sh "C2:" || exit 1
T=ru2 EXTRA="--steps 10" bash tools/r04_bench_ab.sh "C2:" || exit 1
python -c "
import json
for f in ['gpurun_out/ru/C2.json','gpurun_out/ru2/C2.json']:
    e=json.load(open(f))['extra']; print(f, 'steps', e['kernel_ms_steps'], 'reruns', e['docs_rerun_hbm'])"
echo round u done
