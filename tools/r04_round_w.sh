#!/bin/bash
# GPU box: the k_rows restart queue -- k_rows GPU tests, C2 at 12 waves twice (10 steps each, watching for
# host re-runs) and C3 at the default. Fail-stop.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rw
timeout -k 10 600 python -u -m pytest tests/test_gpu_reg.py -v --timeout 300 --timeout-method thread > gpurun_out/rw/tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rw/tests.log | tail -20; tail -1 gpurun_out/rw/tests.log
[ $rc -le 1 ] || exit 1
T=rw EXTRA="--no-cpu-baseline --steps 10" bash tools/r04_bench_ab.sh "C2:rows_bulk=12" || exit 1
T=rw2 EXTRA="--steps 10" bash tools/r04_bench_ab.sh "C2:rows_bulk=12" || exit 1
T=rw EXTRA="--no-cpu-baseline" bash tools/r04_bench_ab.sh "C3:" || exit 1
python -c "
import json
for f in ['gpurun_out/rw/C2_rows_bulk12.json','gpurun_out/rw2/C2_rows_bulk12.json','gpurun_out/rw/C3.json']:
    e=json.load(open(f))['extra']; print(f, 'steps', e['kernel_ms_steps'], 'reruns', e['docs_rerun_hbm'])"
echo round w done
