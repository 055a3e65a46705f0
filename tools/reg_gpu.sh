#!/bin/bash
# One GPU call for the row engine: its GPU tests, then lone-document latency (200k and 1M ops).
# Usage (GPU box): bash tools/reg_gpu.sh <tag> [extra pytest files]
T=${1:-r}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_reg.py "$@" > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${T}_tests.log | tail -30 | cut -c1-200
[ $rc -ne 0 ] && { tail -40 gpurun_out/${T}_tests.log; exit $rc; }
timeout -k 10 200 python tools/lone_doc.py --ops 200000 > gpurun_out/${T}_lone200k.json 2> gpurun_out/${T}_lone.err || { echo lone failed; tail gpurun_out/${T}_lone.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/${T}_lone200k.json')); print('200k us/op', round(a['us_per_op'],3), 'verified', a.get('verified'), 'mode', a['doc0']['mode'])"
timeout -k 10 300 python tools/lone_doc.py --ops 1000000 > gpurun_out/${T}_lone1m.json 2>> gpurun_out/${T}_lone.err || { echo lone1m failed; tail gpurun_out/${T}_lone.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/${T}_lone1m.json')); print('1M us/op', round(a['us_per_op'],3), 'verified', a.get('verified'), 'mode', a['doc0']['mode'], a['doc0'])"
