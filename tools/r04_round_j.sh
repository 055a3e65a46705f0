#!/bin/bash
# GPU box: the PROPS row engine on k_solo (GPU tests), the lone 10^6-op kind-3 document (mode 4, vs the
# oracle), and a lone-document A/B of the lean k_solo over this round's builds (base = round start,
# e = before the shared row pool, p = the pool commit, cur). Fail-stop.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rj
timeout -k 10 600 python -u -m pytest tests/test_gpu_reg.py -v --timeout 300 --timeout-method thread > gpurun_out/rj/tests.log 2>&1; rc=$?
grep -E "FAILED" gpurun_out/rj/tests.log | tail -20; tail -1 gpurun_out/rj/tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 400 python tools/lone_doc.py --kind 3 --ops 1000000 --reps 2 --verify 1 > gpurun_out/rj/lone1m_k3.json 2> gpurun_out/rj/lone1m_k3.err || { tail -5 gpurun_out/rj/lone1m_k3.err; exit 1; }
python -c "import json; a=json.load(open('gpurun_out/rj/lone1m_k3.json')); print('lone k3', a['us_per_op'], a.get('verified'), a['doc0']['mode'], a['doc0']['status'])"
T=rj bash tools/r04_ab.sh base e p cur || exit 1
echo round j done
