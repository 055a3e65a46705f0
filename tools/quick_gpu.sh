#!/bin/bash
# One GPU call for an engine change: lone-document latency (normal + phase-profile builds) and the
# GPU parity suite. Usage (GPU box): bash tools/quick_gpu.sh <tag> [ops]
set -o pipefail
T=${1:-q}; N=${2:-200000}
mkdir -p gpurun_out
timeout -k 10 200 python tools/lone_doc.py --ops $N > gpurun_out/${T}_lone.json 2> gpurun_out/${T}_lone.err || { echo lone failed; tail gpurun_out/${T}_lone.err; exit 1; }
MTE_LIB=prof timeout -k 10 200 python tools/lone_doc.py --ops $N --reps 1 --verify 0 > gpurun_out/${T}_prof.json 2>> gpurun_out/${T}_lone.err || { echo prof failed; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
python - "$T" <<'PY'
import json, sys
t = sys.argv[1]
a = json.load(open(f"gpurun_out/{t}_lone.json")); b = json.load(open(f"gpurun_out/{t}_prof.json"))
print("us_per_op", round(a["us_per_op"], 3), "verified", a.get("verified"), "mode", a["doc0"]["mode"])
print({k: v for k, v in b["cycles_per_op"].items()})
PY
tail -3 gpurun_out/${T}_tests.log
exit $rc
