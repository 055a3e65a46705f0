#!/bin/bash
# rocprofv3 evidence for the replay kernel (run on the GPU box from the repo root):
#   1) kernel trace + stats of a short bench run
#   2) separate PMC passes for FETCH_SIZE and WRITE_SIZE (counters never combined with tracing)
# Usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
ARGS=${@:---steps 2 --warmup 0 --no-cpu-baseline --verify-docs 2}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc_write.log" 2>&1
echo "profile $TAG done"
