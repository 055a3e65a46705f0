#!/bin/bash
# GPU box: PC sampling of the lone 200k-op replay (critical-path wave), stochastic then host-trap.
# Usage: bash tools/r04_pcsamp.sh <tag> [ops] [lib]
set -o pipefail
export TMPDIR=/tmp
T=${1:-pcs}; N=${2:-200000}; LIB=${3:-}
OUT=$PWD/gpurun_out/$T
mkdir -p $OUT
for M in stochastic host_trap; do
  if [ $M = stochastic ]; then U=cycles; I=65536; else U=time; I=10; fi
  MTE_LIB=$LIB timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
    --pc-sampling-interval $I -d $OUT/$M -o run --output-format csv -- python3 tools/lone_doc.py --ops $N --reps 1 --verify 0 \
    > $OUT/$M.log 2>&1 && { echo "$M ok"; break; } || { echo "$M failed"; tail -5 $OUT/$M.log; }
done
find $OUT -name "*.csv" | head
