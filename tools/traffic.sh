#!/bin/bash
# HBM write-traffic attribution for one replay pass of a bench config (GPU box): the pass's output
# sizes (rows, text units) from run_info, then counter passes per kernel: FETCH_SIZE, WRITE_SIZE and
# the vector-memory instruction counts (stores to HBM slots / outputs vs scratch spills).
# Usage: bash tools/traffic.sh <tag> <config>
set -o pipefail
T=${1:-t}; C=${2:-C4}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/traffic_$T
mkdir -p $OUT
timeout -k 10 200 python3 tools/replay_once.py --config $C > $OUT/run.json 2> $OUT/run.err || { echo run failed; exit 1; }
i=0
for P in "WRITE_SIZE" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 tools/replay_once.py --config $C > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo traffic done
