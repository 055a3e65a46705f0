#!/bin/bash
# SQ counter passes over the lone-document replay (critical path), one pass per counter set.
# Usage (GPU box): bash tools/pmc_lone.sh <tag> [ops]
set -o pipefail
T=${1:-l}; N=${2:-100000}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_$T
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 tools/lone_doc.py --ops $N --reps 1 --verify 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
