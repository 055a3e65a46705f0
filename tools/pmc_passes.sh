#!/bin/bash
# SQ counter passes over one replay (tools/replay_once.py), one rocprofv3 run per pass.
# Usage (GPU box, repo root): tools/pmc_passes.sh <outdir> [replay_once args]
set -uo pipefail
OUT=${1:-gpurun_out/pmc}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_IFETCH" \
            "SQ_INST_CYCLES_SALU SQ_INSTS_VSKIPPED SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS -d "$OUT/p$i" -o run --output-format csv -- python3 tools/replay_once.py "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
