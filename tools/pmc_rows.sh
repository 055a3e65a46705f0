#!/bin/bash
# GPU box: SQ counters of k_rows on C2 (8 waves per CU, the shared row pool) in two --pmc passes of one
# bench step each (counters never combined with tracing). Fail-stop. Parse: python tools/pmc_rows.py
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_rows
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 bench.py --config C2 --steps 1 --warmup 0 --no-cpu-baseline --verify-docs 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo pmc rows done
