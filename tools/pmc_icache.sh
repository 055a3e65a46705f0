#!/bin/bash
# Instruction-fetch counters over the lone-document replay (critical path), one small pass each.
# Usage (GPU box): bash tools/pmc_icache.sh <tag> [ops]
set -o pipefail
T=${1:-ic}; N=${2:-100000}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_$T
mkdir -p $OUT
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH" "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_REQ SQC_TC_INST_REQ"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 tools/lone_doc.py --ops $N --reps 1 --verify 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
for p in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "k_solo<false, 0>" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
print({k: v for k, v in sorted(tot.items())})
PY
