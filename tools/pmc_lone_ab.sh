#!/bin/bash
# GPU box: SQ / SQC counter passes of the lone-document replay (k_solo<false, 0>) for each library
# variant (MTE_LIB names, "cur" = default build); prints per-op counts.
# Usage: bash tools/pmc_lone_ab.sh <tag> <ops> lib...
set -o pipefail
export TMPDIR=/tmp
T=$1; N=$2; shift 2
for lib in "$@"; do
  v=$lib; [ "$lib" = cur ] && v=""
  OUT=$PWD/gpurun_out/$T/$lib
  mkdir -p $OUT
  i=0
  for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_IFETCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    MTE_LIB=$v timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 tools/lone_doc.py --ops $N --reps 1 --verify 0 > $OUT/p$i.log 2>&1 || { echo "$lib pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  python3 - "$OUT" "$N" "$lib" <<'PY'
import csv, glob, sys, collections
out, n, lib = sys.argv[1], int(sys.argv[2]), sys.argv[3]
tot = collections.defaultdict(float)
for p in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "k_solo<false, 0" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
print(lib, {k: round(v / n, 2) for k, v in sorted(tot.items())}, flush=True)
PY
done
