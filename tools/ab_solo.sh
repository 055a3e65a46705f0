#!/bin/bash
# GPU box: A/B of library variants on the lone 1M-op document and the C4 pass.
# Usage: bash tools/ab_solo.sh <variant>... ("" = the default build)
for v in "$@"; do
  [ "$v" = "default" ] && v=""
  MTE_LIB=$v timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --verify 0 > gpurun_out/ab_lone_$v.json 2>/dev/null || { echo "lone $v failed"; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/ab_lone_$v.json')); print('lone [$v]', round(a['us_per_op'],3), a['doc0']['mode'])"
done
for v in "$@"; do
  [ "$v" = "default" ] && v=""
  MTE_LIB=$v timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --verify-docs 0 > gpurun_out/ab_c4_$v.json 2>/dev/null || { echo "c4 $v failed"; exit 1; }
  echo "c4 [$v]" $(grep -o "\"kernel_ms_steps[^]]*]" gpurun_out/ab_c4_$v.json)
done
