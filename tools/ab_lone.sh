#!/bin/bash
# GPU box: the lone 1M-op document on several library variants (MTE_LIB names; "cur" = default build).
for lib in "$@"; do
  v=$lib; [ "$lib" = cur ] && v=""
  MTE_LIB=$v timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --verify 0 > gpurun_out/abl_$lib.json 2>/dev/null || { echo "$lib failed"; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/abl_$lib.json')); print('$lib', round(a['us_per_op'],3))"
done
