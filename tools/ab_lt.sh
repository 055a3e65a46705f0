#!/bin/bash
# GPU box: lone 1M-op document with LDS text on / off (reg_lt_limit=1), the previous build, and C4.
for o in "" "--opt reg_lt_limit=1"; do
  timeout -k 10 200 python tools/lone_doc.py --ops 1000000 $o > gpurun_out/ab3.json 2>/dev/null || { echo "lone [$o] failed"; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/ab3.json')); print('lone [$o]', round(a['us_per_op'],3), a['verified'], a['doc0']['n_gc'])"
done
MTE_LIB=prev timeout -k 10 200 python tools/lone_doc.py --ops 1000000 --verify 0 > gpurun_out/ab3p.json 2>/dev/null
python -c "import json; a=json.load(open('gpurun_out/ab3p.json')); print('lone prev', round(a['us_per_op'],3))"
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --verify-docs 0 > gpurun_out/ab3_c4.json 2>/dev/null
grep -o "\"kernel_ms_steps[^]]*]" gpurun_out/ab3_c4.json
