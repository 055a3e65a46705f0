#!/bin/bash
# GPU box: row-engine single-scope profiles, the new GPU tests, then the C4 bench.
bash tools/rg_prof_run.sh r03g
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py "tests/test_gpu_parity.py::test_hbm_slot_exhaustion_completes" > gpurun_out/r03g_new.log 2>&1
rc=$?
tail -6 gpurun_out/r03g_new.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r03g_bench_c4.json 2> gpurun_out/r03g_bench_c4.err || { tail gpurun_out/r03g_bench_c4.err; exit 1; }
grep -o "\"value\": [0-9.]*\|\"kernel_ms_steps.*solo_lead" gpurun_out/r03g_bench_c4.json
