#!/bin/bash
# GPU box: lone-document bisect of this round's row-engine changes, C4 with the solo gate (5 steps)
# and without, the per-scope cycle profile (tools/rg_prof_run.sh), and the FETCH/WRITE calibration
# incl. u16 reads. Fail-stop.
set -o pipefail
export TMPDIR=/tmp
T=rd bash tools/r04_ab.sh base v2 cur nsi ng2 nsn || exit 1
T=rd TO=400 EXTRA="--no-cpu-baseline --steps 5 --warmup 1" bash tools/r04_bench_ab.sh "C4:" "C4:solo_gate=0" || exit 1
bash tools/rg_prof_run.sh rpd || exit 1
mkdir -p gpurun_out/calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/fetch -o run --output-format csv -- ./tools/microbench/fetch_calib > gpurun_out/calib/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib/write -o run --output-format csv -- ./tools/microbench/fetch_calib > gpurun_out/calib/write.log 2>&1 || exit 1
echo round d done
