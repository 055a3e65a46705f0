#!/bin/bash
# GPU box, final tree: the default bench line (C4 with cpu_baseline) and C5. Fail-stop.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rs
timeout -k 10 600 python bench.py > gpurun_out/rs/C4.json 2> gpurun_out/rs/C4.err || { tail -5 gpurun_out/rs/C4.err; exit 1; }
cat gpurun_out/rs/C4.json
T=rs TO=600 bash tools/r04_bench_ab.sh "C5:" || exit 1
echo round s done
