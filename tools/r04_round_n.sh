#!/bin/bash
# GPU box: rocprofv3 kernel trace + stats and FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh) for the
# row-engine configs C2, C3 and C5, so their bench lines carry calibrated traffic. Fail-stop.
set -o pipefail
export TMPDIR=/tmp
bash tools/profile.sh r04c2 --config C2 --steps 2 --warmup 0 --no-cpu-baseline --verify-docs 2 || exit 1
bash tools/profile.sh r04c3 --config C3 --steps 2 --warmup 0 --no-cpu-baseline --verify-docs 2 || exit 1
bash tools/profile.sh r04c5 --config C5 --steps 2 --warmup 0 --no-cpu-baseline --verify-docs 2 || exit 1
echo round n done
