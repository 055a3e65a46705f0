#!/bin/bash
# PC sampling of the lone critical wave (rocprofv3, beta): where the replay's cycles go, per
# instruction. Usage (GPU box): bash tools/pcsample.sh <tag> <method> <unit> <interval> [ops]
set -o pipefail
T=${1:?tag}; M=${2:-host_trap}; U=${3:-time}; I=${4:-1}; N=${5:-100000}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pcs_$T
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
  --pc-sampling-interval $I -d $OUT/run -o pcs --output-format csv -- python3 tools/lone_doc.py --ops $N --reps 1 --verify 0 \
  > $OUT/run.log 2>&1; rc=$?
tail -5 $OUT/run.log
find $OUT -name '*.csv' | head
exit $rc
