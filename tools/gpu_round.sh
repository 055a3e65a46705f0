#!/bin/bash
# GPU box: one round of measurements, steps chosen on the command line, results under gpurun_out/<tag>/.
# Stops at the first step that crashes or hits its time limit (no GPU step runs after a failure).
# Usage: bash tools/gpu_round.sh <tag> <step>...
#   suite[:<-k expr>]     the -m gpu parity suite in one process   -> <tag>/gpu_tests.log
#   smoke                 __graft_entry__.smoke()                  -> <tag>/smoke.log
#   lone:<lib>[,<lib>..]  lone 10^6-op document A/B over MTE_LIB variants ("cur" = default build)
#   bench:<spec>[;<spec>] bench.py lines, spec = config:opt[,opt] (tools/bench_ab.sh)
#   profile               rocprofv3 kernel trace + FETCH/WRITE passes of the default bench (tools/profile.sh)
#   pmclone:<ops>:<lib>[,<lib>..]  SQ counter passes of the lone document per library (tools/pmc_lone_ab.sh)
set -o pipefail
T=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
for step in "$@"; do
  case "$step" in
    suite*)
      k=${step#suite}; k=${k#:}  # suite:<pytest -k expression>
      timeout -k 10 ${SUITE_TO:-900} python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread ${k:+-k "$k"} \
        > gpurun_out/$T/gpu_tests.log 2>&1; rc=$?
      grep -E "FAILED|ERROR" gpurun_out/$T/gpu_tests.log | tail -20; tail -1 gpurun_out/$T/gpu_tests.log
      [ $rc -le 1 ] || exit 1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 \
        || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
      tail -1 gpurun_out/$T/smoke.log ;;
    lone:*)
      libs=${step#lone:}
      T=$T bash tools/lone_ab.sh ${libs//,/ } || exit 1 ;;
    bench:*)
      specs=${step#bench:}
      IFS=';' read -ra S <<< "$specs"
      T=$T TO=${BENCH_TO:-600} bash tools/bench_ab.sh "${S[@]}" || exit 1 ;;
    profile)
      bash tools/profile.sh $T || exit 1 ;;
    pmclone:*)
      x=${step#pmclone:}; n=${x%%:*}; libs=${x#*:}
      bash tools/pmc_lone_ab.sh $T/pmc $n ${libs//,/ } || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "round $T done"
