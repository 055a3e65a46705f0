#!/bin/bash
# Run GPU steps in order, stopping at a fault / abort / segfault / time limit (124, 134, 137, 139) but
# not at a test failure (pytest 1). Usage: bash tools/gpu_chain.sh "cmd1" "cmd2" ...
for c in "$@"; do
  bash -c "$c"
  rc=$?
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc: $c"; exit $rc;; esac
done
