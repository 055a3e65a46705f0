#!/bin/bash
# Available rocprofv3 counters on the box (GPU box), filtered to the instruction-fetch / cache ones.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_all.txt 2>&1
grep -iE "SQC|IFETCH|ICACHE|INST_CACHE|WAIT_INST" gpurun_out/counters_all.txt | head -80
