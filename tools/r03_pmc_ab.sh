#!/bin/bash
# GPU box: SQ / I-cache counters of the lone critical-path wave for two builds, and the FETCH_SIZE /
# WRITE_SIZE calibration microbench.
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/f -o run --output-format csv -- ./tools/microbench/fetch_calib > gpurun_out/calib/f.log 2>&1 || { echo calib f failed; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib/w -o run --output-format csv -- ./tools/microbench/fetch_calib > gpurun_out/calib/w.log 2>&1 || { echo calib w failed; exit 1; }
echo calib ok
for lib in prev cur; do
  v=$lib; [ "$lib" = cur ] && v=""
  MTE_LIB=$v bash tools/pmc_icache.sh ic_$lib 200000 || exit 1
  MTE_LIB=$v bash tools/pmc_lone.sh pl_$lib 200000 || exit 1
done
