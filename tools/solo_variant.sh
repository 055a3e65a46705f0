#!/bin/bash
# Build a k_solo-only experiment library: mte_solo.hip with extra flags, linked with the default
# build's other objects. Usage: bash tools/solo_variant.sh <name> [extra hipcc flags...]
#   -> fluidframework_amd/_build/<name>/libmte.so  (select on the GPU box with MTE_LIB=<name>)
set -e
cd "$(dirname "$0")/../fluidframework_amd/csrc"
B=../_build
V=$1; shift
make -s -C . >/dev/null
mkdir -p $B/$V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable ${SOLOFLAGS--mllvm -amdgpu-sched-strategy=iterative-ilp} "$@" \
  -c mte_solo.hip -o $B/$V/mte_solo.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/$V/libmte.so $B/mte_kernels.o $B/$V/mte_solo.o $B/emit.o \
  $B/mte_host.o -lpthread
echo "$B/$V/libmte.so"
