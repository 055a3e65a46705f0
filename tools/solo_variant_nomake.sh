#!/bin/bash
# Like solo_variant.sh but without rebuilding the default library first (safe while a GPU call that
# snapshots the tree is pending): bash tools/solo_variant_nomake.sh <name> [extra hipcc flags...]
set -e
cd "$(dirname "$0")/../fluidframework_amd/csrc"
B=../_build
V=$1; shift
mkdir -p $B/$V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable "$@" \
  -c mte_solo.hip -o $B/$V/mte_solo.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/$V/libmte.so $B/mte_kernels.o $B/$V/mte_solo.o $B/emit.o \
  $B/mte_host.o -lpthread
echo "$B/$V/libmte.so"
