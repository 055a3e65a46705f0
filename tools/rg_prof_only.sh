#!/bin/bash
# Build one profiling library per row-engine scope (reg_engine.hpp RG_PROF_ONLY): each times only its
# own scope, so no scope pays for the s_memtime pairs of the scopes inside it.
# Usage (here, after `make prof`): bash tools/rg_prof_only.sh   -> fluidframework_amd/_build/rp_<name>/libmte.so
set -e
cd "$(dirname "$0")/../fluidframework_amd/csrc"
B=../_build
declare -A S=([apply]=2 [resolve]=3 [insert_slot]=4 [split]=5 [range]=6 [zamboni]=7 [scour]=8 [heap]=9 \
              [find_seg]=10 [pack]=11 [lru]=12 [split_at]=21 [op_ins]=22 [op_rem]=23 [zam_msn]=24 [zam_edit]=25)
build() {
  mkdir -p $B/rp_$1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable \
    -mllvm -amdgpu-sched-strategy=iterative-ilp -DMTE_PROFILE -DRG_PROF_ONLY=$2 -c mte_solo.hip -o $B/rp_$1/mte_solo.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/rp_$1/libmte.so $B/prof/mte_kernels.o $B/rp_$1/mte_solo.o $B/emit.o \
    $B/prof/mte_host.o -lpthread
}
n=0
for k in "${!S[@]}"; do
  build $k ${S[$k]} &
  n=$((n+1)); if [ $((n % 4)) -eq 0 ]; then wait; fi
done
wait
ls $B | grep rp_ | tr '\n' ' '; echo
