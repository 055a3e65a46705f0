#!/bin/bash
# k_solo experiment library from another git revision's csrc (mte_solo.hip + headers), linked with
# this tree's other objects: bash tools/solo_variant_rev.sh <name> <rev> [extra hipcc flags...]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
V=$1; REV=$2; shift 2
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" fluidframework_amd/csrc include | tar -x -C "$T"
# the kernel parameter block must match this tree's host code
cp "$ROOT/fluidframework_amd/csrc/engine_types.hpp" "$T/fluidframework_amd/csrc/engine_types.hpp"
B="$ROOT/fluidframework_amd/_build"
make -s -C "$ROOT/fluidframework_amd/csrc" >/dev/null
mkdir -p "$B/$V"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable "$@" \
  -c "$T/fluidframework_amd/csrc/mte_solo.hip" -o "$B/$V/mte_solo.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$B/$V/libmte.so" "$B/mte_kernels.o" "$B/$V/mte_solo.o" "$B/emit.o" \
  "$B/mte_host.o" -lpthread
rm -rf "$T"
echo "$B/$V/libmte.so"
