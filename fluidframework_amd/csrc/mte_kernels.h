// Host-callable launchers for the replay engine kernels (mte_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "engine_types.hpp"

namespace mte {
hipError_t launch_replay(const Params& p, u32 n_blocks, hipStream_t s);
hipError_t launch_generate(const Params& p, u32 n_blocks, hipStream_t s);
hipError_t launch_wave_selftest(const u32* in, u32* out, u32 n_waves, hipStream_t s);
}  // namespace mte
