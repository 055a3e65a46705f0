// HIP kernels of the replay engine (gfx950). One 64-lane workgroup == one wavefront == one document.
#include "wave_hip.hpp"
#include "engine_core.hpp"
#include "mte_kernels.h"

namespace mte {

__global__ __launch_bounds__(64) void k_replay(Params p) {
    __shared__ u32 scratch[32];
    u32 d = p.doc_order ? p.doc_order[blockIdx.x] : blockIdx.x;
    Engine e(p, d);
    e.replay(scratch);
}

__global__ __launch_bounds__(64) void k_generate(Params p) {
    __shared__ u32 scratch[32];
    u32 d = p.doc_order ? p.doc_order[blockIdx.x] : blockIdx.x;
    Engine e(p, d);
    e.generate(scratch);
}

// Self-test of the DPP prefix scan and the ballot/shuffle primitives (used by the GPU unit tests).
__global__ __launch_bounds__(64) void k_wave_selftest(const u32* in, u32* out) {
    u32 L = lane_id();
    u32 v = in[blockIdx.x * 64 + L];
    out[blockIdx.x * 64 * 3 + L] = wave_scan_incl(v);
    out[blockIdx.x * 64 * 3 + 64 + L] = wave_shfl(v, 63 - L);
    u64 b = wave_ballot((v & 1u) != 0);
    out[blockIdx.x * 64 * 3 + 128 + L] = (u32)(L < 32 ? b : (b >> 32));
}

hipError_t launch_replay(const Params& p, u32 n_blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_replay, dim3(n_blocks), dim3(64), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_generate(const Params& p, u32 n_blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_generate, dim3(n_blocks), dim3(64), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_wave_selftest(const u32* in, u32* out, u32 n_waves, hipStream_t s) {
    hipLaunchKernelGGL(k_wave_selftest, dim3(n_waves), dim3(64), 0, s, in, out);
    return hipGetLastError();
}

}  // namespace mte
