// Wave64 primitives for gfx950 (CDNA4). One wavefront replays one document; these are the only
// cross-lane operations the engine uses (engine.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MTE_DEV __device__ __forceinline__

namespace mte {

MTE_DEV uint32_t lane_id() { return __lane_id(); }

// Full barrier for cross-lane GLOBAL-memory hand-offs inside a wave: every lane's earlier
// global/LDS writes are complete and visible to every lane's later reads.
MTE_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// Cross-lane LDS hand-off inside a wave: LDS instructions of one wavefront execute in order, so
// only compiler reordering has to be prevented (no s_waitcnt, no cache maintenance).
MTE_DEV void lds_order() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
}

MTE_DEV uint64_t wave_ballot(bool p) { return __ballot(p); }

MTE_DEV uint32_t wave_shfl(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
MTE_DEV int32_t wave_shfl(int32_t v, uint32_t src) { return (int32_t)wave_shfl((uint32_t)v, src); }
MTE_DEV uint64_t wave_shfl(uint64_t v, uint32_t src) {
    uint32_t lo = wave_shfl((uint32_t)v, src), hi = wave_shfl((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// Uniform broadcast from a known lane (v_readlane -> SGPR).
MTE_DEV uint32_t wave_read(uint32_t v, uint32_t src) { return __builtin_amdgcn_readlane(v, src); }
MTE_DEV int32_t wave_read(int32_t v, uint32_t src) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)v, src); }
MTE_DEV uint32_t wave_first(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
MTE_DEV int32_t wave_first(int32_t v) { return (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)v); }

// Inclusive prefix sum over the 64 lanes with DPP: row_shr:1,2,4,8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 to carry across rows (GFX9-family DPP controls, present on gfx950).
MTE_DEV uint32_t wave_scan_incl(uint32_t v) {
    uint32_t x = v, t;
    // update_dpp(old, src, dpp_ctrl, row_mask, bank_mask, bound_ctrl): lanes with no source keep `old`
    t = __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false); x += t;  // row_shr:1
    t = __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false); x += t;  // row_shr:2
    t = __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false); x += t;  // row_shr:4
    t = __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false); x += t;  // row_shr:8
    t = __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false); x += t;  // row_bcast:15 -> rows 1,3
    t = __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false); x += t;  // row_bcast:31 -> rows 2,3
    return x;
}

MTE_DEV uint32_t wave_sum(uint32_t v) { return wave_read(wave_scan_incl(v), 63); }

// Inclusive prefix sum inside each aligned group of 8 lanes (one leaf block per group).
MTE_DEV uint32_t group8_scan(uint32_t v) {
    const uint32_t g = lane_id() & 7;
    uint32_t x = v, t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false); if (g >= 1) x += t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false); if (g >= 2) x += t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false); if (g >= 4) x += t;
    return x;
}
// Inclusive prefix max (signed) inside each aligned group of 8 lanes.
MTE_DEV int32_t group8_max(int32_t v) {
    const uint32_t g = lane_id() & 7;
    int32_t x = v, t;
    t = (int32_t)__builtin_amdgcn_update_dpp(0u, (uint32_t)x, 0x111, 0xf, 0xf, false); if (g >= 1 && t > x) x = t;
    t = (int32_t)__builtin_amdgcn_update_dpp(0u, (uint32_t)x, 0x112, 0xf, 0xf, false); if (g >= 2 && t > x) x = t;
    t = (int32_t)__builtin_amdgcn_update_dpp(0u, (uint32_t)x, 0x114, 0xf, 0xf, false); if (g >= 4 && t > x) x = t;
    return x;
}

MTE_DEV uint32_t atomic_add_u32(uint32_t* p, uint32_t v) { return atomicAdd(p, v); }

}  // namespace mte
