// Kernel launchers (mte_kernels.hip) used by the host side (mte_host.cpp). full: the engine level
// (0 lean, 1 FULL, 2 FULL + EXT; engine.hpp).
#pragma once
#include <hip/hip_runtime.h>

#include "engine_types.hpp"

namespace mte {
hipError_t launch_lds(const Params& p, bool gen, int full, u32 n_groups, hipStream_t s);
hipError_t launch_solo(const Params& p, bool gen, int full, u32 n_solo, bool ck, hipStream_t s);
// wait (one wave, <= 20 ms) until `n_solo` solo workgroups have started: issued on the bulk's stream
hipError_t launch_solo_gate(const u32* started, u32 n_solo, hipStream_t s);
// lean replays: the bulk (doc_list[n_prio ..)) on the row engine, waves_per_cu 4 or 8 per CU
hipError_t launch_rows(const Params& p, u32 waves_per_cu, u32 n_groups, bool props, bool wide, bool ck, hipStream_t s);
hipError_t launch_hbmq(const Params& p, bool gen, int full, u32 n_waves, hipStream_t s);
hipError_t launch_rows_cont(const Params& p, bool props, bool wide, u32 n_slots, hipStream_t s);
extern const u64 ROWS_DUMP_BYTES;  // a slot must hold k_rows' state dump (mte_solo.hip RowsDump)
hipError_t launch_hbm(const Params& p, bool gen, int full, u32 n_docs, hipStream_t s);
hipError_t launch_wave_selftest(const u32* in, u32* out, u32 n_waves, hipStream_t s);
}  // namespace mte
