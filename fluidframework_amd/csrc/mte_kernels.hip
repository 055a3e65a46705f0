// HIP kernels of the replay engine (gfx950).
//
//   k_lds<GEN>: ONE workgroup per CU, LDS_WAVES waves, all 160 KiB of LDS (engine_types.hpp LdsPlan).
//               Waves pull documents from a queue in LPT order (longest first) and replay
//               (or generate) each with the whole per-document state resident in LDS. A document
//               that outgrows the plan is marked DOC_SPILL and its blocks go back to the CU's pool.
//   k_hbm<GEN>: one wave per listed document, state resident in HBM (DocCfg::hb_*): the host's
//               second pass for spilled documents.
#include "wave_hip.hpp"
#include "engine.hpp"
#include "mte_kernels.h"

namespace mte {

template <bool GEN>
__global__ __launch_bounds__(64 * LDS_WAVES) void k_lds(Params p) {
    LdsPlan* lp = &g_plan;
    const u32 t = threadIdx.x, L = t & 63;
    const u32 w = wave_first(t >> 6);  // wave-uniform (the compiler cannot infer it from threadIdx)
    u32 usable = POOL_BLOCKS;
    if (p.pool_limit && p.pool_limit < usable) usable = p.pool_limit;
    if (t < 16) {
        const u32 lo = t * 32;
        u32 word = 0;
        for (u32 b = 0; b < 32; b++)
            if (lo + b >= usable) word |= 1u << b;
        lp->bitmap[t] = word;
    }
    for (u32 b = t; b < POOL_BLOCKS; b += 64 * LDS_WAVES) lp->owner[b] = 0xFF;
    if (t == 0) lp->pool_avail = usable;
    __syncthreads();
    for (;;) {
        u32 i = 0;
        if (L == 0) i = atomicAdd(&p.counters[0], 1u);
        i = wave_read(i, 0);
        if (i >= p.n_list) break;
        const u32 d = p.doc_list[i];
        Engine<true> e(p, d);
        e.bind_lds(w);
        GenState g;
        bool done;
        u64 at = 0;
        e.init();
        if (GEN) {
            e.gen_init(g);
            done = e.generate_run(g);
        } else {
            at = e.replay_run(p.docs[d].op_begin);
            done = at >= p.docs[d].op_end;
        }
        if (e.st.status == DOC_SPILL) {
            e.mark_spilled();  // failed mid-op: the host re-runs it (rare)
        } else if (!done && e.st.status == 0) {
            // the LDS plan ran out of room between two ops: continue HBM-resident, same wave
            Engine<false> h(p, d);
            h.continued = true;
            if (h.bind_spill()) {
                h.adopt(e);
                e.release();
                if (L == 0) atomicAdd(&p.counters[4], 1u);
                if (GEN) {
                    h.generate_run(g);
                } else {
                    h.replay_run(at);
                }
                h.finish();
            } else {
                e.mark_spilled();
            }
        } else {
            e.finish();
        }
        e.release();
    }
}

template <bool GEN>
__global__ __launch_bounds__(64) void k_hbm(Params p) {
    const u32 d = p.doc_list[blockIdx.x];
    Engine<false> e(p, d);
    e.bind_hbm();
    e.init();
    if (GEN) {
        GenState g;
        e.gen_init(g);
        e.generate_run(g);
    } else {
        e.replay_run(p.docs[d].op_begin);
    }
    e.finish();
}

// Self-test of the DPP prefix scans and the ballot/shuffle primitives (used by the GPU unit tests).
__global__ __launch_bounds__(64) void k_wave_selftest(const u32* in, u32* out) {
    const u32 L = lane_id();
    const u32 v = in[blockIdx.x * 64 + L];
    u32* o = out + blockIdx.x * 64 * 5;
    o[L] = wave_scan_incl(v);
    o[64 + L] = wave_shfl(v, 63 - L);
    const u64 b = wave_ballot((v & 1u) != 0);
    o[128 + L] = (u32)(L < 32 ? b : (b >> 32));
    o[192 + L] = group8_scan(v);
    o[256 + L] = (u32)group8_max((i32)v);
}

hipError_t launch_lds(const Params& p, bool gen, u32 n_groups, hipStream_t s) {
    if (gen) hipLaunchKernelGGL(k_lds<true>, dim3(n_groups), dim3(64 * LDS_WAVES), 0, s, p);
    else hipLaunchKernelGGL(k_lds<false>, dim3(n_groups), dim3(64 * LDS_WAVES), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_hbm(const Params& p, bool gen, u32 n_docs, hipStream_t s) {
    if (gen) hipLaunchKernelGGL(k_hbm<true>, dim3(n_docs), dim3(64), 0, s, p);
    else hipLaunchKernelGGL(k_hbm<false>, dim3(n_docs), dim3(64), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_wave_selftest(const u32* in, u32* out, u32 n_waves, hipStream_t s) {
    hipLaunchKernelGGL(k_wave_selftest, dim3(n_waves), dim3(64), 0, s, in, out);
    return hipGetLastError();
}

}  // namespace mte
