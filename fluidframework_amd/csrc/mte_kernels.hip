// HIP kernels of the replay engine (gfx950); k_solo is in mte_solo.hip (built with other flags).
//
//   k_lds<GEN>: ONE workgroup per CU, LDS_WAVES waves, all 160 KiB of LDS (engine_types.hpp LdsPlan).
//               Waves pull documents from a queue in LPT order (longest first) and replay
//               (or generate) each with the whole per-document state resident in LDS. A document
//               that outgrows the plan between two ops continues HBM-resident in the wave's own
//               HBM slot; one that fails mid-op is marked DOC_SPILL for the host's re-run.
//   k_hbmq<GEN>: one wave per document taken from the same queue, state HBM-resident in a slot
//               from a bitmap, co-resident with k_lds on every CU (second stream).
//   k_hbm<GEN>: one wave per listed document, state resident in HBM (DocCfg::hb_*): the host's
//               re-run of DOC_SPILL documents.
#include "wave_hip.hpp"
#include "engine.hpp"
#include "reg_handoff.hpp"
#include "mte_kernels.h"

namespace mte {

// Waves per SIMD the register allocation of k_lds / k_hbmq is sized for (512 VGPRs / n each): the
// two kernels share every CU, LDS_WAVES / 4 LDS waves plus hbm_waves_per_cu / 4 HBM waves per SIMD.
#ifndef MTE_LDS_WPE
#define MTE_LDS_WPE 4
#endif
#ifndef MTE_HBMQ_WPE
#define MTE_HBMQ_WPE 4
#endif
template <bool GEN, int LVL>
__global__ __launch_bounds__(64 * LDS_WAVES) __attribute__((amdgpu_waves_per_eu(MTE_LDS_WPE))) void k_lds(Params p) {
    LdsPlan* lp = &g_plan;
    const u32 t = threadIdx.x, L = t & 63;
    const u32 w = wave_first(t >> 6);  // wave-uniform (the compiler cannot infer it from threadIdx)
    // the bulk's start on the 100 MHz reference clock, beside k_solo's own stamps (dispatch delays)
    if (blockIdx.x == 0 && t == 0 && p.solo_clk) p.solo_clk[4 * SOLO_CLK_SLOTS] = __builtin_amdgcn_s_memrealtime();
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
    // a small batch is spread over every CU (lds_active waves per workgroup); critical-path
    // documents (doc_list[0, n_prio), counters[5]) are taken by LDS waves only
    for (; w < p.lds_active;) {
        u32 i = 0;
        if (L == 0) {  // doc_list[0, n_solo) belongs to k_solo
            i = p.n_prio > p.n_solo ? p.n_solo + atomicAdd(&p.counters[5], 1u) : p.n_prio;
            if (i >= p.n_prio) i = p.n_prio + atomicAdd(&p.counters[0], 1u);
        }
        i = wave_read(i, 0);
        if (i >= p.n_list) break;
        const u32 d = p.doc_list[i];
        const bool prio = p.docs[d].prio != 0;
        if (prio) __builtin_amdgcn_s_setprio(3);  // the critical path issues first on its SIMD
        Engine<true, false, LVL> e(p, d);
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
        } else if (!done && e.st.status == 0 && p.slot_blk < POOL_BLOCKS + 64) {
            e.mark_spilled();  // slots too small to hold the LDS block ids (test knob): host re-run
        } else if (!done && e.st.status == 0) {
            // the LDS plan ran out of room between two ops: continue HBM-resident, same wave
            Engine<false, false, LVL> h(p, d);
            h.continued = true;
            h.bind_slot(blockIdx.x * LDS_WAVES + w);
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
            e.finish();
        }
        e.release();
        if (prio) __builtin_amdgcn_s_setprio(0);
    }
}

// HBM slot of a k_hbmq wave: a free bit of the slot bitmap (cleared by the host before each run).
// At most n_hslots waves of k_hbmq are resident at once (the host sizes it from the occupancy
// bound), so a search finds a free slot unless slots are budget-limited; then the wave waits for
// a holder to finish its document.
MTE_DEV u32 acquire_hslot(const Params& p) {
    const u32 L = lane_id();
    const u32 nw = (p.n_hslots + 31) >> 5;
    const u32 start = blockIdx.x % nw;
    for (;;) {
        for (u32 base = 0; base < nw; base += 64) {
            const u32 w = (start + base + L) % nw;
            u32 word = 0xFFFFFFFFu;
            if (base + L < nw) {
                word = __hip_atomic_load(&p.slot_bits[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (w == nw - 1 && (p.n_hslots & 31)) word |= ~0u << (p.n_hslots & 31);
            }
            u64 m = wave_ballot(word != 0xFFFFFFFFu);
            while (m) {
                const u32 l = (u32)__builtin_ctzll(m);
                const u32 ww = wave_read(w, l);
                const u32 bit = (u32)__builtin_ctz(~wave_read(word, l));
                u32 old = 0;
                if (L == 0) old = atomicOr(&p.slot_bits[ww], 1u << bit);
                old = wave_read(old, 0);
                if (!(old & (1u << bit))) {
                    // acquire: the previous holder (any CU, any XCD) released its writes
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    return ww * 32 + bit;
                }
                m &= m - 1;
            }
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

// HBM-resident waves beside the LDS workgroups: each workgroup is one wave that takes ONE document
// from the queue k_lds drains (LPT order), replays it in a free HBM slot and exits; the grid has a
// workgroup per document, so waves keep arriving as CU resources free up. k_lds holds 2 waves per
// SIMD and all the LDS, these waves hold no LDS: on the second stream they fill the issue slots
// the LDS waves leave idle while they wait on LDS/ALU latency chains. (One document per workgroup
// rather than a persistent loop: with the engine inlined into a loop, hipcc 7.2 built a divergent
// loop latch that came back with EXEC narrowed to one lane.)
template <bool GEN, int LVL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MTE_HBMQ_WPE))) void k_hbmq(Params p) {
    const u32 L = lane_id();
    // A slot first, then a document: a wave that claimed a document before it held a slot waited,
    // with the document, for one of the few slots -- hundreds of the batch's longest documents then
    // queued behind k_hbmq's slots while the LDS waves ran dry (2 048 x 3 000-op logs: 41 ms to 2.4 s per
    // pass, now 50-57 ms, profiles/r06/mixed_route.json). A wave that finds the queue drained
    // before or after taking its slot gives the slot back and exits.
    if (wave_first(__hip_atomic_load(&p.counters[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + p.n_prio >= p.n_list)
        return;
    const u32 slot = acquire_hslot(p);
    u32 i = 0;
    if (L == 0) i = p.n_prio + atomicAdd(&p.counters[0], 1u);
    i = wave_read(i, 0);
    if (i >= p.n_list) {
        if (L == 0) atomicAnd(&p.slot_bits[slot >> 5], ~(1u << (slot & 31)));
        return;
    }
    const u32 d = p.doc_list[i];
    Engine<false, false, LVL> e(p, d);
    e.bind_slot(p.slot_hbm0 + slot);
    e.reset_stats();
    e.init();
    if (GEN) {
        GenState g;
        e.gen_init(g);
        e.generate_run(g);
    } else {
        e.replay_run(p.docs[d].op_begin);
    }
    e.finish();
    // release: write this XCD's dirty lines of the slot back before another wave (possibly on
    // another XCD, whose L2 is not coherent with this one) can take it over
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (L == 0) atomicAnd(&p.slot_bits[slot >> 5], ~(1u << (slot & 31)));
}

template <bool GEN, int LVL>
__global__ __launch_bounds__(64) void k_hbm(Params p) {
    const u32 d = p.doc_list[blockIdx.x];
    Engine<false, false, LVL> e(p, d);
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

// Kernel instantiations: the generator always runs the FULL engine (its C3 kind uses properties);
// a replay runs the lean one (level 0) when the host found the batch free of the optional features,
// the EXT one (level 2) when it carries catch-up records or permutation runs, else FULL (level 1)
// (mte_host.cpp mte_load).
#define MTE_PICK(K, gen, lvl)                                                                           \
    ((gen) ? (const void*)K<true, 1> : (lvl) >= 2 ? (const void*)K<false, 2> : (lvl) == 1 ? (const void*)K<false, 1> \
                                                                               : (const void*)K<false, 0>)

template <class Plan>
static hipError_t lds_attr(const void* k) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(Plan));
}

hipError_t launch_lds(const Params& p, bool gen, int full, u32 n_groups, hipStream_t s) {
    // the LdsPlan is dynamic LDS: a static 160 KiB declaration makes the compiler size registers
    // for the 2 waves/SIMD that LDS allows, while k_lds is kept to <= 128 VGPRs so k_hbmq waves fit
    // beside it (2 + 2 per SIMD)
    static const hipError_t attr = [] {
        hipError_t r = lds_attr<LdsPlan>((const void*)k_lds<true, 1>);
        for (const void* k : {(const void*)k_lds<false, 0>, (const void*)k_lds<false, 1>, (const void*)k_lds<false, 2>})
            if (r == hipSuccess) r = lds_attr<LdsPlan>(k);
        return r;
    }();
    if (attr != hipSuccess) return attr;
    void* args[] = {(void*)&p};
    return hipLaunchKernel(MTE_PICK(k_lds, gen, full), dim3(n_groups), dim3(64 * LDS_WAVES), args, sizeof(LdsPlan), s);
}
hipError_t launch_hbm(const Params& p, bool gen, int full, u32 n_docs, hipStream_t s) {
    void* args[] = {(void*)&p};
    return hipLaunchKernel(MTE_PICK(k_hbm, gen, full), dim3(n_docs), dim3(64), args, 0, s);
}
hipError_t launch_hbmq(const Params& p, bool gen, int full, u32 n_waves, hipStream_t s) {  // n_waves >= docs left
    void* args[] = {(void*)&p};
    return hipLaunchKernel(MTE_PICK(k_hbmq, gen, full), dim3(n_waves), dim3(64), args, 0, s);
}

// The bulk kernels start only once every solo workgroup is resident. Launched on the bulk's stream
// between k_solo (its own stream) and k_lds / k_rows: without it the bulk sometimes took the CUs first
// and a solo workgroup waited ~1.2 s for one to drain (solo_start_delay_ms in the bench line), on about
// every other C4 step. One wave, no LDS; gives up after `limit` 100 MHz ticks so it can never hold
// the bulk back for long (or hang) whatever the dispatcher does.
__global__ __launch_bounds__(64) void k_solo_gate(const u32* started, u32 n, u64 limit) {
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const u32 v = __hip_atomic_load(started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wave_read(v, 0) >= n) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > limit) break;
        __builtin_amdgcn_s_sleep(16);
    }
}

hipError_t launch_solo_gate(const u32* started, u32 n_solo, hipStream_t s) {
    hipLaunchKernelGGL(k_solo_gate, dim3(1), dim3(64), 0, s, started, n_solo, (u64)2000000);  // 20 ms
    return hipGetLastError();
}

hipError_t launch_wave_selftest(const u32* in, u32* out, u32 n_waves, hipStream_t s) {
    hipLaunchKernelGGL(k_wave_selftest, dim3(n_waves), dim3(64), 0, s, in, out);
    return hipGetLastError();
}

}  // namespace mte
