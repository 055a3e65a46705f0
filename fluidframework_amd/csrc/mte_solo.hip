// k_solo: the critical-path documents (gfx950). Its own translation unit so it builds without the
// spill-sinking flag of the bulk kernels (mte_kernels.hip; measured 3.93 vs 3.98 us/op on the lone
// 10^6-op document with it).
#include "wave_hip.hpp"
#include "engine.hpp"
#include "reg_handoff.hpp"
#include "mte_kernels.h"

namespace mte {

// k_solo owns its CU's LDS, so one wave per SIMD is all it ever has: the hint lets the scheduler
// trade registers for latency hiding instead of aiming at an occupancy it can never reach.
#ifndef MTE_SOLO_WPE
#define MTE_SOLO_WPE 1
#endif
// waves of a solo workgroup: one per SIMD, so the critical-path CU holds no other kernel's waves
#ifndef SOLO_WAVES
#define SOLO_WAVES 4
#endif

// Critical-path documents (doc_list[0, n_solo), the longest of the batch): one single-wave
// workgroup each, owning all of a CU's LDS (SoloPlan), at the highest wave priority. The replay
// latency of the longest document bounds a Zipf batch, so it gets the plan with the
// most room and no LDS-pool sharing; it continues HBM-resident only if it outgrows even that.
// CK (option retain): the row engine continues from the previous pass's checkpoint and leaves its
// own -- separate instantiations, so the kernels of a pass without retain are exactly the ones before
// (the checkpoint code in the same kernel cost the lone 10^6-op document 1.6 %: 3.885 vs 3.825 us/op
// on one box, profiles/r06/ck_ab.json)
template <bool GEN, int LVL, bool CK = false>
MTE_DEV void solo_doc(const Params& p) {
    const u32 i = blockIdx.x;
    if (i >= p.n_solo) return;
    const u32 d = p.doc_list[i];
    __builtin_amdgcn_s_setprio(3);
    if (p.solo_started && lane_id() == 0) atomicAdd(p.solo_started, 1u);  // resident: k_solo_gate may go
    // the critical wave's own clock: cycles (s_memtime) against the 100 MHz reference counter
    // (s_memrealtime) over its replay tells a lower shader clock from extra cycles
    const u64 c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    auto stamp = [&]() {
        const u64 c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (p.solo_clk && i < SOLO_CLK_SLOTS && lane_id() == 0) {  // (slot SOLO_CLK_SLOTS: the bulk's stamp)
            u64* o = p.solo_clk + 4 * (u64)i;
            o[0] = c0;
            o[1] = r0;
            o[2] = c1;
            o[3] = r1;
        }
    };
    GenState g;
    bool done;
    u64 at = p.docs[d].op_begin;
    bool handed = false;
    St hst;  // the LDS engine's replay state after a handoff (its LDS arrays are written in place)
    // The LDS engine is constructed only after the row engine is done with the document: nothing of
    // it is live across the row engine's replay loop (its registers were, for the whole replay).
    if constexpr (!GEN && LVL == 0) {
        // lean replay: the whole document state in this wave's registers (reg_engine.hpp); it moves
        // to the LDS plan below only if it outgrows the registers or reaches an op they do not cover
        if (p.reg_solo) {
            RegEngine<> r(p, d);
            if constexpr (CK) at = r.ckpt_resume(at);  // the previous pass's state, if this log extends it
            at = r.replay(at, p.docs[d].op_end);
            if (r.status != REG_HANDOFF) {
                if constexpr (CK) r.ckpt_save(at - p.docs[d].op_begin);
                r.finish();
                stamp();
                __builtin_amdgcn_s_setprio(0);
                return;
            }
            Engine<true, true, LVL> t(p, d);
            t.bind_lds(0);
            if (!reg_handoff(r, t)) t.st.status = DOC_SPILL;  // (the SoloPlan holds any row-engine state)
            hst = t.st;
            handed = true;
        }
    } else if constexpr (!GEN && LVL == 1) {
        // FULL replay (properties, clients up to 63): the PROPS + WIDE row engine, its map ids and
        // high removers in arrays past the rows' slots in the SoloPlan's aux array (blocks
        // RG_BLOCKS.., unused until a handoff has read them)
        if (p.reg_solo) {
            constexpr u32 vb = (u32)offsetof(SoloPlan, vis), ab = (u32)offsetof(SoloPlan, aux);
            static_assert(RG_BLOCKS * 8 * 16 + 2 * RG_BLOCKS * 8 * 4 <= SOLO_POOL * 8 * 16, "props / rm2 arrays in the aux pool");
            // WIDE: clients 32..63 too (a second removers array after the map ids)
            RegEngine<(int)RG_ROWS, false, true, true> r(p, d, vb, ab, 4, 0, ab + RG_BLOCKS * 8 * 16,
                                                         ab + RG_BLOCKS * 8 * 16 + RG_BLOCKS * 8 * 4);
            if constexpr (CK) at = r.ckpt_resume(at);
            if (!r.status) at = r.replay(at, p.docs[d].op_end);
            if (r.status != REG_HANDOFF) {
                if constexpr (CK) r.ckpt_save(at - p.docs[d].op_begin);
                r.finish();
                stamp();
                __builtin_amdgcn_s_setprio(0);
                return;
            }
            Engine<true, true, LVL> t(p, d);
            t.bind_lds(0);
            if (!reg_handoff(r, t)) t.st.status = DOC_SPILL;  // (the SoloPlan holds any row-engine state)
            hst = t.st;
            handed = true;
        }
    }
    Engine<true, true, LVL> e(p, d);
    if (handed) {
        e.wave = 0;  // (bind_lds(0) without clearing the counters the handoff wrote)
        e.st = hst;
    } else {
        e.bind_lds(0);
        e.init();
    }
    if (GEN) {
        e.gen_init(g);
        done = e.generate_run(g);
    } else {
        at = e.replay_run(at);
        done = at >= p.docs[d].op_end;
    }
    if (e.st.status == DOC_SPILL) {
        e.mark_spilled();
    } else if (!done && e.st.status == 0) {
        Engine<false, false, LVL> h(p, d);
        h.continued = true;
        h.bind_solo_slot(i);
        h.adopt(e);
        if (lane_id() == 0) atomicAdd(&p.counters[4], 1u);
        if (GEN) {
            h.generate_run(g);
        } else {
            h.replay_run(at);
        }
        h.finish();
    } else {
        e.finish();
    }
    stamp();
    __builtin_amdgcn_s_setprio(0);
}

// The solo workgroup is SOLO_WAVES waves that each claim a whole SIMD's register file (512 VGPRs +
// AGPRs: the clobbers below make the kernel's allocation the maximum), and all of the CU's LDS: no
// other wave of the pass can be resident on a critical-path CU. Wave 0 replays the document; the
// others wait at the barrier (issuing nothing) until it is done.
template <bool GEN, int LVL, bool CK = false>
__global__ __launch_bounds__(64 * SOLO_WAVES) __attribute__((amdgpu_waves_per_eu(MTE_SOLO_WPE, MTE_SOLO_WPE))) void k_solo(Params p) {
#if SOLO_WAVES > 1
    asm volatile("" ::: "v255", "a255");
    if (wave_first(threadIdx.x >> 6) == 0) solo_doc<GEN, LVL, CK>(p);
    __syncthreads();
#else
    solo_doc<GEN, LVL, CK>(p);
#endif
}

// Bulk lean documents on the row engine (reg_engine.hpp): RW single-SIMD waves per CU (4, 8 = two per
// SIMD, or 12), each with its SIMD's register file (or a half / third of it), replay one document
// after another from the LPT queue. At 4 waves each wave owns a fixed quarter of the CU's LDS, 20
// contiguous slot rows (160 leaf blocks: the long documents of C5 peak at 117). At 8 and 12 the
// waves' rows come from ONE pool of 79 rows (PAGED engine: logical -> pool row table in a VGPR),
// taken as a document grows and given back as it shrinks or ends, so a document at a transient peak
// borrows what its neighbours do not use. (The table lookup costs a lone wave ~11 %: C5 4.93 s
// paged against 4.45 s on fixed rows, hence the fixed quarters at 4 waves.) A document the rows
// cannot hold between two ops, or that reaches an op the row engine does not implement, continues
// HBM-resident in the pass (rows_continue); one the pool cannot grow in the middle of an op restarts
// from its first op (the restart queue) or is re-run by the host (DOC_SPILL). WIDE: batches with writers 32..63 (a second removers
// word per slot, as k_solo's FULL row engine).
// LDS geometry of k_rows: 32 B per slot (vis + aux), +4 with the property map ids (PROPS), +4 with
// the removers 32..63 (WIDE). The pool (8 / 12 waves): vis array, aux array, [props array], [rm2
// array], row mask. Fixed quarters (4 waves): per wave its rows' vis, aux, [props] and [rm2] arrays.
template <bool PROPS, bool WIDE>
struct RowsGeom {
    static constexpr u32 SLOT = 32 + (PROPS ? 4 : 0) + (WIDE ? 4 : 0);  // LDS bytes per slot
    static constexpr u32 POOL = (LDS_BYTES - ROWS_POOL_WORDS * 4) / (64 * SLOT);  // 79, 71 or 63 rows
    static constexpr u32 VIS = 0, AUX = POOL * 64 * 16, PRP = 2 * POOL * 64 * 16;
    static constexpr u32 RM2 = PRP + (PROPS ? POOL * 64 * 4 : 0);
    static constexpr u32 MASK = RM2 + (WIDE ? POOL * 64 * 4 : 0);
    static constexpr u32 LDS = MASK + ROWS_POOL_WORDS * 4;
    static constexpr u32 FIXED_NR = LDS_BYTES / 4 / (64 * SLOT);  // 20, 17 or 16 rows per wave
    static constexpr u32 FIXED_WAVE = FIXED_NR * 64 * SLOT;
    static constexpr u32 FIXED_LDS = 4 * FIXED_WAVE;
    static_assert(LDS <= LDS_BYTES && FIXED_LDS <= LDS_BYTES && POOL <= 32 * ROWS_POOL_WORDS, "k_rows LDS plan");
};
// A k_rows document that outgrows the row plan (or reaches an op the row engine does not implement)
// between two ops continues in the same pass, HBM-resident: the wave claims a free HBM slot
// (Params::spill, the bitmap slot_bits over n_hslots slots; k_lds / k_hbmq do not run beside k_rows),
// dumps the row engine's state into it as it is (rows_dump: every row's fields, the interior levels
// and heap registers; the scalars in a queue record, Params::rows_cont) and goes on to its next
// document. k_rows_cont, launched right after k_rows, rebuilds the row engine from the dump in its
// own LDS, hands it to the HBM engine in the same slot (reg_handoff) and replays the rest of its ops
// there (DocRes mode 6). k_rows itself holds only the dump (with the HBM engine's replay compiled in,
// the 12-wave PROPS build spilled 441 VGPRs: C3 1.34 -> 1.61 s), and only in its fixed-row builds.
// No free slot, a slot too small for the state, or a slot it outgrows later: the host's re-run.
// A free slot, or NONE when every slot is held: the bitmap is scanned from a per-workgroup start, and
// a bit lost to another wave's claim moves on to the next free bit of the same word (the word the
// atomic returned), so a wave gives up only when it saw every word full.
MTE_DEV u32 try_hslot(const Params& p) {
    const u32 L = lane_id();
    const u32 nw = (p.n_hslots + 31) >> 5;
    const u32 start = (blockIdx.x * 7u) % nw;
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
            const u32 pad = (ww == nw - 1 && (p.n_hslots & 31)) ? ~0u << (p.n_hslots & 31) : 0u;
            u32 cur = wave_read(word, l);
            for (u32 t = 0; t < 32 && cur != 0xFFFFFFFFu; t++) {
                const u32 bit = (u32)__builtin_ctz(~cur);
                u32 old = 0;
                if (L == 0) old = atomicOr(&p.slot_bits[ww], 1u << bit);
                old = wave_read(old, 0);
                if (!(old & (1u << bit))) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the previous holder's writes
                    return ww * 32 + bit;
                }
                cur = old | pad | (1u << bit);
            }
            m &= m - 1;
        }
    }
    return NONE;
}
// The dump in a slot: logical row rr's field f (len, seq, rseq, meta, cap, toff, rm, sid, [props],
// [rm2]) at words ((rr * NF + f) * 64 + lane), then LV, HK and HS (8 registers each) from word
// RG_ROWS * NF * 64; the record: doc, slot, op index (lo, hi), then the scalars below.
template <bool PROPS, bool WIDE>
struct RowsDump {
    static constexpr u32 NF = 8 + (PROPS ? 1u : 0u) + (WIDE ? 1u : 0u);
    static constexpr u32 REGS = (u32)RG_ROWS * NF * 64;
    static constexpr u64 BYTES = (u64)(REGS + 24 * 64) * 4;
};
const u64 ROWS_DUMP_BYTES = RowsDump<true, true>::BYTES;  // (mte_kernels.h: the host checks slots against it)
enum : u32 { RD_NLB = 4, RD_HEIGHT, RD_HEAPSIZE, RD_HEAPTOP, RD_MINSEQ, RD_CURSEQ, RD_SEGNEXT, RD_ARENATOP,
             RD_ARENASEL, RD_MAPNEXT, RD_NOPS, RD_NMSGS, RD_NGC, RD_MAXLB, RD_END };
static_assert(RD_END <= ROWS_CONT_WORDS, "rows_cont record");

// Returns 0 when the document was queued for k_rows_cont, else why not (DocRes::spill_why's low byte
// after the caller's mark): 1 no free slot or queue, 3 the rows do not hold the whole state (a PAGED
// engine that never got its first row)
template <class R>
MTE_DEV u32 rows_dump(const Params& p, R& r, u32 d, u64 at) {
    typedef RowsDump<R::kProps, R::kWide> D;
    if (!r.rows_whole()) return 3;
    if (!p.slot_bits || !p.n_hslots || !p.rows_cont) return 1;
    const u32 slot = try_hslot(p);
    if (slot == NONE) return 1;
    const u32 L = lane_id();
    u32* base = reinterpret_cast<u32*>(p.spill + (u64)(p.slot_hbm0 + slot) * p.slot_bytes);
    const u32 nrows = (r.n_lb + 7) >> 3;
    for (u32 rr = 0; rr < nrows; rr++) {
        const auto w = r.ldrow(rr);
        u32* o = base + (u64)rr * D::NF * 64 + L;
        o[0] = w.len.x;
        o[64] = w.seq.x;
        o[128] = w.rseq.x;
        o[192] = w.meta.x;
        o[256] = w.cap.x;
        o[320] = w.toff.x;
        o[384] = w.rm.x;
        o[448] = w.sid.x;
        if constexpr (R::kProps) o[512] = w.props.x;
        if constexpr (R::kWide) o[64 * (D::NF - 1)] = w.rm2.x;
    }
    u32* g = base + D::REGS + L;
#pragma unroll
    for (u32 i = 0; i < 8; i++) {
        g[64 * i] = r.LV.get(i).x;
        g[64 * (8 + i)] = r.HK.get(i).x;
        g[64 * (16 + i)] = r.HS.get(i).x;
    }
    u32 k = 0;
    if (L == 0) k = atomicAdd(&p.counters[10], 1u);
    k = wave_read(k, 0);
    u32* rec = p.rows_cont + (u64)k * ROWS_CONT_WORDS;
    const u32 v = L == 0 ? d : L == 1 ? slot : L == 2 ? (u32)at : L == 3 ? (u32)(at >> 32)
                : L == RD_NLB ? r.n_lb : L == RD_HEIGHT ? r.height : L == RD_HEAPSIZE ? r.heapSize
                : L == RD_HEAPTOP ? (u32)r.heapTop : L == RD_MINSEQ ? (u32)r.minSeq : L == RD_CURSEQ ? (u32)r.curSeq
                : L == RD_SEGNEXT ? r.segNext : L == RD_ARENATOP ? r.arenaTop : L == RD_ARENASEL ? r.arenaSel
                : L == RD_MAPNEXT ? r.mapNext : L == RD_NOPS ? r.ops_n() : L == RD_NMSGS ? r.msgs_n()
                : L == RD_NGC ? r.n_gc : r.max_lb;
    if (L < RD_END) rec[L] = v;
    // release: the dump and the record before k_rows_cont (another XCD's L2) reads them
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    return 0;
}

// k_rows documents dumped into HBM slots mid-pass: workgroup i rebuilds queued record i's row engine
// in its LDS (the rows at the k_solo layout's offsets, 32 rows), hands it to the HBM engine in the same
// slot, replays the rest of its ops (DocRes mode 6) and gives the slot back. One workgroup per slot
// (every record holds one); those past the queue exit at once.
template <bool PROPS, bool WIDE>
__global__ __launch_bounds__(64) void k_rows_cont(Params p) {
    typedef RowsDump<PROPS, WIDE> D;
    typedef RegEngine<(int)RG_ROWS, false, PROPS, WIDE> R;
    constexpr int LVL = PROPS ? 1 : 0;
    const u32 L = lane_id();
    const u32 i = blockIdx.x;
    if (i >= wave_first(p.counters[10])) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const u32 w = p.rows_cont[(u64)i * ROWS_CONT_WORDS + (L < ROWS_CONT_WORDS ? L : 0u)];
    const u32 d = wave_read(w, 0), slot = wave_read(w, 1);
    const u64 at = (u64)wave_read(w, 2) | ((u64)wave_read(w, 3) << 32);
    constexpr u32 VB = 0, AB = RG_ROWS * 64 * 16, PB = 2 * RG_ROWS * 64 * 16, R2B = PB + (PROPS ? RG_ROWS * 64 * 4 : 0);
    R r(p, d, VB, AB, 5, 0, PB, R2B);  // (init: every row zero)
    r.n_lb = wave_read(w, RD_NLB);
    r.height = wave_read(w, RD_HEIGHT);
    r.heapSize = wave_read(w, RD_HEAPSIZE);
    r.heapTop = (i32)wave_read(w, RD_HEAPTOP);
    r.minSeq = (i32)wave_read(w, RD_MINSEQ);
    r.curSeq = (i32)wave_read(w, RD_CURSEQ);
    r.segNext = wave_read(w, RD_SEGNEXT);
    r.arenaTop = wave_read(w, RD_ARENATOP);
    r.arenaSel = wave_read(w, RD_ARENASEL);
    r.mapNext = wave_read(w, RD_MAPNEXT);
    r.set_counts(wave_read(w, RD_NOPS), wave_read(w, RD_NMSGS));
    r.n_gc = wave_read(w, RD_NGC);
    r.max_lb = wave_read(w, RD_MAXLB);
    r.status = 0;
    const u32* base = reinterpret_cast<const u32*>(p.spill + (u64)(p.slot_hbm0 + slot) * p.slot_bytes);
    const u32 nrows = (r.n_lb + 7) >> 3;
    for (u32 rr = 0; rr < nrows && rr < RG_ROWS; rr++) {
        const u32* o = base + (u64)rr * D::NF * 64 + L;
        typename R::Row x;
        x.len = simd::V{o[0]};
        x.seq = simd::V{o[64]};
        x.rseq = simd::V{o[128]};
        x.meta = simd::V{o[192]};
        x.cap = simd::V{o[256]};
        x.toff = simd::V{o[320]};
        x.rm = simd::V{o[384]};
        x.sid = simd::V{o[448]};
        if constexpr (PROPS) x.props = simd::V{o[512]};
        if constexpr (WIDE) x.rm2 = simd::V{o[64 * (D::NF - 1)]};
        r.strow(rr, x);
    }
    const u32* g = base + D::REGS + L;
#pragma unroll
    for (u32 q = 0; q < 8; q++) {
        r.LV.set(q, simd::V{g[64 * q]});
        r.HK.set(q, simd::V{g[64 * (8 + q)]});
        r.HS.set(q, simd::V{g[64 * (16 + q)]});
    }
    // every read of the dump done before the handoff writes the HBM engine's arrays over it
    __builtin_amdgcn_s_waitcnt(0);
    wave_sync();
    {
        Engine<false, false, LVL> h(p, d);
        h.bind_slot(p.slot_hbm0 + slot);
        h.reset_stats();
        if (!reg_handoff(r, h)) {
            r.mark_spilled();
            if (L == 0) p.res[d].spill_why |= 2u;
        } else {
            h.from_rows = true;
            h.replay_run(at);
            if (h.st.status == DOC_SPILL) h.mark_spilled();
            else h.finish();
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (L == 0) atomicAnd(&p.slot_bits[slot >> 5], ~(1u << (slot & 31)));
}
template <bool PROPS, bool WIDE>
static hipError_t launch_rows_cont_t(const Params& p, u32 n_slots, hipStream_t s) {
    const void* k = (const void*)k_rows_cont<PROPS, WIDE>;
    constexpr u32 LDS = RG_ROWS * 64 * (32 + (PROPS ? 4 : 0) + (WIDE ? 4 : 0));
    static const hipError_t attr = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
    if (attr != hipSuccess) return attr;
    void* args[] = {(void*)&p};
    return hipLaunchKernel(k, dim3(n_slots), dim3(64), args, LDS, s);
}
hipError_t launch_rows_cont(const Params& p, bool props, bool wide, u32 n_slots, hipStream_t s) {
    if (!n_slots || !p.rows_cont) return hipSuccess;
    if (wide) return props ? launch_rows_cont_t<true, true>(p, n_slots, s) : hipErrorInvalidValue;
    return props ? launch_rows_cont_t<true, false>(p, n_slots, s) : launch_rows_cont_t<false, false>(p, n_slots, s);
}

// CK (option retain, 4 waves only): documents continue from the previous pass's checkpoints and leave
// their own (reg_engine.hpp ckpt_*)
template <int RW, bool PROPS, bool WIDE, bool CK = false>
__global__ __launch_bounds__(64 * RW) __attribute__((amdgpu_waves_per_eu(RW / 4, RW / 4))) void k_rows(Params p) {
    typedef RowsGeom<PROPS, WIDE> G;
    constexpr bool PAGED = RW > 4;
    const u32 w = wave_first(threadIdx.x >> 6);
    if constexpr (PAGED) {
        u32* mask = reinterpret_cast<u32*>(reinterpret_cast<unsigned char*>(g_lds_dyn) + G::MASK);
        // rows past the pool (or past the rows_pool_lim test knob) are marked taken
        const u32 np = p.rows_pool_lim && p.rows_pool_lim < G::POOL ? p.rows_pool_lim : G::POOL;
        if (threadIdx.x < ROWS_POOL_WORDS)
            mask[threadIdx.x] = threadIdx.x * 32 + 32 <= np ? 0u
                                : threadIdx.x * 32 >= np   ? ~0u
                                                           : ~((1u << (np - threadIdx.x * 32)) - 1u);
        __syncthreads();
    }
    const u32 vb = PAGED ? G::VIS : w * G::FIXED_WAVE;
    const u32 ab = PAGED ? G::AUX : vb + G::FIXED_NR * 64u * 16u;
    const u32 pb = PAGED ? G::PRP : vb + G::FIXED_NR * 64u * 32u;
    const u32 r2b = PAGED ? G::RM2 : pb + (PROPS ? G::FIXED_NR * 64u * 4u : 0u);
    if (blockIdx.x == 0 && threadIdx.x == 0 && p.solo_clk) p.solo_clk[4 * SOLO_CLK_SLOTS] = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        // a document another wave gave back when the pool was full restarts first (once; a second
        // failure goes to the host's re-run), then the LPT queue
        u32 d = NONE;
        bool again = false;
        if (PAGED && p.rows_retry) {
            u32 slot = NONE;
            if (lane_id() == 0) {
                u32* pushed = &p.counters[8];
                u32* popped = &p.counters[9];
                u32 old = __hip_atomic_load(popped, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                while (old < __hip_atomic_load(pushed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) {
                    const u32 seen = atomicCAS(popped, old, old + 1u);
                    if (seen == old) {
                        slot = old;
                        break;
                    }
                    old = seen;
                }
                if (slot != NONE) {  // the pusher bumps the count before its slot write lands: wait for it
                    u32 v = 0;
                    for (u32 t = 0; t < (1u << 20) && v == 0; t++)
                        v = __hip_atomic_load(p.rows_retry + slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    slot = v ? v - 1u : NONE;
                }
            }
            d = wave_read(slot, 0);
            again = d != NONE;
        }
        if (d == NONE) {
            u32 i = 0;
            if (lane_id() == 0) i = p.n_prio + atomicAdd(&p.counters[0], 1u);
            i = wave_read(i, 0);
            if (i >= p.n_list) {
                // the queue is drained; documents still being given back are picked up by waves that
                // have not finished yet, or go to the host's re-run
                break;
            }
            d = p.doc_list[i];
        }
        RegEngine<PAGED ? (int)RG_ROWS : (int)G::FIXED_NR, PAGED, PROPS, WIDE> r(p, d, vb, ab, 5, G::MASK, pb, r2b);
        u64 at = p.docs[d].op_begin;
        if constexpr (CK) at = r.ckpt_resume(at);
        if (!r.status) at = r.replay(at, p.docs[d].op_end);
        if (r.status == REG_HANDOFF && PAGED && p.rows_retry && r.pool_full && !again) {
            // marked for the host's re-run first (so a document no wave restarts is still replayed),
            // then queued to restart from its first op; a restart that finishes overwrites the mark
            r.mark_spilled();
            if (lane_id() == 0) {
                const u32 k = atomicAdd(&p.counters[8], 1u);
                __hip_atomic_store(p.rows_retry + k, d + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (r.status == REG_HANDOFF) {
            // between two ops on fixed rows (4 waves: the route of long and of many-writer documents,
            // the ones that outgrow their rows): continue HBM-resident in this pass (rows_dump,
            // k_rows_cont); inside an op (half applied), or on the shared pool (8 / 12 waves, whose
            // builds even the dump's code took from 0-16 to 8-90 spilled VGPRs), the host's re-run
            u32 why = 5;
            if constexpr (!PAGED) why = r.midop ? 4u : rows_dump(p, r, d, at);
            if (why) {
                r.mark_spilled();
                if (lane_id() == 0) p.res[d].spill_why |= why;
            }
        } else {
            if constexpr (CK) r.ckpt_save(at - p.docs[d].op_begin);
            r.finish();
        }
        r.release_rows();
    }
}

template <bool PROPS, bool WIDE>
static hipError_t launch_rows_t(const Params& p, u32 rw, u32 n_groups, bool ck, hipStream_t s) {
    typedef RowsGeom<PROPS, WIDE> G;
    const void* k = ck ? (const void*)k_rows<4, PROPS, WIDE, true>
                  : rw == 12 ? (const void*)k_rows<12, PROPS, WIDE>
                  : rw == 8  ? (const void*)k_rows<8, PROPS, WIDE>
                             : (const void*)k_rows<4, PROPS, WIDE>;
    if (ck) rw = 4;
    static const hipError_t attr = [] {
        hipError_t r = hipFuncSetAttribute((const void*)k_rows<4, PROPS, WIDE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::FIXED_LDS);
        if (r == hipSuccess)
            r = hipFuncSetAttribute((const void*)k_rows<4, PROPS, WIDE, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::FIXED_LDS);
        for (const void* f : {(const void*)k_rows<8, PROPS, WIDE>, (const void*)k_rows<12, PROPS, WIDE>})
            if (r == hipSuccess) r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
        return r;
    }();
    if (attr != hipSuccess) return attr;
    void* args[] = {(void*)&p};
    return hipLaunchKernel(k, dim3(n_groups), dim3(64 * rw), args, (size_t)(rw == 4 ? G::FIXED_LDS : G::LDS), s);
}
// WIDE (clients 32..63) only with PROPS: such a batch is a FULL one (the lean LDS kernels keep 32-bit
// removers masks), whose row engine is the property-carrying one. ck (option retain): the checkpointing
// instantiation, 4 waves per CU on fixed rows.
hipError_t launch_rows(const Params& p, u32 waves_per_cu, u32 n_groups, bool props, bool wide, bool ck, hipStream_t s) {
    const u32 rw = waves_per_cu >= 12 ? 12u : waves_per_cu >= 8 ? 8u : 4u;
    if (wide) return props ? launch_rows_t<true, true>(p, rw, n_groups, ck, s) : hipErrorInvalidValue;
    return props ? launch_rows_t<true, false>(p, rw, n_groups, ck, s) : launch_rows_t<false, false>(p, rw, n_groups, ck, s);
}

#define MTE_PICK(K, gen, lvl)                                                                           \
    ((gen) ? (const void*)K<true, 1> : (lvl) >= 2 ? (const void*)K<false, 2> : (lvl) == 1 ? (const void*)K<false, 1> \
                                                                               : (const void*)K<false, 0>)

hipError_t launch_solo(const Params& p, bool gen, int full, u32 n_solo, bool ck, hipStream_t s) {
    static const hipError_t attr = [] {
        hipError_t r = hipFuncSetAttribute((const void*)k_solo<true, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(SoloPlan));
        for (const void* k : {(const void*)k_solo<false, 0>, (const void*)k_solo<false, 1>, (const void*)k_solo<false, 2>,
                              (const void*)k_solo<false, 0, true>, (const void*)k_solo<false, 1, true>})
            if (r == hipSuccess) r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(SoloPlan));
        return r;
    }();
    if (attr != hipSuccess) return attr;
    void* args[] = {(void*)&p};
    // (the checkpointing instantiations exist for the row-engine levels only: lean and FULL)
    const void* k = ck && !gen && full == 0 ? (const void*)k_solo<false, 0, true>
                  : ck && !gen && full == 1 ? (const void*)k_solo<false, 1, true>
                                            : MTE_PICK(k_solo, gen, full);
    return hipLaunchKernel(k, dim3(n_solo), dim3(64 * SOLO_WAVES), args, sizeof(SoloPlan), s);
}

}  // namespace mte
