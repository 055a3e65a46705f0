// engine.hpp — the per-document replay engine executed by ONE wavefront (64 lanes).
//
// Restates the observer replay path of @fluidframework/merge-tree 0.31.0 (paths below are relative
// to packages/dds/merge-tree/src) in an MI355X-first shape:
//   * the B-tree is kept exactly (8-slot leaf blocks, 8->4+4 splits, root growth, zamboni
//     scour/pack), because segment boundaries and SnapshotV1 bytes depend on it;
//   * Engine<true>: the whole per-document state is resident in LDS. Leaf blocks come from a pool
//     shared by the 8 waves of the CU (engine_types.hpp LdsPlan); the doc-order block list `ord`
//     carries per block (id, observer-visible length, max seq, child count), so position resolution
//     is ONE wavefront prefix scan over up to 64 blocks (lane = block): a block whose max seq is
//     <= refSeq has the same visible length for every client (mergeTree.ts:1673-1696), only blocks
//     touched inside the collaboration window evaluate the predicate slot by slot;
//     then one 8-lane scan inside the chosen block finds the slot (breakTie, mergeTree.ts:2248-2277);
//   * Engine<false>: the same code over an HBM-resident copy of the same layout, used for documents
//     that outgrow the LDS plan (the host re-runs them);
//   * PartialSequenceLengths (partialLengths.ts) is not needed: the scan evaluates the predicate;
//   * serial pieces (heap, tree maintenance) run uniformly with lane-0 stores.
#pragma once
#include <stdint.h>

#include "engine_types.hpp"
#include "wave_hip.hpp"

namespace mte {

// The LDS of the replay kernel: one plan per CU (k_lds declares nothing else).
extern __shared__ uint4 g_lds_dyn[];  // LdsPlan, dynamic (so waves_per_eu bounds VGPRs)
#define g_plan (*reinterpret_cast<LdsPlan*>(g_lds_dyn))
#define g_solo (*reinterpret_cast<SoloPlan*>(g_lds_dyn))  // k_solo's plan (the same dynamic LDS)

// Phase profiling (compile with -DMTE_PROFILE): inclusive s_memtime cycles per phase.
enum ProfSlot : u32 {
    PF_APPLY = 0, PF_RESOLVE, PF_INSERT_SLOT, PF_RANGE, PF_ZAMBONI, PF_SCOUR, PF_HEAP, PF_FIND_SEG,
    PF_MAP, PF_PACK, PF_FETCH, PF_LRU, PF_TEXT, PF_ALLOC, PF_OPS, PF_TOTAL,
    // event counts
    PN_RESOLVE, PN_DIRTY, PN_SCOUR, PN_SCOUR_CHANGED, PN_PACK, PN_POP, PN_PUSH, PN_SPLIT_BLK,
    // finer scopes
    PF_OP_INS, PF_OP_REM, PF_EDIT, PF_SPLIT, PF_ZAM_EDIT, PF_ZAM_MSN, PF_RES_BLOCKS, PF_RES_SLOT, PF_BLEN_DIRTY,
    PF_SCOUR_CHAIN, PF_SCOUR_WRITE, PF_LOOP, PN_INS, PN_REM, PF_APRE, PF_APOST
};
#ifdef MTE_PROFILE
// MTE_PROF_ONLY=<slot>: time that one phase only (every s_memtime scope and counter atomic perturbs
// a lone wave, so a full phase profile overstates the small phases); the op count stays on
#ifdef MTE_PROF_ONLY
#define MTE_PON(slot) ((slot) == MTE_PROF_ONLY)
#else
#define MTE_PON(slot) true
#endif
// counters accumulate straight into the per-document HBM record (fire-and-forget atomics: no
// registers held across the engine, which runs at its 128-VGPR bound)
#define MTE_COUNT(slot, n)                                                          \
    do {                                                                            \
        if (MTE_PON(slot) || (slot) == PF_OPS)                                      \
            if (lane_id() == 0) atomicAdd(prof + (slot), (u64)(n));                 \
    } while (0)
#else
#define MTE_COUNT(slot, n) \
    do {                   \
    } while (0)
#endif
#ifdef MTE_PROFILE
template <bool ON>
struct ProfScopeT {
    u64* acc;
    u64 t0;
    MTE_DEV ProfScopeT(u64* a) : acc(a), t0(ON ? __builtin_amdgcn_s_memtime() : 0) {}
    MTE_DEV ~ProfScopeT() {
        if (ON) {
            const u64 dt = __builtin_amdgcn_s_memtime() - t0;
            if (lane_id() == 0) atomicAdd(acc, dt);
        }
    }
};
typedef ProfScopeT<true> ProfScope;
#define MTE_PROF(slot) ProfScopeT<MTE_PON(slot)> _prof_scope_##slot(prof + (slot))
#elif defined(MTE_MARKERS)
// static code-size analysis (tools/asm_regions.py): phase scopes as assembly comments
template <u32 S>
struct MarkScope {
    MTE_DEV MarkScope() { asm volatile("; MTE_BEGIN %0" ::"i"(S)); }
    MTE_DEV ~MarkScope() { asm volatile("; MTE_END %0" ::"i"(S)); }
};
#define MTE_PROF(slot) MarkScope<slot> _mark_scope_##slot
#else
#define MTE_PROF(slot) \
    do {               \
    } while (0)
#endif

struct Found {
    bool ok;
    u32 k;      // doc-order index of the leaf block
    u32 blk;    // leaf block id
    u32 cnt;    // its child count
    i32 slot;   // first qualifying slot, -1 => append at block end
    i32 r;      // pos - cumBefore(slot)
    i32 cum;    // visible length before the block
};

struct Rng {  // xoshiro256** seeded through splitmix64
    u64 s[4];
    MTE_DEV static u64 splitmix(u64& x) {
        u64 z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    MTE_DEV void seed(u64 x) {
        for (int i = 0; i < 4; i++) s[i] = splitmix(x);
    }
    MTE_DEV static u64 rotl(u64 x, int k) { return (x << k) | (x >> (64 - k)); }
    MTE_DEV u64 next() {
        u64 r = rotl(s[1] * 5, 7) * 9;
        u64 t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    MTE_DEV u32 below(u32 n) { return (u32)(((next() >> 32) * (u64)n) >> 32); }
};

// One leaf slot in registers: vis = (len, seq, rseq, meta), aux = (props, toff, tcap, sid).
struct Seg {
    u32 len;
    i32 seq;
    i32 rseq;
    u32 meta;   // client | removedClient << 8 | flags
    u32 props;  // property-map id (0 = undefined)
    u32 toff;   // text offset (ARENA_BIT => merge arena, else doc payload); marker: refType
    u32 tcap;   // owned arena capacity from toff (0 for payload text)
    u32 sid;    // segment id (LRU heap identity)
};

// Synthetic writers' state (generator), resumable across the LDS -> HBM hand-off.
struct GenState {
    Rng rng;
    i32 ref[GEN_MAX_CLIENTS];
    u32 sid_of[GEN_MAX_CLIENTS];
    u32 nextShort, pay;
    i32 lastC, lastR, lastPos;
    u64 step;
};

// Uniform replay state (identical in every lane).
struct St {
    u32 root, height, n_lb;
    i32 minSeq, curSeq;
    u32 heapSize, segNext, arenaTop, arenaSel, mapNext;
    i32 heapTop;  // key (maxSeq) of the heap's root; meaningful while heapSize > 0
    u32 lbFree, lbBump, inFree, inBump, inUsed, credit;
    i32 status;
    u32 adirty, gdirty;
};

// FULL = false: the instantiation for batches that use no property sets, no client id above 31 and no
// '\n' in any payload (the host checks, mte_host.cpp batch_is_lean): property maps, the HBM half of
// the overlap masks and TextSegment.canAppend's newline test compile out, which leaves the replay
// loop fewer live registers. Same results on such batches (tests/test_gpu_c4.py).
// LVL 0: the lean instantiation (FULL = false); 1: FULL; 2: FULL + EXT, the extensions few batches use
// -- legacy catch-up delta records (MTE_F_CATCHUP) and SharedMatrix permutation runs (MTE_F_PERM) --
// kept out of the FULL kernels so they cost those no registers.
template <bool LDSM, bool SOLO = false, int LVL = 1>
struct Engine {
    static constexpr bool FULL = LVL >= 1, EXT = LVL >= 2;
    static_assert(LDSM || !SOLO, "the solo plan is LDS-resident");
    const Params& p;
    u32 doc;
    // hot per-document limits (DocCfg, engine_types.hpp)
    u32 seg_cap, arena_cap, payload_len, map_cap, mw;  // mw: words per property-map record
    u32 L;  // lane
    St st;
    bool collab, has_nl;
#ifdef MTE_PROFILE
    u64* prof;  // p.prof + doc * PROF_SLOTS (zeroed by the host before each pass)
#endif
    // HBM-resident state arrays (HBM mode); in LDS mode every array is an address in the CU's
    // LdsPlan (g_plan), a compile-time constant plus the wave's region offset.
    uint4* m_vis;  // by block id * 8 + slot
    uint4* m_aux;
    u32* m_bmeta;  // by block id: parent | needsScour << 30
    uint4* m_ord;  // doc order: (block id, observer-visible length, max seq, child count)
    u32* m_in_child;
    u32* m_in_cnt;
    u32* m_in_par;
    uint2* m_heap;
    u32* m_scratch;
    u32* m_stats;
    u32* m_hint;   // HBM mode: HBM_HINTS entries
    u32 m_blk_cap, m_ord_cap, m_in_cap, m_heap_cap;
    u32 wave;
    i32 zseq = 0;            // EXT: seq of the op being applied (UNLINK time of freed handles)
    bool continued = false;  // HBM-resident after starting in LDS
    bool from_rows = false;  // HBM-resident after starting on k_rows' row engine (DocRes mode 6)
    bool capped = false;     // HBM slot smaller than this document's worst case

#define MTE_ARR(T, NAME, MEM, LDSX, SOLOX)     \
    MTE_DEV T* NAME() const {                  \
        if constexpr (SOLO) return (T*)(SOLOX); \
        else if constexpr (LDSM) return (T*)(LDSX); \
        else return MEM;                       \
    }
    MTE_ARR(uint4, VIS, m_vis, g_plan.vis, g_solo.vis)
    MTE_ARR(uint4, AUX, m_aux, g_plan.aux, g_solo.aux)
    MTE_ARR(u32, BMETA, m_bmeta, g_plan.bmeta, g_solo.bmeta)
    MTE_ARR(uint4, ORD, m_ord, g_plan.wave[wave].ord, g_solo.w.ord)
    MTE_ARR(u32, INCH, m_in_child, g_plan.wave[wave].in_child, g_solo.w.in_child)
    MTE_ARR(u32, INCNT, m_in_cnt, g_plan.wave[wave].in_cnt, g_solo.w.in_cnt)
    MTE_ARR(u32, INPAR, m_in_par, g_plan.wave[wave].in_par, g_solo.w.in_par)
    MTE_ARR(uint2, HEAP, m_heap, g_plan.wave[wave].heap, g_solo.w.heap)
    MTE_ARR(u32, SCRATCH, m_scratch, g_plan.wave[wave].scratch, g_solo.w.scratch)
    MTE_ARR(u32, STATS, m_stats, g_plan.wave[wave].stats, g_solo.w.stats)
    MTE_ARR(mte_op, RING, nullptr, g_plan.wave[wave].ring, g_solo.w.ring)
    MTE_ARR(u16, HINT, nullptr, g_plan.wave[wave].hint, g_solo.w.hint)  // segment id -> block at push
    MTE_ARR(u32, BITMAP, nullptr, g_plan.bitmap, nullptr)               // pool allocation bitmap
    MTE_ARR(unsigned char, OWNER, nullptr, g_plan.owner, nullptr)       // pool block -> wave
    MTE_ARR(u32, POOLAV, nullptr, &g_plan.pool_avail, nullptr)          // pool blocks free of credit
#undef MTE_ARR
    // the CU's leaf blocks are shared by its waves (k_lds) rather than owned by one (k_solo, HBM)
    static constexpr bool SHARED = LDSM && !SOLO;
    // LRU heap hints (verified on use, so a stale or uninitialised entry only costs a full search)
    MTE_DEV u32 hint_get(u32 sid) const {
        if constexpr (SOLO) return HINT()[sid & (SOLO_HINTS - 1)];
        else if constexpr (LDSM) return HINT()[sid & 255];
        else return U(m_hint[sid & (HBM_HINTS - 1)]);
    }
    MTE_DEV void hint_set(u32 sid, u32 blk) const {  // per-lane store
        if constexpr (SOLO) HINT()[sid & (SOLO_HINTS - 1)] = (u16)blk;
        else if constexpr (LDSM) HINT()[sid & 255] = (u16)blk;
        else m_hint[sid & (HBM_HINTS - 1)] = blk;
    }
    MTE_DEV u32 blk_cap() const { if constexpr (SOLO) return SOLO_POOL; else if constexpr (LDSM) return POOL_BLOCKS; else return m_blk_cap; }
    MTE_DEV u32 ord_cap() const { if constexpr (SOLO) return SOLO_ORD; else if constexpr (LDSM) return ORD_CAP; else return m_ord_cap; }
    MTE_DEV u32 in_cap() const { if constexpr (SOLO) return SOLO_IN; else if constexpr (LDSM) return IN_CAP; else return m_in_cap; }
    MTE_DEV u32 heap_cap() const { if constexpr (SOLO) return SOLO_HEAP; else if constexpr (LDSM) return HEAP_CAP; else return m_heap_cap; }
    // doc-relative HBM bases
    u16* payload;
    u16* arena0;
    u64* ovl;
    u64* ovl2;  // clients 64..127 (documents whose window holds more than 64 clients), else null
    u32* maps;

    MTE_DEV Engine(const Params& p_, u32 doc_) : p(p_), doc(doc_) {
        L = lane_id();
#ifdef MTE_PROFILE
        prof = p.prof + (u64)doc_ * PROF_SLOTS;
#endif
        const DocCfg& c = p.docs[doc];
        seg_cap = c.seg_cap;
        arena_cap = c.arena_cap;
        payload_len = c.payload_len;
        map_cap = c.map_cap;
        payload = p.payload + c.payload_off;
        arena0 = p.arena + c.arena_off;
        ovl = p.ovl + c.ovl_off;
        ovl2 = (p.ovl2 && c.ovl2_off != OVL2_NONE) ? p.ovl2 + c.ovl2_off : nullptr;
        mw = p.map_words;
        maps = p.maps + c.map_off * mw;
        collab = c.collab != 0;
        has_nl = c.has_nl != 0;
        st.root = NONE;
        st.height = 1;
        st.n_lb = 0;
        st.minSeq = st.curSeq = 0;
        st.heapSize = st.segNext = st.arenaTop = st.arenaSel = 0;
        st.heapTop = 0;
        st.mapNext = 1;  // map id 0 == undefined
        st.lbFree = st.inFree = NONE;
        st.lbBump = st.inBump = st.inUsed = st.credit = 0;
        st.status = 0;
        st.adirty = st.gdirty = 0;
        wave = 0;
    }

    static constexpr u32 ST_CUOP = 7;  // doc-relative index of the MTE_F_CATCHUP op being applied
    // per-document counters kept in memory (few updates; spares scalar registers)
    MTE_DEV void stat_add(u32 i, u32 v) {
        if (L == 0) atomicAdd(&STATS()[i], v);
    }
    MTE_DEV void stat_max(u32 i, u32 v) {
        if (L == 0) atomicMax(&STATS()[i], v);
    }
    MTE_DEV u32 stat_get(u32 i) {
        sync();
        return wave_first(STATS()[i]);
    }

    MTE_DEV void bind_lds(u32 w) {
        wave = w;
        if (L < ST_WORDS) STATS()[L] = L == ST_FAILSEQ ? NONE : 0u;
        lds_order();
    }
    MTE_DEV void bind_region(unsigned char* b, u32 cb, u32 co, u32 ci, u32 ch) {
        const HbmLayout l = HbmLayout::of(cb, co, ci, ch);
        m_vis = (uint4*)(b + l.vis);
        m_aux = (uint4*)(b + l.aux);
        m_bmeta = (u32*)(b + l.bmeta);
        m_ord = (uint4*)(b + l.ord);
        m_in_child = (u32*)(b + l.in_child);
        m_in_cnt = (u32*)(b + l.in_cnt);
        m_in_par = (u32*)(b + l.in_par);
        m_heap = (uint2*)(b + l.heap);
        m_scratch = (u32*)(b + l.scratch);
        m_stats = m_scratch + 64;
        m_hint = (u32*)(b + l.hint);
        m_blk_cap = cb;
        m_ord_cap = co;
        m_in_cap = ci;
        m_heap_cap = ch;
    }
    MTE_DEV void reset_stats() {
        if (L < ST_WORDS) m_stats[L] = L == ST_FAILSEQ ? NONE : 0u;
        wave_sync();
    }
    // per-document HBM state laid out by the host (re-run of a document that failed mid-op)
    MTE_DEV void bind_hbm() {
        const DocCfg& c = p.docs[doc];
        bind_region(p.hbm + c.hb_off, c.hb_blk, c.hb_ord, c.hb_in, c.hb_heap);
        reset_stats();
    }
    // a wave's own HBM slot (Params::slot_*), reused by every document the wave takes over
    MTE_DEV void bind_slot(u32 slot) {
        bind_region(p.spill + (u64)slot * p.slot_bytes, p.slot_blk, p.slot_ord, p.slot_in, p.slot_heap);
        u32 cb, co, ci, ch;
        hbm_caps(p.docs[doc].op_end - p.docs[doc].op_begin, cb, co, ci, ch);
        capped = cb > p.slot_blk || co > p.slot_ord || ci > p.slot_in || ch > p.slot_heap;
    }
    // the HBM slot of solo document i (sized for the longest solo document)
    MTE_DEV void bind_solo_slot(u32 i) {
        bind_region(p.solo_spill + (u64)i * p.solo_slot_bytes, p.solo_blk, p.solo_ord, p.solo_in, p.solo_heap);
        u32 cb, co, ci, ch;
        hbm_caps(p.docs[doc].op_end - p.docs[doc].op_begin, cb, co, ci, ch);
        capped = cb > p.solo_blk || co > p.solo_ord || ci > p.solo_in || ch > p.solo_heap;
    }

    // Wave-uniform reads: a load from a uniform address is broadcast through readfirstlane so the
    // value (and all control flow and state updates that depend on it) stays scalar.
    MTE_DEV static u32 U(u32 v) { return wave_first(v); }
    MTE_DEV static uint4 U(uint4 v) { return make_uint4(wave_first(v.x), wave_first(v.y), wave_first(v.z), wave_first(v.w)); }
    MTE_DEV uint4 ord_u(u32 k) const { return U(ORD()[k]); }
    MTE_DEV u32 incnt_u(u32 n) const { return U(INCNT()[n]); }
    MTE_DEV u32 inpar_u(u32 n) const { return U(INPAR()[n]); }

    // Order lane-crossing hand-offs through the state arrays.
    MTE_DEV void sync() const {
        if (LDSM) lds_order();
        else wave_sync();
    }
    // Before reading HBM data that other lanes wrote (merge-arena text, overlap masks).
    MTE_DEV void fence_arena() {
        if (st.adirty) {
            wave_sync();
            st.adirty = 0;
        }
    }
    MTE_DEV void fence_ovl() {
        if (st.gdirty) {
            wave_sync();
            st.gdirty = 0;
        }
    }

    // ---------------------------------------------------------------- errors
    MTE_DEV void fail(i32 code, i32 seq) {
        if (st.status == 0) {
            st.status = code;
            if (L == 0) STATS()[ST_FAILSEQ] = (u32)seq;
        }
    }

    // ---------------------------------------------------------------- slots
    // Slot index with the block clamped into the pool (ids are validated where they are produced;
    // the clamp keeps a corrupted id from ever addressing outside the state arrays).
    MTE_DEV u32 sidx(u32 blk, u32 s) const { return (blk < blk_cap() ? blk : 0u) * 8 + (s & 7); }
    MTE_DEV Seg load(u32 blk, u32 s) const {
        Seg g;
        const u32 i = sidx(blk, s);
        uint4 v = VIS()[i], a = AUX()[i];
        g.len = v.x;
        g.seq = (i32)v.y;
        g.rseq = (i32)v.z;
        g.meta = v.w;
        g.props = a.x;
        g.toff = a.y;
        g.tcap = a.z;
        g.sid = a.w;
        return g;
    }
    MTE_DEV Seg load_u(u32 blk, u32 s) const {  // a slot at a uniform address, as scalars
        Seg g = load(blk, s);
        g.len = U(g.len);
        g.seq = (i32)U((u32)g.seq);
        g.rseq = (i32)U((u32)g.rseq);
        g.meta = U(g.meta);
        g.props = U(g.props);
        g.toff = U(g.toff);
        g.tcap = U(g.tcap);
        g.sid = U(g.sid);
        return g;
    }
    MTE_DEV void store(u32 blk, u32 s, const Seg& g) const {
        const u32 i = sidx(blk, s);
        VIS()[i] = make_uint4(g.len, (u32)g.seq, (u32)g.rseq, g.meta);
        AUX()[i] = make_uint4(g.props, g.toff, g.tcap, g.sid);
    }
    MTE_DEV Seg shfl_seg(const Seg& r, u32 src) const {
        Seg o;
        o.len = wave_shfl(r.len, src);
        o.seq = wave_shfl(r.seq, src);
        o.rseq = wave_shfl(r.rseq, src);
        o.meta = wave_shfl(r.meta, src);
        o.props = wave_shfl(r.props, src);
        o.toff = wave_shfl(r.toff, src);
        o.tcap = wave_shfl(r.tcap, src);
        o.sid = wave_shfl(r.sid, src);
        return o;
    }
    MTE_DEV static u32 client_of(u32 meta) { return meta & 0xff; }
    MTE_DEV static u32 rclient_of(u32 meta) { return (meta >> 8) & 0xff; }
    MTE_DEV static u32 obs_len(u32 len, u32 meta) { return (meta & F_REMOVED) ? 0u : len; }
    MTE_DEV static i32 seq_hi(i32 seq, i32 rseq, u32 meta) { return (meta & F_REMOVED) && rseq > seq ? rseq : seq; }

    // block metadata
    MTE_DEV u32 bpar(u32 b) const {
        if (b >= blk_cap()) return NONE;
        u32 x = U(BMETA()[b]) & BM_PAR;
        return x == BM_NOPAR ? NONE : x;
    }
    MTE_DEV u32 bscour(u32 b) const { return b < blk_cap() ? U(BMETA()[b]) >> 30 : SC_UNDEF; }
    // the whole metadata word (parent | needsScour), for a read-modify-write with one read
    MTE_DEV u32 bmeta_u(u32 b) const { return b < blk_cap() ? U(BMETA()[b]) : (BM_NOPAR | (SC_UNDEF << 30)); }
    MTE_DEV static u32 par_of_word(u32 w) { return (w & BM_PAR) == BM_NOPAR ? NONE : (w & BM_PAR); }
    MTE_DEV void set_bscour_w(u32 b, u32 w, u32 sc) const {  // w: the block's current metadata word
        if (L == 0 && b < blk_cap()) BMETA()[b] = (w & BM_PAR) | (sc << 30);
    }
    MTE_DEV void set_bpar_lane(u32 b, u32 par) const {  // per-lane write
        if (b < blk_cap()) BMETA()[b] = (BMETA()[b] & ~BM_PAR) | (par == NONE ? BM_NOPAR : (par & BM_PAR));
    }
    MTE_DEV void set_bscour(u32 b, u32 sc) const {
        if (L == 0 && b < blk_cap()) BMETA()[b] = (BMETA()[b] & BM_PAR) | (sc << 30);
    }

    // Visible length of a slot for (refSeq R, client C): nodeLength for a leaf
    // (mergeTree.ts:1659-1699) in branch-free 32-bit integer arithmetic:
    //   ins = client == C || seq <= R;  rem = removed && (rclient == C || rseq <= R || C in overlap)
    //   len if ins && !rem, else 0.
    // z = the slot's aux.z (the overlap mask of clients 0..31 once removed). cz: C == 0, the
    // observer / local client (localNetLength, :1161-1172) for whom every seq is <= R.
    MTE_DEV static u32 le1(i32 a, i32 b) { return (u32)~(b - a) >> 31; }  // a <= b (|b - a| < 2^31)
    MTE_DEV static u32 eq1(u32 a, u32 b) { return ((a ^ b) - 1u) >> 31; }   // a == b (a, b < 2^31)
    MTE_DEV u32 vis_len(uint4 q, u32 z, u32 idx, i32 R, u32 C, u32 cz) const {
        const u32 meta = q.w;
        const u32 rm = (meta >> 16) & 1u;  // F_REMOVED
        const u32 ins = eq1(meta & 0xffu, C) | le1((i32)q.y, R) | cz;
        u32 ovh;
        if (!FULL || C < 32) {
            ovh = (z >> C) & 1u;
        } else {  // clients 32..63: HBM half of the mask (rare)
            ovh = 0;
            if ((meta & (F_REMOVED | F_OVLHI)) == (F_REMOVED | F_OVLHI)) ovh = ovl_hides(idx, C, meta) ? 1u : 0u;
        }
        ovh &= (meta >> 18) & 1u;  // F_OVL
        const u32 rem = rm & (eq1((meta >> 8) & 0xffu, C) | le1((i32)q.z, R) | cz | ovh);
        return q.x & (0u - (ins & (rem ^ 1u)));
    }
    // C among the overlapping removers (removedClientOverlap, mergeTree.ts:2544-2552): clients
    // 0..31 in the removed slot's aux.z (its arena-capacity word is dead once removed), 32..63 in
    // the document's HBM mask by segment id, 64..127 in its second HBM mask (F_OVLHI: both words
    // valid).
    MTE_DEV bool ovl_hides(u32 idx, u32 C, u32 meta) const {
        if (C < 32) return (AUX()[idx].z >> C) & 1u;
        if (!(meta & F_OVLHI)) return false;
        const u32 sid = AUX()[idx].w;
        if (sid >= seg_cap) return false;
        if (C < 64) return (ovl[sid] >> C) & 1ull;
        return ovl2 && ((ovl2[sid] >> (C - 64)) & 1ull);
    }
    // breakTie for a zero-visible leaf at pos 0: skip tombstones already seen at R (mergeTree.ts:2257-2261)
    MTE_DEV static u32 tie_ok(uint4 q, i32 R, u32 cz) {
        const u32 seen = ((q.w >> 16) & 1u) & (((u32)(i32)q.z != 0u) ? 1u : 0u) & le1((i32)q.z, R);
        return cz | (seen ^ 1u);
    }
    // Visible lengths of the leaf blocks held one per lane (ord entries) for (R, C). A block whose
    // children are all settled at R (max seq <= R) has the same length for every client; the others
    // read their slots (independent LDS reads) and evaluate the predicate. C != 0 there (the
    // observer sees every block settled), so the writer form below applies; the overlap masks
    // (aux.z) are read only when some slot of the batch carries one.
    MTE_DEV static u32 vis_w(uint4 q, u32 z, i32 R, u32 C) {  // nodeLength for a writer C in 1..31
        const u32 meta = q.w;
        const bool ins = ((meta & 0xffu) == C) | ((i32)q.y <= R);
        const bool ovh = (((z >> C) & 1u) != 0) & ((meta & F_OVL) != 0);
        const bool rem = ((meta & F_REMOVED) != 0) & ((((meta >> 8) & 0xffu) == C) | ((i32)q.z <= R) | ovh);
        return (ins & !rem) ? q.x : 0u;
    }
    // The dirty blocks (max seq > R) are evaluated slot by slot, lane = slot: up to 8 blocks per
    // pass, lanes 8g..8g+7 holding the slots of the g-th dirty block of the batch; each block's sum
    // goes back to the lane that holds it (mbcnt rank -> bpermute from its group's last lane).
    MTE_DEV u32 blen_all(uint4 o, bool valid, i32 R, u32 C) const {
        const u32 cz = C == 0 ? 1u : 0u;
        const bool fast = !valid | (cz != 0) | ((i32)o.z <= R);
        u32 v = valid ? o.y : 0u;
        const u64 dm = wave_ballot(!fast);
        if (dm) {
            MTE_PROF(PF_BLEN_DIRTY);
            if (!(dm & (dm - 1))) {
                // one dirty block (the common case): lane = slot, one conflict-free LDS read per lane
                // instead of every lane reading 8 slots of its own block (the 128-B block stride
                // puts all 64 lanes on 2 bank groups)
                const u32 j = (u32)__builtin_ctzll(dm);
                const u32 bj = wave_read(o.x, j), cj = wave_read(o.w, j);
                const u32 bb = bj < blk_cap() ? bj : 0u;
                const u32 s = L & 7u;
                const u32 idx = bb * 8 + s;
                const uint4 q1 = VIS()[idx];
                const u32 z1 = AUX()[idx].z;
                const u32 sv1 = (L < 8 && s < cj) ? vis_len(q1, z1, idx, R, C, cz) : 0u;
                const u32 tot = wave_read(group8_scan(sv1), 7);
                return L == j ? tot : v;
            }
            const u32 b = o.x < blk_cap() ? o.x : 0u;
            u32 sv = 0;
            if (FULL && C >= 32) {  // clients 32..63: the general predicate (HBM half of the overlap mask)
                for (u32 s = 0; s < 8; s++)
                    sv += s < o.w ? vis_len(VIS()[b * 8 + s], AUX()[b * 8 + s].z, b * 8 + s, R, C, cz) : 0u;
            } else {
                // two halves of four independent LDS reads: half the live registers of eight at once
                // (k_lds sits at its 128-VGPR bound: 116 -> 56 spilled bytes per lane, C2 -5 %); the
                // overlap mask is read only for a slot that has one
#pragma unroll
                for (u32 h = 0; h < 2; h++) {
                    uint4 q4[4];
#pragma unroll
                    for (u32 s = 0; s < 4; s++) q4[s] = VIS()[b * 8 + 4 * h + s];
#pragma unroll
                    for (u32 s = 0; s < 4; s++) {
                        const bool ov = (q4[s].w & F_OVL) != 0;
                        sv += 4 * h + s < o.w ? vis_w(q4[s], ov ? AUX()[b * 8 + 4 * h + s].z : 0u, R, C) : 0u;
                    }
                }
            }
            v = fast ? v : sv;
        }
        return v;
    }

    // Recompute (visible length, max seq) of ORD()[k0 .. k0+n), n <= 8, from the slots.
    MTE_DEV void refresh(u32 k0, u32 n) {
        const u32 g = L >> 3, s = L & 7;
        const bool act = g < n;
        uint4 o = act ? ORD()[k0 + g] : make_uint4(0, 0, 0, 0);
        u32 len = 0;
        i32 mx = 0;
        if (act && s < o.w && o.x < blk_cap()) {
            uint4 v = VIS()[o.x * 8 + s];
            len = obs_len(v.x, v.w);
            mx = seq_hi((i32)v.y, (i32)v.z, v.w);
        }
        u32 tl = group8_scan(len);
        i32 tm = group8_max(mx);
        sync();
        if (act && s == 7) {
            ORD()[k0 + g].y = tl;
            ORD()[k0 + g].z = (u32)tm;
        }
        sync();
    }

    // ---------------------------------------------------------------- position resolution
    MTE_DEV Found resolve(i32 pos, i32 R, u32 C) {
        MTE_PROF(PF_RESOLVE);
        Found f;
        f.ok = false;
        f.k = 0;
        f.blk = NONE;
        f.cnt = 0;
        f.slot = -1;
        f.r = 0;
        f.cum = 0;
        fence_ovl();
        i32 cum = 0;
#ifdef MTE_PROFILE
        MTE_PROF(PF_RES_BLOCKS);
#endif
        for (u32 base = 0; base < st.n_lb; base += 64) {
            const u32 k = base + L;
            const bool valid = k < st.n_lb;
            uint4 o = valid ? ORD()[k] : make_uint4(0, 0, 0, 0);
            const u32 v = blen_all(o, valid, R, C);
            MTE_COUNT(PN_DIRTY, __builtin_popcountll(wave_ballot(valid && !(C == 0 || (i32)o.z <= R))));
            MTE_COUNT(PN_RESOLVE, 1);
            u32 incl = wave_scan_incl(v);
            u64 hit = wave_ballot(valid && cum + (i32)incl >= pos);
            if (hit) {
                u32 j = (u32)__builtin_ctzll(hit);
                f.ok = true;
                f.k = base + j;
                f.blk = wave_read(o.x, j);
                f.cnt = wave_read(o.w, j);
                f.cum = cum + (i32)wave_read(incl - v, j);
                break;
            }
            cum += (i32)wave_read(incl, 63);
        }
        if (!f.ok) return f;
        resolve_slot(f, pos, R, C);
        return f;
    }
    // The block of `pos` from one block scan already held per lane (lane = doc-order index, n_lb <= 64:
    // o, its visible length v and the inclusive prefix incl), then the slot inside it. The block's child
    // count is re-read (a split since the scan may have added a slot; block splits invalidate the scan).
    // The fused scan's per-lane block lengths: kept in registers by k_solo (no register budget), in the
    // wave's scratch words by the budgeted kernels, whose registers it would otherwise hold across the
    // split phases (lean k_lds: 42 -> 67 spilled VGPRs in registers)
    static constexpr bool PRE_REGS = SOLO;
    MTE_DEV void pre_put(u32 v) {
        if constexpr (!PRE_REGS) {
            sync();
            SCRATCH()[L] = v;
            sync();
        }
    }
    MTE_DEV void pre_get(u32& v, u32& incl) {
        if constexpr (!PRE_REGS) {
            v = SCRATCH()[L];
            incl = wave_scan_incl(v);
        }
    }
    MTE_DEV Found resolve_pre(u32 v, u32 incl, i32 pos, i32 R, u32 C) {
        pre_get(v, incl);
        Found f;
        f.ok = false;
        f.k = 0;
        f.blk = NONE;
        f.cnt = 0;
        f.slot = -1;
        f.r = 0;
        f.cum = 0;
        fence_ovl();
        const u64 hit = wave_ballot(L < st.n_lb && (i32)incl >= pos);
        if (!hit) return f;
        const u32 j = (u32)__builtin_ctzll(hit);
        f.ok = true;
        f.k = j;
        const uint4 oj = ord_u(j);  // the block id, and its child count after any split since the scan
        f.blk = oj.x;
        f.cnt = oj.w;
        f.cum = (i32)wave_read(incl - v, j);
        resolve_slot(f, pos, R, C);
        return f;
    }
    MTE_DEV void resolve_slot(Found& f, i32 pos, i32 R, u32 C) {
        MTE_PROF(PF_RES_SLOT);
        // inside the block: first slot with r < vislen, or a zero-visible slot at r == 0 that wins breakTie
        const u32 s = L;
        const u32 idx = sidx(f.blk, s);
        const uint4 q = VIS()[idx];
        const u32 z = AUX()[idx].z;
        const bool in = s < f.cnt && s < 8;
        const u32 cz = C == 0 ? 1u : 0u;
        const u32 v = in ? vis_len(q, z, idx, R, C, cz) : 0u;
        const bool tie = tie_ok(q, R, cz) != 0;
        const u32 incl = group8_scan(v);
        const i32 r = pos - (f.cum + (i32)(incl - v));
        const bool cand = in & ((r < (i32)v) | ((r == 0) & (v == 0) & tie));
        u64 m2 = wave_ballot(cand);
        if (m2) {
            u32 l2 = (u32)__builtin_ctzll(m2);
            f.slot = (i32)l2;
            f.r = wave_read(r, l2);
        }
    }

    MTE_DEV i32 get_length(i32 R, u32 C) {  // MergeTree.getLength (mergeTree.ts:1577-1579)
        fence_ovl();
        i32 cum = 0;
        for (u32 base = 0; base < st.n_lb; base += 64) {
            const u32 k = base + L;
            const bool valid = k < st.n_lb;
            const uint4 o = valid ? ORD()[k] : make_uint4(0, 0, 0, 0);
            cum += (i32)wave_sum(blen_all(o, valid, R, C));
        }
        return cum;
    }

    // posFromRelativePos (mergeTree.ts:1943-1966) for the op's RELPOS record (include/mte.h): the
    // marker is found by its builder tag (bits 16..31 of its refType word, aux.y) and
    // getPosition(marker, R, C) (mergeTree.ts:1586-1603) is the visible length before it in document
    // order. An unmapped tag fails the document (unsupported). A tagged marker no longer in the tree
    // was dropped by zamboni, which unlinks it (scourNode: parent = undefined, mergeTree.ts:1317): the
    // reference's parent walk is then empty, getPosition 0.
    MTE_DEV bool marker_pos(u32 tag, i32 R, u32 C, i32 seq, i32& out) {
        if (tag == 0 || tag > 0xFFFFu) {
            fail(MTE_DOC_UNSUPPORTED, seq);
            return false;
        }
        fence_ovl();
        u32 k = NONE, s = 0;
        for (u32 base = 0; base < st.n_lb; base += 8) {
            const u32 kk = base + (L >> 3), sl = L & 7;
            const uint4 o = kk < st.n_lb ? ORD()[kk] : make_uint4(NONE, 0, 0, 0);
            const u32 idx = sidx(o.x, sl);
            const bool hit = kk < st.n_lb && sl < o.w && (VIS()[idx].w & F_MARKER) != 0 && (AUX()[idx].y >> 16) == tag;
            const u64 m = wave_ballot(hit);
            if (m) {
                const u32 l = (u32)__builtin_ctzll(m);
                k = base + (l >> 3);
                s = l & 7;
                break;
            }
        }
        if (k == NONE) {  // unlinked by zamboni
            out = 0;
            return true;
        }
        i32 cum = 0;
        for (u32 base = 0; base < k; base += 64) {
            const u32 kk = base + L;
            const bool valid = kk < k;
            const uint4 o = valid ? ORD()[kk] : make_uint4(0, 0, 0, 0);
            cum += (i32)wave_sum(blen_all(o, valid, R, C));
        }
        const u32 blk = wave_first(ORD()[k].x);
        const u32 idx = sidx(blk, L);
        const u32 cz = C == 0 ? 1u : 0u;
        const u32 v = L < s ? vis_len(VIS()[idx], AUX()[idx].z, idx, R, C, cz) : 0u;
        out = cum + (i32)wave_sum(v);
        return true;
    }
    MTE_DEV bool rel_positions(mte_op& op, u64 i, i32 R, u32 C) {
        if (i <= p.docs[doc].op_begin) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return false;
        }
        const mte_op rr = read_op(p.ops + i - 1);
        if (rr.type != MTE_OP_RELPOS) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return false;
        }
        i32 q;
        if (rr.pos1) {
            if (!marker_pos((u32)rr.pos1, R, C, op.seq, q)) return false;
            op.pos1 = (rr.flags & MTE_F_REL_BEFORE1) ? q - rr.msn : q + 1 + rr.msn;  // Marker cachedLength 1
        }
        if (rr.a) {
            if (!marker_pos((u32)rr.a, R, C, op.seq, q)) return false;
            op.a = (rr.flags & MTE_F_REL_BEFORE2) ? q - (i32)rr.props : q + 1 + (i32)rr.props;
        }
        // a position before 0 (an unlinked marker, "before" with an offset): not modelled (the
        // reference's walks then run below the tree's start)
        if ((rr.pos1 && op.pos1 < 0) || (rr.a && op.a < 0)) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return false;
        }
        return true;
    }

    // ---------------------------------------------------------------- SharedMatrix cell ops
    // getContainingSegment (mergeTree.ts:1623-1634 -> searchBlock :1797-1829): the first segment whose
    // visible length in the (R, C) view exceeds the remaining position. f.slot / f.r: the segment and
    // the offset in it; !f.ok when pos is beyond the view's length.
    MTE_DEV Found contain(i32 pos, i32 R, u32 C) {
        Found f;
        f.ok = false;
        f.k = 0;
        f.blk = NONE;
        f.cnt = 0;
        f.slot = -1;
        f.r = 0;
        f.cum = 0;
        if (pos < 0) return f;
        fence_ovl();
        i32 cum = 0;
        for (u32 base = 0; base < st.n_lb; base += 64) {
            const u32 k = base + L;
            const bool valid = k < st.n_lb;
            const uint4 o = valid ? ORD()[k] : make_uint4(0, 0, 0, 0);
            const u32 v = blen_all(o, valid, R, C);
            const u32 incl = wave_scan_incl(v);
            const u64 hit = wave_ballot(valid && cum + (i32)incl > pos);
            if (hit) {
                const u32 j = (u32)__builtin_ctzll(hit);
                f.k = base + j;
                f.blk = wave_read(o.x, j);
                f.cnt = wave_read(o.w, j);
                f.cum = cum + (i32)wave_read(incl - v, j);
                const u32 idx = sidx(f.blk, L);
                const bool in = L < f.cnt && L < 8;
                const u32 sv = in ? vis_len(VIS()[idx], AUX()[idx].z, idx, R, C, C == 0 ? 1u : 0u) : 0u;
                const u32 si = group8_scan(sv);
                const i32 r = pos - (f.cum + (i32)(si - sv));
                const u64 m = wave_ballot(in && r >= 0 && r < (i32)sv);
                if (m) {
                    f.ok = true;
                    f.slot = (i32)__builtin_ctzll(m);
                    f.r = wave_read(r, (u32)f.slot);
                }
                return f;
            }
            cum += (i32)wave_read(incl, 63);
        }
        return f;
    }
    // PermutationVector.adjustPosition (permutationvector.ts:198-209): the containing segment in the
    // op's view; undefined (-1) when there is none or it is removed (removedSeq set, whatever its
    // seq), else its position in the local view (getPosition at currentSeq, mergeTree.ts:1586-1603)
    // plus the offset.
    MTE_DEV i32 cell_adjust(i32 pos, i32 R, u32 C) {
        const Found f = contain(pos, R, C);
        if (!f.ok) return -1;
        const u32 meta = wave_first(VIS()[sidx(f.blk, (u32)f.slot)].w);
        if (meta & F_REMOVED) return -1;
        return obs_prefix(f.k, f.blk, (u32)f.slot) + f.r;
    }
    // HandleTable (handletable.ts:19-86) of this vector in HBM: ht[0] = the handles array's length,
    // ht[1 + i] = handles[i] (handles[0] = the free-list head), ht[1 + cap + i] = the seq of the op
    // whose zamboni last freed handle i (0 = never). Lane 0 owns it; results are broadcast.
    MTE_DEV u32* ht_base() const { return p.htab + p.docs[doc].ht_off; }
    MTE_DEV void ht_reset() {  // new HandleTable(): [1], or HandleTable.load of a matrix summary (htab0)
        const u32 cap = p.docs[doc].ht_cap;
        if (!cap || !p.htab || !p.htab0) return;
        u32* ht = ht_base();
        const u32* h0 = p.htab0 + p.docs[doc].ht_off;
        for (u32 i = L; i < 1 + 2 * cap; i += 64) ht[i] = h0[i];
        wave_sync();
    }
    MTE_DEV u32 ht_alloc() {  // HandleTable.allocate (handletable.ts:35-40)
        const u32 cap = p.docs[doc].ht_cap;
        u32 h = NONE;
        if (L == 0 && cap && p.htab) {
            u32* ht = ht_base();
            const u32 len = ht[0], fr = ht[1];
            if (fr >= 1 && fr < cap && fr <= len) {
                ht[1] = fr < len ? ht[1 + fr] : fr + 1;  // handles[free] ?? free + 1
                ht[1 + fr] = 0;
                if (fr == len) ht[0] = len + 1;
                h = fr;
            }
        }
        h = wave_read(h, 0);
        if (h == NONE) fail(MTE_DOC_CAPACITY, st.curSeq);
        return h;
    }
    MTE_DEV void ht_free(u32 h0, u32 n) {  // HandleTable.free (:56-59) of h0 .. h0 + n - 1
        const u32 cap = p.docs[doc].ht_cap;
        bool bad = false;
        if (L == 0) {
            u32* ht = ht_base();
            for (u32 i = 0; i < n; i++) {
                const u32 h = h0 + i;
                if (h >= cap) {
                    bad = true;
                    break;
                }
                ht[1 + h] = ht[1];
                ht[1] = h;
                ht[1 + cap + h] = (u32)zseq;
            }
        }
        if (wave_ballot(bad)) fail(MTE_DOC_CAPACITY, st.curSeq);
        wave_sync();
    }
    // getAllocatedHandle (permutationvector.ts:176-196) at local position pos: the segment's handle
    // when allocated, else walkSegments(pos, pos + 1, splitRange) -- ensureIntervalBoundary at pos
    // and pos + 1 in the local view (mergeTree.ts:2797-2807, 2241-2245) -- and the new length-1
    // segment takes the next handle.
    MTE_DEV u32 cell_handle(i32 pos, i32 seq) {
        const i32 R = st.curSeq;
        Found f = contain(pos, R, 0);
        if (!f.ok) {
            fail(MTE_DOC_CAPACITY, seq);
            return 0;
        }
        const u32 toff = wave_first(AUX()[sidx(f.blk, (u32)f.slot)].y);
        if (toff) return toff + (u32)f.r;
        Seg none;
        none.len = 0;
        edit(MTE_OP_CELL, pos, pos + 1, R, 0, seq, none, 0, false, false);
        if (st.status) return 0;
        f = contain(pos, R, 0);
        if (!f.ok || f.r != 0) {
            fail(MTE_DOC_CAPACITY, seq);
            return 0;
        }
        const u32 h = ht_alloc();
        if (st.status) return 0;
        sync();
        if (L == 0) AUX()[sidx(f.blk, (u32)f.slot)].y = h;
        sync();
        return h;
    }
    // SharedMatrix.processCore's remote set (matrix.ts:575-601) as this vector sees it: pass 1 records
    // adjustPosition; pass 2 allocates when both vectors' positions were defined (the row's gates the
    // column's, and both gate the handles).
    MTE_DEV void cell_op(const mte_op& op, i32 R, u32 C) {
        const u32 g = op.b, w = (op.flags & MTE_F_CELL_COL) ? 1u : 0u;
        if (!p.cell_pos || !p.cell_h) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        if (p.cell_mode == 1) {
            const i32 a = cell_adjust(op.pos1, R, C);
            if (L == 0) p.cell_pos[2 * (u64)g + w] = a < 0 ? NONE : (u32)a;
            return;
        }
        const u32 pr = wave_first(p.cell_pos[2 * (u64)g]), pc = wave_first(p.cell_pos[2 * (u64)g + 1]);
        u32 h = 0;
        if (pr != NONE && pc != NONE) h = cell_handle((i32)(w ? pc : pr), op.seq);
        if (L == 0) p.cell_h[2 * (u64)g + w] = h;
    }

    // ---------------------------------------------------------------- legacy catch-up delta ranges
    // SnapshotLegacy's catch-up rewrite (sequence.ts:597-634) rebuilds an MTE_F_CATCHUP message's
    // contents from its sequenceDelta ranges: each delta segment at client.getPosition(segment)
    // (sequenceDeltaEvent.ts:26-46 -> mergeTree.ts:1586-1603), the local (observer) view, in which
    // nodeLength is the segment's length unless removed -- the op itself included.
    MTE_DEV i32 obs_prefix(u32 k, u32 blk, u32 s) {
        sync();
        u32 cum = 0;
        for (u32 base = 0; base < k; base += 64) {
            const u32 kk = base + L;
            cum += wave_sum(kk < k ? ORD()[kk].y : 0u);
        }
        const uint4 q = VIS()[sidx(blk, L)];
        cum += wave_sum(L < s && L < 8 ? obs_len(q.x, q.w) : 0u);
        return (i32)cum;
    }
    MTE_DEV void cu_record(u32 kind, i32 pos, u32 len, u32 nmap, u32 omap) {
        const u32 n = stat_get(ST_CU), op = stat_get(ST_CUOP);
        const DocCfg& c = p.docs[doc];
        if (n >= c.cu_cap || !p.cu_rec) {
            fail(MTE_DOC_CAPACITY, st.curSeq);
            return;
        }
        if (L == 0) {
            uint4* r = p.cu_rec + (c.cu_off + n) * 2;
            r[0] = make_uint4(op, (u32)pos, len, kind);
            r[1] = make_uint4(nmap, omap, 0, 0);
            STATS()[ST_CU] = n + 1;
        }
        sync();
    }

    // ---------------------------------------------------------------- allocation
    // Out of room: in LDS mode the document leaves the LDS plan (DOC_SPILL: its LDS state is
    // dropped and the host re-runs it HBM-resident); in HBM mode it is a capacity failure.
    // Out of room: LDS plan or an HBM slot smaller than the document's worst case -> DOC_SPILL
    // (the host re-runs it with worst-case capacities); a worst-case region -> capacity error.
    MTE_DEV void fail_cap() {
        if (LDSM || capped) fail(DOC_SPILL, st.curSeq);
        else fail(MTE_DOC_CAPACITY, st.curSeq);
    }

    // Take credit from the CU's pool: `want` blocks if available, at least `need`.
    MTE_DEV bool take_credit(u32 need, u32 want) {
        u32 got = 0;
        if (L == 0) {
            u32 cur = __atomic_load_n(POOLAV(), __ATOMIC_RELAXED);
            for (;;) {
                const u32 w = want < cur ? want : cur;
                if (w < need) {
                    got = NONE;
                    break;
                }
                const u32 prev = atomicCAS(POOLAV(), cur, cur - w);
                if (prev == cur) {
                    got = w;
                    break;
                }
                cur = prev;
            }
        }
        got = wave_read(got, 0);
        if (got == NONE) return false;
        st.credit += got;
        return true;
    }
    // Room for one more op while LDS-resident (per-wave caps with margins, OP_CREDIT leaf blocks
    // in hand); false => the document continues HBM-resident from this op.
    MTE_DEV bool room() {
        if (!LDSM) return true;
        if (st.n_lb + 16 > ord_cap() || st.inUsed + 12 > in_cap() || st.heapSize + st.n_lb + 8 > heap_cap())
            return false;
        if (SOLO) return st.lbFree != NONE || st.lbBump + OP_CREDIT <= blk_cap();
        if (st.credit >= OP_CREDIT) return true;
        return take_credit(OP_CREDIT - st.credit, 2 * OP_CREDIT - st.credit);
    }

    MTE_DEV u32 alloc_lb() {
        MTE_PROF(PF_ALLOC);
        u32 id = NONE;
        if (SHARED) {
            if (st.credit == 0) {
                // mid-op and the CU's pool is dry: the other waves return blocks as their scours,
                // packs and documents complete, so wait (bounded) rather than abandon the replay
                bool ok = take_credit(1, 1);
                for (u32 spin = 0; !ok && spin < 20000; spin++) {
                    __builtin_amdgcn_s_sleep(4);
                    ok = take_credit(1, 1);
                }
                if (!ok) {
                    fail_cap();
                    return NONE;
                }
            }
            // claim a free bit of the CU's pool bitmap (other waves claim concurrently)
            for (int guard = 0; guard < 64; guard++) {
                u32 w = L < 16 ? BITMAP()[L] : 0xFFFFFFFFu;
                u64 m = wave_ballot(w != 0xFFFFFFFFu);
                if (!m) break;
                u32 wl = (u32)__builtin_ctzll(m);
                u32 word = wave_read(w, wl);
                u32 bit = (u32)__builtin_ctz(~word);
                u32 old = 0;
                if (L == 0) old = atomicOr(&BITMAP()[wl], 1u << bit);
                old = wave_read(old, 0);
                if (!(old & (1u << bit))) {
                    id = wl * 32 + bit;
                    break;
                }
            }
            if (id == NONE || id >= blk_cap()) {
                fail_cap();
                return NONE;
            }
            st.credit--;
            if (L == 0) OWNER()[id] = (unsigned char)wave;
        } else {
            if (st.lbFree != NONE) {
                id = st.lbFree;
                u32 nx = U(BMETA()[id]) & BM_PAR;
                st.lbFree = nx == BM_NOPAR ? NONE : nx;
            } else if (st.lbBump < blk_cap()) {
                id = st.lbBump++;
            } else {
                fail_cap();
                return NONE;
            }
        }
        id = U(id);
        sync();
        if (L == 0) BMETA()[id] = BM_NOPAR | (SC_UNDEF << 30);
        sync();
        return id;
    }
    MTE_DEV void free_lb(u32 id) {
        if (id >= blk_cap()) return;
        if (SHARED) {
            if (L == 0) {
                OWNER()[id] = 0xFF;
                atomicAnd(&BITMAP()[id >> 5], ~(1u << (id & 31)));
            }
            st.credit++;
            if (st.credit >= 2 * OP_CREDIT) {  // hand surplus back: no hoarding across the CU's waves
                if (L == 0) atomicAdd(POOLAV(), st.credit - OP_CREDIT);
                st.credit = OP_CREDIT;
            }
        } else {
            if (L == 0) BMETA()[id] = st.lbFree == NONE ? BM_NOPAR : st.lbFree;
            st.lbFree = id;
        }
        sync();
    }
    MTE_DEV u32 alloc_in() {
        u32 id = NONE;
        if (st.inFree != NONE) {
            id = st.inFree;
            st.inFree = inpar_u(id);
        } else if (st.inBump < in_cap()) {
            id = st.inBump++;
        } else {
            fail_cap();
            return NONE;
        }
        st.inUsed++;
        sync();
        if (L == 0) {
            INCNT()[id] = 0;
            INPAR()[id] = NONE;
        }
        sync();
        return id;
    }
    MTE_DEV void free_in(u32 id) {
        if (id >= in_cap()) return;
        if (L == 0) INPAR()[id] = st.inFree;
        st.inFree = id;
        st.inUsed--;
        sync();
    }
    MTE_DEV u32 new_sid() {
        if (st.segNext >= seg_cap) {
            fail(MTE_DOC_CAPACITY, st.curSeq);
            return NONE;
        }
        return st.segNext++;
    }

    // ---------------------------------------------------------------- doc-order block list
    MTE_DEV void ord_shift_right(u32 from, u32 d) {  // ORD()[from..n_lb) -> ORD()[from+d..)
        for (i32 end = (i32)st.n_lb; end > (i32)from; end -= 64) {
            i32 start = end - 64 < (i32)from ? (i32)from : end - 64;
            i32 idx = start + (i32)L;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (idx < end) v = ORD()[idx];
            sync();
            if (idx < end) ORD()[idx + d] = v;
            sync();
        }
    }
    MTE_DEV void ord_shift_left(u32 from, u32 d) {  // ORD()[from..n_lb) -> ORD()[from-d..)
        for (u32 start = from; start < st.n_lb; start += 64) {
            u32 idx = start + L;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (idx < st.n_lb) v = ORD()[idx];
            sync();
            if (idx < st.n_lb) ORD()[idx - d] = v;
            sync();
        }
    }
    MTE_DEV u32 ord_find(u32 blk) const {
        for (u32 base = 0; base < st.n_lb; base += 64) {
            u32 idx = base + L;
            u64 m = wave_ballot(idx < st.n_lb && ORD()[idx].x == blk);
            if (m) return base + (u32)__builtin_ctzll(m);
        }
        return NONE;
    }
    // Current leaf block of segment `sid` (the LRU heap entry's segment.parent), NONE if unlinked.
    MTE_DEV bool find_seg(u32 sid, u32& k, u32& blk, u32& cnt, u32& bm) {
        MTE_PROF(PF_FIND_SEG);
        {  // the block recorded at push time (kept current by splits and packs): its slots, its
           // metadata word and the doc-order entry holding it are independent reads
            const u32 hb = hint_get(sid);
            const u32 hs = AUX()[sidx(hb, L)].w;
            const u32 hw = BMETA()[hb < blk_cap() ? hb : 0u];
            u32 kk = NONE, c = 0;
            for (u32 base = 0; base < st.n_lb; base += 64) {
                const u32 idx = base + L;
                const uint4 o = idx < st.n_lb ? ORD()[idx] : make_uint4(NONE, 0, 0, 0);
                const u64 m = wave_ballot(idx < st.n_lb && o.x == hb);
                if (m) {
                    const u32 j = (u32)__builtin_ctzll(m);
                    kk = base + j;
                    c = wave_read(o.w, j);
                    break;
                }
            }
            if (kk != NONE) {
                const u64 m = wave_ballot((L < c) & (L < 8) & (hs == sid));
                if (m) {
                    k = kk;
                    blk = hb;
                    cnt = c;
                    bm = U(hw);
                    return true;
                }
            }
        }
        for (u32 base = 0; base < st.n_lb; base += 8) {
            const u32 kk = base + (L >> 3), s = L & 7;
            uint4 o = kk < st.n_lb ? ORD()[kk] : make_uint4(NONE, 0, 0, 0);
            const bool hit = (kk < st.n_lb) & (s < o.w) & (AUX()[sidx(o.x, s)].w == sid);
            u64 m = wave_ballot(hit);
            if (m) {
                u32 l = (u32)__builtin_ctzll(m);
                k = base + (l >> 3);
                blk = wave_read(o.x, l);
                cnt = wave_read(o.w, l);
                bm = bmeta_u(blk);
                return true;
            }
        }
        return false;
    }

    // ---------------------------------------------------------------- tree structure
    MTE_DEV u32 parent_of(u32 node, u32 lvl) const { return lvl == 0 ? bpar(node) : (node < in_cap() ? inpar_u(node) : NONE); }
    MTE_DEV void set_parent(u32 node, u32 lvl, u32 par) const {
        if (L == 0) {
            if (lvl == 0) set_bpar_lane(node, par);
            else if (node < in_cap()) INPAR()[node] = par;
        }
    }
    // Insert `nn` after `child` in `parent` (a node at level `lvl` >= 1); splits and root growth
    // follow insertingWalk/split/updateRoot (mergeTree.ts:2446-2489, 1876-1887).
    MTE_DEV void insert_after(u32 child, u32 nn, u32 lvl_child) {
        for (u32 guard = 0;; guard++) {
            if (guard > 32) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            u32 par = parent_of(child, lvl_child);
            if (par != NONE && par >= in_cap()) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            if (par == NONE) {  // child is the root: updateRoot
                u32 r = alloc_in();
                if (r == NONE) return;
                if (L == 0) {
                    INCH()[r * 8 + 0] = child;
                    INCH()[r * 8 + 1] = nn;
                    INCNT()[r] = 2;
                    INPAR()[r] = NONE;
                }
                set_parent(child, lvl_child, r);
                set_parent(nn, lvl_child, r);
                sync();
                st.root = r;
                st.height++;
                return;
            }
            u32 cnt = incnt_u(par);
            if (cnt > 8) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            u32 c = (L < cnt) ? INCH()[par * 8 + L] : NONE;
            u64 m = wave_ballot(L < cnt && c == child);
            if (!m) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            u32 idx = (u32)__builtin_ctzll(m);
            sync();
            if (L > idx && L < cnt && L + 1 < 8) INCH()[par * 8 + L + 1] = c;
            if (L == 0) {
                INCH()[par * 8 + idx + 1] = nn;
                INCNT()[par] = cnt + 1;
            }
            set_parent(nn, lvl_child, par);
            sync();
            if (cnt + 1 < 8) return;
            // split interior node `par` (mergeTree.ts:2476-2489)
            u32 q = alloc_in();
            if (q == NONE) return;
            u32 moved = NONE;
            if (L < 4) moved = INCH()[par * 8 + 4 + L];
            sync();
            if (L < 4) {
                INCH()[q * 8 + L] = moved;
                if (lvl_child == 0) set_bpar_lane(moved, q);
                else if (moved < in_cap()) INPAR()[moved] = q;
            }
            if (L == 0) {
                INCNT()[par] = 4;
                INCNT()[q] = 4;
            }
            sync();
            child = par;
            nn = q;
            lvl_child++;
        }
    }

    // Insert `rec` at slot j of leaf block `blk` (doc-order index k, child count cnt); a block that
    // reaches 8 children splits 4+4. fresh: rec is a new segment (else a split piece: the block's
    // visible length and max seq are unchanged). Returns the block holding rec (NONE on failure).
    MTE_DEV u32 insert_slot(u32 k, u32 blk, u32 cnt, u32 j, const Seg& rec, bool fresh) {
        MTE_PROF(PF_INSERT_SLOT);
        if (cnt >= 8 || j > cnt) {
            fail(MTE_DOC_CAPACITY, st.curSeq);
            return NONE;
        }
        const bool mv = L >= j && L < cnt;
        Seg t;
        if (mv) t = load(blk, L);
        const u32 oky = ORD()[k].y, okz = ORD()[k].z;  // read beside the slots (the stores do not touch them)
        sync();
        if (mv) store(blk, L + 1, t);
        if (L == 0) store(blk, j, rec);
        const u32 nc = cnt + 1;
        if (nc < 8) {
            if (L == 0) {
                u32 y = oky, z = okz;
                if (fresh) {
                    y += obs_len(rec.len, rec.meta);
                    const i32 hi = seq_hi(rec.seq, rec.rseq, rec.meta);
                    if (hi > (i32)z) z = (u32)hi;
                }
                ORD()[k].y = y;
                ORD()[k].z = z;
                ORD()[k].w = nc;
            }
            sync();
            return blk;
        }
        if (st.n_lb + 1 > ord_cap()) {
            fail_cap();
            return NONE;
        }
        MTE_COUNT(PN_SPLIT_BLK, 1);
        u32 nb = alloc_lb();
        if (nb == NONE) return NONE;
        Seg m;
        if (L < 4) m = load(blk, 4 + L);
        sync();
        if (L < 4) {
            store(nb, L, m);
            hint_set(m.sid, nb);
        }
        ord_shift_right(k + 1, 1);
        if (L == 0) {
            ORD()[k].w = 4;
            ORD()[k + 1] = make_uint4(nb, 0, 0, 4);
        }
        st.n_lb++;
        stat_max(ST_MAXLB, st.n_lb);
        sync();
        refresh(k, 2);
        insert_after(blk, nb, 0);
        return j < 4 ? blk : nb;
    }

    // ---------------------------------------------------------------- LRU heap (collections.ts:213-265)
    // Binary heap exactly as collections.ts:213-265 (key maxSeq, strict comparisons).
    // Push: the key is the current op's seq (add_lru's only callers) and seqs are validated
    // strictly increasing (client.ts:469-470), so every key already in the heap is <= the new one
    // and the sift-up (collections.ts:241-250, which moves strictly larger parents) never moves an
    // entry: a push appends.
    MTE_DEV void heap_push(u32 sid, i32 maxSeq, u32 blk) {
        MTE_PROF(PF_HEAP);
        if (st.heapSize + 1 >= heap_cap()) {
            fail_cap();
            return;
        }
        const u32 n = U(++st.heapSize);
        if (n == 1) st.heapTop = maxSeq;  // keys only grow: a push moves the root only into an empty heap
        MTE_COUNT(PN_PUSH, 1);
        if (L == 0) {
            HEAP()[n] = make_uint2(sid, (u32)maxSeq);
            hint_set(sid, blk);
        }
        sync();
    }
    // Pop: sift-down of collections.ts:252-264 (the smaller child, left on ties, moves up while
    // strictly below the moved last entry). k_lds: the whole heap (<= HEAP_CAP) read once as a
    // register image, the root-to-leaf path followed with readlanes; k_solo and HBM mode: lane 0
    // walks the child pairs in memory. Only the moved entries are written.
    // heap entry at a uniform position held in registers (position i: lane i % 64 of set i / 64)
    MTE_DEV static uint2 hent(uint2 h0, uint2 h1, uint2 h2, uint2 h3, u32 i) {
        if (i < 64) return make_uint2(wave_read(h0.x, i), wave_read(h0.y, i));
        if (i < 128) return make_uint2(wave_read(h1.x, i - 64), wave_read(h1.y, i - 64));
        if (HEAP_CAP < 192 || i < 192) return make_uint2(wave_read(h2.x, i - 128), wave_read(h2.y, i - 128));
        return make_uint2(wave_read(h3.x, i - 192), wave_read(h3.y, i - 192));
    }
    MTE_DEV uint2 heap_pop() {
        MTE_PROF(PF_HEAP);
        MTE_COUNT(PN_POP, 1);
        uint2* H = HEAP();
        const u32 n = st.heapSize;
        const u32 m = n - 1;
        uint2 x;
        if constexpr (SHARED) {  // the whole heap (<= HEAP_CAP) as a register image, scalar walk
            static_assert(HEAP_CAP < 256, "heap register image holds 256 positions");
            uint2 h0 = make_uint2(0, 0), h1 = h0, h2 = h0, h3 = h0;
            if (L <= n) h0 = H[L];
            if (n >= 64 && 64 + L <= n) h1 = H[64 + L];
            if (n >= 128 && 128 + L <= n) h2 = H[128 + L];
            if (HEAP_CAP >= 192 && n >= 192 && 192 + L <= n) h3 = H[192 + L];
            x = hent(h0, h1, h2, h3, 1);
            const uint2 last = hent(h0, h1, h2, h3, n);
            i32 newTop = (i32)last.y;
            u32 k = 1;
            while ((k << 1) <= m) {
                u32 j = k << 1;
                uint2 hj = hent(h0, h1, h2, h3, j);
                if (j < m) {
                    const uint2 hj1 = hent(h0, h1, h2, h3, j + 1);
                    if ((i32)hj.y - (i32)hj1.y > 0) {
                        j++;
                        hj = hj1;
                    }
                }
                if ((i32)last.y - (i32)hj.y <= 0) break;
                if (k == 1) newTop = (i32)hj.y;
                if (L == 0) H[k] = hj;
                k = j;
            }
            if (m >= 1 && L == 0) H[k] = last;
            st.heapTop = newTop;
        } else {
            x = make_uint2(0, 0);
            i32 newTop = 0;
            if (L == 0) {
                x = H[1];
                const uint2 last = H[n];
                newTop = (i32)last.y;
                u32 k = 1;
                while ((k << 1) <= m) {
                    u32 j = k << 1;
                    uint2 hj;
                    if (j < m) {
                        const uint4 pr = *(const uint4*)(H + j);  // both children (16-B aligned)
                        hj = make_uint2(pr.x, pr.y);
                        if ((i32)pr.y - (i32)pr.w > 0) {
                            j++;
                            hj = make_uint2(pr.z, pr.w);
                        }
                    } else {
                        hj = H[j];
                    }
                    if ((i32)last.y - (i32)hj.y <= 0) break;
                    if (k == 1) newTop = (i32)hj.y;
                    H[k] = hj;
                    k = j;
                }
                if (m >= 1) H[k] = last;
            }
            x.x = wave_read(x.x, 0);
            x.y = wave_read(x.y, 0);
            st.heapTop = wave_read(newTop, 0);
        }
        st.heapSize = m;
        sync();
        return x;
    }
    // addToLRUSet (mergeTree.ts:1273-1283) for a segment whose parent is `blk`.
    MTE_DEV void add_lru(u32 blk, u32 sid, i32 seq) {
        MTE_PROF(PF_LRU);
        if (!collab || blk == NONE) return;
        const u32 w = bmeta_u(blk);
        if ((w >> 30) != SC_TRUE && seq > st.curSeq) {
            sync();
            set_bscour_w(blk, w, SC_TRUE);
            sync();
            heap_push(sid, seq, blk);
        }
    }

    // ---------------------------------------------------------------- property maps (HBM, lane 0)
    MTE_DEV bool val_match(u32 a, u32 b) const {  // matchProperties on one key (properties.ts:72-80)
        if (a == b) return true;
        if (U(p.val_flags[b]) & 2u) {
            const u32 j = U(p.val_objidx[b]);
            if (j == NONE) return false;
            const u64 om = p.val_objmatch[a];
            return (U((u32)(j < 32 ? om : (om >> 32))) >> (j & 31)) & 1u;
        }
        return false;
    }
    MTE_DEV bool match_props(u32 a, u32 b) const {  // properties.ts:62-93
        if (a == b) return true;
        if constexpr (!FULL) return false;  // a batch without properties: every map id is 0
        if (a == 0 || b == 0) return false;
        if (a >= map_cap || b >= map_cap) return false;
        const_cast<Engine*>(this)->fence_ovl();  // map records are written lane-parallel (build_map)
        const u32* ma = maps + (u64)a * mw;
        const u32* mb = maps + (u64)b * mw;
        const u32 na = U(ma[0]), nb = U(mb[0]);
        if (na != nb) return false;
        for (u32 i = 0; i < na; i++) {
            const u32 k = U(ma[1 + 2 * i]), v = U(ma[2 + 2 * i]);
            bool found = false;
            for (u32 q = 0; q < nb; q++) {
                if (U(mb[1 + 2 * q]) == k) {
                    if (!val_match(v, U(mb[2 + 2 * q]))) return false;
                    found = true;
                    break;
                }
            }
            if (!found) return false;
        }
        return true;
    }
    // SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111) on an immutable map:
    // returns a fresh map id. Lane-parallel: lane i holds the map's pair i (key, value ids) in JS
    // insertion order, up to (mw - 1) / 2 pairs (<= MTE_MAX_PROPS); more fails the document alone.
    MTE_DEV u32 build_map(u32 old, u32 propset, bool rewrite) {
        if constexpr (!FULL) return 0;
        MTE_PROF(PF_MAP);
        if (st.mapNext >= map_cap) {  // the load-time estimate was short: re-run with the worst case
            fail(p.map_rerun ? MTE_DOC_CAPACITY : DOC_SPILL, st.curSeq);
            return 0;
        }
        const u32 maxp = (mw - 1) / 2 < MTE_MAX_PROPS ? (mw - 1) / 2 : MTE_MAX_PROPS;
        u32 n = 0, K = 0, V = 0;
        if (old && old < map_cap) {
            const u32* mo = maps + (u64)old * mw;
            n = U(mo[0]);
            if (n > maxp) n = maxp;
            if (L < n) {
                K = mo[1 + 2 * L];
                V = mo[2 + 2 * L];
            }
        }
        const mte_propset ps = p.propsets[propset];
        const u32 pc = U(ps.count), pf = U(ps.first);
        if (rewrite) {  // delete keys whose new value is falsy / absent (:65-78); order kept
            bool keep = false;
            for (u32 q = 0; q < pc; q++) {
                const u32 k = U(p.prop_keys[pf + q]);
                const bool falsy = (U(p.val_flags[U(p.prop_vals[pf + q])]) & 1u) != 0;
                if (L < n && K == k) keep = !falsy;
            }
            keep = keep && L < n;
            const u64 km = wave_ballot(keep);
            const u32 nk = (u32)__builtin_popcountll(km);
            const u32 below = __builtin_amdgcn_mbcnt_hi((u32)(km >> 32), __builtin_amdgcn_mbcnt_lo((u32)km, 0u));
            const u32 dst = keep ? below : nk + (L - below);  // a permutation of the lanes
            K = (u32)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)K);
            V = (u32)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)V);
            n = nk;
        }
        i32 err = 0;
        for (u32 q = 0; q < pc && !err; q++) {
            const u32 k = U(p.prop_keys[pf + q]), v = U(p.prop_vals[pf + q]);
            const u64 hm = wave_ballot(L < n && K == k);
            if (v == 0) {  // null deletes (:98-100): the pairs after it move down one lane
                if (hm) {
                    const u32 at = (u32)__builtin_ctzll(hm);
                    const u32 K1 = wave_shfl(K, (L + 1) & 63), V1 = wave_shfl(V, (L + 1) & 63);
                    if (L >= at) {
                        K = K1;
                        V = V1;
                    }
                    n--;
                }
            } else if (hm) {
                if (L == (u32)__builtin_ctzll(hm)) V = v;
            } else if (n < maxp) {
                if (L == n) {
                    K = k;
                    V = v;
                }
                n++;
            } else {
                err = MTE_DOC_UNSUPPORTED;
            }
        }
        if (err) {
            fail(err, st.curSeq);
            return 0;
        }
        const u32 id = st.mapNext;
        u32* m = maps + (u64)id * mw;
        if (L < n) {
            m[1 + 2 * L] = K;
            m[2 + 2 * L] = V;
        }
        if (L == 0) m[0] = n;
        st.gdirty = 1;  // other lanes read these pairs later: fence_ovl first
        st.mapNext++;
        return id;
    }

    // ---------------------------------------------------------------- text arena (HBM)
    MTE_DEV u16* text_ptr(u32 off) const {
        return (off & ARENA_BIT) ? arena0 + (u64)st.arenaSel * arena_cap + (off & ~ARENA_BIT) : payload + off;
    }
    MTE_DEV bool text_ok(u32 off, u32 n) const {
        u64 end = (u64)(off & ~ARENA_BIT) + n;
        return (off & ARENA_BIT) ? end <= arena_cap : end <= payload_len;
    }
    // TextSegment.canAppend's `!text.endsWith("\n")` (textSegment.ts:63-69): only documents whose
    // payload holds a newline read text here.
    MTE_DEV bool ends_nl(u32 off, u32 n) const {
        if (!has_nl || n == 0 || !text_ok(off, n)) return false;
        return text_ptr(off)[n - 1] == (u16)u'\n';
    }
    // Semispace compaction of the merge arena (all live arena-resident segment texts).
    MTE_DEV void arena_gc() {
        fence_arena();
        const u32 other = st.arenaSel ^ 1u;
        u16* dst = arena0 + (u64)other * arena_cap;
        u32 top = 0;
        for (u32 k = 0; k < st.n_lb; k++) {
            uint4 o = ord_u(k);
            const u32 cnt = o.w > 8 ? 8u : o.w;
            for (u32 s = 0; s < cnt; s++) {
                uint4 v = U(VIS()[o.x * 8 + s]);
                uint4 a = U(AUX()[o.x * 8 + s]);
                if ((v.w & F_MARKER) || !(a.y & ARENA_BIT)) continue;
                const u32 len = v.x;
                const bool rm = (v.w & F_REMOVED) != 0;  // aux.z is the overlap mask then
                const u32 cap = (rm || a.z < len) ? len : a.z;
                if (!text_ok(a.y, len) || top + cap > arena_cap) {
                    fail(MTE_DOC_CAPACITY, st.curSeq);
                    return;
                }
                const u16* src = text_ptr(a.y);
                for (u32 i = L; i < len; i += 64) dst[top + i] = src[i];
                sync();
                if (L == 0) AUX()[o.x * 8 + s] = make_uint4(a.x, top | ARENA_BIT, rm ? a.z : cap, a.w);
                sync();
                top += cap;
            }
        }
        wave_sync();
        st.arenaSel = other;
        st.arenaTop = top;
        stat_add(ST_GC, 1);
    }
    // ---------------------------------------------------------------- zamboni (mergeTree.ts:1289-1478)
    // Text copies recorded by one scour, executed together: lane j < nj holds job j.
    struct Jobs {
        u32 n;               // uniform: number of jobs
        u32 dst, src, len;   // per lane
    };
    MTE_DEV void job_add(Jobs& jb, u32 dst, u32 src, u32 len) {
        if (L == jb.n) {
            jb.dst = dst;
            jb.src = src;
            jb.len = len;
        }
        jb.n++;
    }
    // All recorded copies as one flattened gather: lane l moves char base+l of the concatenated
    // jobs (sources are never destinations of the same batch, see scour()).
    MTE_DEV void run_jobs(const Jobs& jb) {
        MTE_PROF(PF_TEXT);
        const u32 jl = L < jb.n ? jb.len : 0u;
        const u32 jinc = wave_scan_incl(jl);
        const u32 total = wave_read(jinc, 63);
        const u32 jstart = jinc - jl;
        for (u32 base = 0; base < total; base += 64) {
            const u32 f = base + L;
            u32 j = 0;
            for (u32 q = 1; q < jb.n; q++)
                if (f >= wave_read(jstart, q)) j = q;
            const u32 s0 = wave_shfl(jstart, j), d = wave_shfl(jb.dst, j), sr = wave_shfl(jb.src, j);
            if (f < total) {
                const u32 o = f - s0;
                text_ptr(d)[o] = text_ptr(sr)[o];
            }
        }
        st.adirty = 1;
    }

    // scourNode on leaf block `blk` (doc-order index k, child count cnt), compacting the kept
    // slots in place; returns the new child count (mergeTree.ts:1289-1366).
    //  1. lane-parallel classification of the slots into bit masks (ballots);
    //  2. the left-to-right merge chain on those masks (uniform scalar code): tombstones at or
    //     below the MSN are dropped and reset the chain, settled live text appends to the chain
    //     head under TextSegment.canAppend + matchProperties (textSegment.ts:63-85,
    //     properties.ts:62-93); text moves are recorded as copy jobs;
    //  3. the jobs run as one gather (arena GC first if the merge arena is full), the kept slots
    //     are compacted.
    MTE_DEV u32 scour(u32 k, u32 blk, u32 cnt) {
        MTE_PROF(PF_SCOUR);
        if (cnt > 8) cnt = 8;
        fence_arena();
        Seg me;
        const bool act = L < cnt;
        if (act) me = load(blk, L);
        const bool rem = act && (me.meta & F_REMOVED);
        const u64 mREM = wave_ballot(rem);
        const u64 mKEPT = wave_ballot(rem && me.rseq > st.minSeq);  // tombstones still in the window
        const u64 mSET = wave_ballot(act && !rem && me.seq <= st.minSeq);
        MTE_COUNT(PN_SCOUR, 1);
        if (!(mREM & ~mKEPT) && !(mSET & (mSET << 1))) return cnt;  // nothing dropped, nothing to merge
        MTE_COUNT(PN_SCOUR_CHANGED, 1);
        const u64 mTXT = wave_ballot(act && !(me.meta & (F_MARKER | F_PERM)));
        // PermutationSegment runs (EXT batches only): canAppend holds between two unallocated runs or
        // two handle runs where the second starts at the first's end (permutationvector.ts:88-94; toff
        // holds the start handle, 0 = unallocated), no granularity, no text
        const u64 mPERM = EXT ? wave_ballot(act && (me.meta & F_PERM)) : 0ull;
        const u64 mNL = (FULL && has_nl) ? wave_ballot(act && !(me.meta & F_MARKER) && ends_nl(me.toff, me.len)) : 0ull;
        u32 nkeep = 0;
        u32 kSrc = 0, kLen = 0, kOff = 0, kCap = 0;  // lane i < nkeep: kept slot i
        Jobs jb;
#ifdef MTE_PROFILE
        u64 _tc0 = MTE_PON(PF_SCOUR_CHAIN) ? __builtin_amdgcn_s_memtime() : 0;
#endif
        for (u32 attempt = 0; attempt < 2; attempt++) {
            nkeep = 0;
            jb.n = 0;
            jb.dst = jb.src = jb.len = 0;
            u32 top = st.arenaTop, need = 0;
            i32 prev = -1;  // kept index of the chain head
            // pMat: leading chars of the head's text already in memory; [pMat, pLen) are pending
            // in-place append jobs of this batch (a copy of the head must not read them)
            u32 pLen = 0, pOff = 0, pCap = 0, pProps = 0, pMat = 0;
            bool pText = false, pNL = false, pFresh = false, pPerm = false;
            for (u32 s = 0; s < cnt; s++) {
                const u64 bit = 1ull << s;
                bool keep = true;
                if (mREM & bit) {
                    keep = (mKEPT & bit) != 0;
                    prev = -1;
                } else if (mSET & bit) {
                    const u32 len = wave_read(me.len, s), props = wave_read(me.props, s);
                    const u32 toff = wave_read(me.toff, s), tcap = wave_read(me.tcap, s);
                    const bool ok = prev >= 0 && match_props(pProps, props) &&
                                    (pPerm ? (mPERM & bit) != 0 && toff == (pOff ? pOff + pLen : 0u)
                                           : pText && !pNL && (mTXT & bit) &&
                                                 (pLen <= (u32)GRANULARITY || len <= (u32)GRANULARITY));
                    if (ok) {  // TextSegment.append (textSegment.ts:74-85) / PermutationSegment.append
                        if (pPerm) {
                        } else if ((pOff & ARENA_BIT) && pLen + len <= pCap) {
                            job_add(jb, pOff + pLen, toff, len);
                        } else if (pOff + pLen == toff && pMat == pLen) {  // text already contiguous
                            if (pOff & ARENA_BIT) pCap = toff + tcap - pOff;
                            pMat += len;
                        } else {
                            u32 ncap = 2 * (pLen + len);
                            if (ncap < 32) ncap = 32;
                            const u32 dst = top | ARENA_BIT;
                            top += ncap;
                            need += ncap;
                            // pending jobs into the head's chunk follow it to the new one; the
                            // materialised prefix (none for a chunk built by this batch) is copied
                            const u32 m0 = pFresh ? 0u : pMat;
                            if (L < jb.n && jb.dst >= pOff + m0 && jb.dst < pOff + pLen) jb.dst = jb.dst - pOff + dst;
                            if (m0) job_add(jb, dst, pOff, m0);
                            job_add(jb, dst + pLen, toff, len);
                            pOff = dst;
                            pCap = ncap;
                            pFresh = true;
                        }
                        pLen += len;
                        pNL = (mNL & bit) != 0;
                        if ((i32)L == prev) {
                            kLen = pLen;
                            kOff = pOff;
                            kCap = pCap;
                        }
                        keep = false;
                    } else {
                        prev = (i32)nkeep;
                        pLen = len;
                        pMat = len;
                        pOff = toff;
                        pCap = tcap;
                        pProps = props;
                        pText = (mTXT & bit) != 0;
                        pPerm = (mPERM & bit) != 0;
                        pNL = pText && (mNL & bit);
                        pFresh = false;
                    }
                } else {
                    prev = -1;
                }
                if (keep) {
                    if (L == nkeep) {
                        kSrc = s;
                        kLen = wave_read(me.len, s);
                        kOff = wave_read(me.toff, s);
                        kCap = wave_read(me.tcap, s);
                    }
                    nkeep++;
                }
            }
            if (nkeep == cnt) return cnt;
            if (st.arenaTop + need <= arena_cap && jb.n <= 64) {
                st.arenaTop = top;
                break;
            }
            if (attempt == 1) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return cnt;
            }
            arena_gc();  // moves every arena text: re-read the slots and redo the chain
            if (st.status) return cnt;
            if (act) me = load(blk, L);
        }
        if constexpr (EXT) {
            // MergeTreeMaintenanceType.UNLINK of each dropped permutation run, in slot order
            // (PermutationVector.onMaintenance, permutationvector.ts:357-382): its handles go back to
            // the free list in ascending order
            for (u64 fm = mREM & ~mKEPT & mPERM; fm && p.docs[doc].ht_cap; fm &= fm - 1) {
                const u32 s = (u32)__builtin_ctzll(fm);
                const u32 h0 = wave_read(me.toff, s), n = wave_read(me.len, s);
                if (h0) ht_free(h0, n);
            }
        }
#ifdef MTE_PROFILE
        if (MTE_PON(PF_SCOUR_CHAIN) && L == 0) atomicAdd(prof + PF_SCOUR_CHAIN, __builtin_amdgcn_s_memtime() - _tc0);
        MTE_PROF(PF_SCOUR_WRITE);
#endif
        if (jb.n) run_jobs(jb);
        Seg out = load(blk, L < nkeep ? kSrc : 0u);  // the kept slots, re-read (not yet overwritten)
        if (L < nkeep) {
            out.len = kLen;
            out.toff = kOff;
            out.tcap = kCap;
        }
        sync();
        if (L < nkeep) store(blk, L, out);
        const u32 ol = L < nkeep ? obs_len(out.len, out.meta) : 0u;
        const i32 om = L < nkeep ? seq_hi(out.seq, out.rseq, out.meta) : 0;
        const u32 tl = wave_read(group8_scan(ol), 7);
        const i32 tm = wave_read(group8_max(om), 7);
        if (L == 0) ORD()[k] = make_uint4(blk, tl, (u32)tm, nkeep);
        sync();
        return nkeep;
    }

    // pack (mergeTree.ts:1368-1420), second half: the m children of `par` (doc-order run k0..k0+m,
    // already re-scoured; lane i < m holds child i's id in `kids` and its count in `cnts`) are
    // redistributed into max(1, min(7, T/4)) fresh blocks.
    MTE_DEV void pack_leaves(u32 par, u32 m, u32 kids, u32 k0, u32 cnts) {
        MTE_PROF(PF_PACK);
        MTE_COUNT(PN_PACK, 1);
        const u32 T = wave_sum(L < m ? cnts : 0u);
        u32 kk = T / 4;
        if (kk > 7) kk = 7;
        if (kk < 1) kk = 1;
        const u32 base = T / kk, extra = T % kk;
        if (st.n_lb + kk > ord_cap() + m) {
            fail_cap();
            return;
        }
        // lane t < T holds item t of the concatenated children
        u32 sib = 0, q = L;
        for (u32 i = 0; i < m; i++) {
            u32 n = wave_read(cnts, i);
            if (q >= n && sib == i) {
                q -= n;
                sib = i + 1;
            }
        }
        const u32 srcBlk = wave_shfl(kids, sib < m ? sib : 0u);
        Seg rec;
        if (L < T) rec = load(srcBlk, q);
        sync();
        // The kk packed blocks reuse the ids of the first min(kk, m) old children (block ids are
        // not observable): only the difference is freed or allocated.
        for (u32 i = kk; i < m; i++) free_lb(wave_read(kids, i));
        u32 nb = L < m ? kids : NONE;
        for (u32 j = m; j < kk; j++) {
            u32 id = alloc_lb();
            if (id == NONE) return;
            if (L == j) nb = id;
        }
        u32 dj, dq;
        const u32 big = extra * (base + 1);
        if (L < big) {
            dj = L / (base + 1);
            dq = L % (base + 1);
        } else {
            dj = extra + (L - big) / (base ? base : 1);
            dq = (L - big) % (base ? base : 1);
        }
        const u32 dstBlk = wave_shfl(nb, dj < kk ? dj : 0u);
        if (L < T) {
            store(dstBlk, dq, rec);
            hint_set(rec.sid, dstBlk);
        }
        if (L < kk) {
            BMETA()[nb] = (par & BM_PAR) | (SC_UNDEF << 30);
            INCH()[par * 8 + L] = nb;
        }
        if (L == 0) INCNT()[par] = kk;
        sync();
        // splice ord: the run of the parent's old children becomes the kk new blocks
        if (kk > m) {
            ord_shift_right(k0 + m, kk - m);
            st.n_lb += kk - m;
            stat_max(ST_MAXLB, st.n_lb);
        } else if (kk < m) {
            ord_shift_left(k0 + m, m - kk);
            st.n_lb -= m - kk;
        }
        if (L < kk) ORD()[k0 + L] = make_uint4(nb, 0, 0, base + (L < extra ? 1u : 0u));
        sync();
        refresh(k0, kk);
        if (kk < 4 && par < in_cap() && inpar_u(par) != NONE) pack_internal(par, 1);
    }

    // pack on an interior level: `node` (level lvl) underflowed; redistribute the grandchildren of
    // its parent over max(1, min(7, T/4)) fresh interior nodes.
    MTE_DEV void pack_internal(u32 node, u32 lvl) {
        for (u32 guard = 0;; guard++) {
            if (guard > 32) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            const u32 par = inpar_u(node);
            if (par >= in_cap() || incnt_u(par) > 8) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            const u32 m = incnt_u(par);
            const u32 kids = L < m ? INCH()[par * 8 + L] : NONE;
            const u32 cnts = (L < m && kids < in_cap()) ? INCNT()[kids] : 0u;
            if (wave_ballot(L < m && (kids >= in_cap() || cnts > 8))) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            const u32 T = wave_sum(cnts);
            u32 kk = T / 4;
            if (kk > 7) kk = 7;
            if (kk < 1) kk = 1;
            const u32 base = T / kk, extra = T % kk;
            u32 sib = 0, q = L;
            for (u32 i = 0; i < m; i++) {
                u32 n = wave_read(cnts, i);
                if (q >= n && sib == i) {
                    q -= n;
                    sib = i + 1;
                }
            }
            const u32 srcN = wave_shfl(kids, sib < m ? sib : 0u);
            u32 gc = NONE;
            if (L < T) gc = INCH()[srcN * 8 + q];
            sync();
            // reuse the first min(kk, m) old interior ids (not observable)
            for (u32 i = kk; i < m; i++) free_in(wave_read(kids, i));
            u32 nb = L < m ? kids : NONE;
            for (u32 j = m; j < kk; j++) {
                u32 id = alloc_in();
                if (id == NONE) return;
                if (L == j) nb = id;
            }
            const u32 big = extra * (base + 1);
            u32 dj, dq;
            if (L < big) {
                dj = L / (base + 1);
                dq = L % (base + 1);
            } else {
                dj = extra + (L - big) / (base ? base : 1);
                dq = (L - big) % (base ? base : 1);
            }
            const u32 dstN = wave_shfl(nb, dj < kk ? dj : 0u);
            if (L < T) {
                INCH()[dstN * 8 + dq] = gc;
                if (lvl == 1) set_bpar_lane(gc, dstN);
                else if (gc < in_cap()) INPAR()[gc] = dstN;
            }
            if (L < kk) {
                INCNT()[nb] = base + (L < extra ? 1u : 0u);
                INPAR()[nb] = par;
                INCH()[par * 8 + L] = nb;
            }
            if (L == 0) INCNT()[par] = kk;
            sync();
            if (kk < 4 && inpar_u(par) != NONE) {
                node = par;
                lvl++;
                continue;
            }
            return;
        }
    }

    // zamboniSegments (mergeTree.ts:1422-1478): up to 2 heap entries with maxSeq <= minSeq; each
    // live one scours its segment's block, and an underflowing block packs its parent, which
    // re-scours every sibling (the block included). One scour call site: a task loop.
    MTE_DEV void zamboni() {
        if (!collab) return;
        MTE_PROF(PF_ZAMBONI);
        for (int i = 0; i < 2 && !st.status; i++) {
            if (st.heapSize == 0 || st.heapTop > st.minSeq) break;
            uint2 e = heap_pop();
            u32 k, blk, cnt, bm;
            if (!find_seg(e.x, k, blk, cnt, bm)) continue;  // segment no longer linked
            if ((bm >> 30) == SC_FALSE) continue;
            bool packing = false;
            u32 par = NONE, m = 0, kids = NONE, k0 = 0, cnts = 0, idx = 0;
            for (;;) {
                const u32 nc = scour(k, blk, cnt);
                if (st.status) return;
                if (!packing) {
                    set_bscour_w(blk, bm, SC_FALSE);  // scour leaves the metadata word alone
                    sync();
                    if (!(nc < cnt && nc < 4 && st.height > 1)) break;
                    par = par_of_word(bm);
                    if (par == NONE || par >= in_cap() || incnt_u(par) > 8 || incnt_u(par) == 0) {
                        fail(MTE_DOC_CAPACITY, st.curSeq);
                        return;
                    }
                    m = incnt_u(par);
                    kids = L < m ? INCH()[par * 8 + L] : NONE;
                    k0 = ord_find(wave_read(kids, 0));
                    if (k0 == NONE || k0 + m > st.n_lb ||
                        wave_ballot(L < m && ORD()[k0 + (L < m ? L : 0)].x != kids)) {
                        fail(MTE_DOC_CAPACITY, st.curSeq);
                        return;
                    }
                    packing = true;
                    idx = 0;
                } else {
                    if (L == idx) cnts = nc;
                    idx++;
                }
                if (idx == m) {
                    pack_leaves(par, m, kids, k0, cnts);
                    break;
                }
                const uint4 o = ord_u(k0 + idx);
                k = k0 + idx;
                blk = o.x;
                cnt = o.w;
            }
        }
    }

    // ---------------------------------------------------------------- ops
    // One merge-tree edit. Insert (insertSegments, mergeTree.ts:1968-1998): split at pos
    // (ensureIntervalBoundary), then place the new segment. Remove / annotate
    // (mergeTree.ts:2565-2719): split at p1 and p2, then mark the range. The phases share ONE
    // resolve and ONE insert_slot call site. Returns false when nothing was edited (empty insert).
    MTE_DEV bool edit(u32 type, i32 p1, i32 p2, i32 R, u32 C, i32 seq, Seg rec, u32 propset, bool rewrite, bool cu) {
        MTE_PROF(PF_EDIT);
        const bool ins = type == MTE_OP_INSERT || type == MTE_OP_INSERT_MARKER;
        const u32 nphase = ins ? 2u : 3u;
        Found known;  // insert after a split: the insertion point follows from the split (below)
        known.ok = false;
        // remove / annotate: ONE block scan serves both boundaries and the mark pass while the block
        // layout it saw holds (a boundary split that splits its block 8 -> 4+4 changes n_lb: the later
        // phases scan again); blocks keep their visible lengths across a boundary split
        u32 pv = 0, pincl = 0, pn = NONE;
        if (!ins && st.n_lb <= 64) {
            fence_ovl();
            const bool valid = L < st.n_lb;
            const uint4 po = valid ? ORD()[L] : make_uint4(0, 0, 0, 0);
            pv = blen_all(po, valid, R, C);
            pincl = wave_scan_incl(pv);
            pn = st.n_lb;
            if constexpr (!PRE_REGS) {
                pre_put(pv);
                pv = pincl = 0;  // not live across the phases
            }
        }
        for (u32 ph = 0; ph < nphase; ph++) {
            if (!ins && ph == 2) {
                if (EXT && type == MTE_OP_CELL) return st.status == 0;  // walkSegments' splitRange only
                range_op(type == MTE_OP_REMOVE, p1, p2, R, C, seq, propset, rewrite, pn == st.n_lb, pv, pincl, cu);
                return st.status == 0;
            }
            const bool place = ins && ph == 1;
            const i32 pos = ph == 1 && !ins ? p2 : p1;
            const Found f = known.ok ? known : (pn == st.n_lb ? resolve_pre(pv, pincl, pos, R, C) : resolve(pos, R, C));
            if (!f.ok) {
                if (ins) {
                    fail(MTE_DOC_INSERT_FAILED, seq);
                    return false;
                }
                continue;
            }
            Seg task;
            u32 j;
            if (place) {
                if (rec.len == 0) return false;  // blockInsert skips empty segments (:2196)
                rec.sid = new_sid();
                if (rec.sid == NONE) return false;
                task = rec;
                j = f.slot >= 0 ? (u32)f.slot : f.cnt;
            } else {
                if (!(f.slot >= 0 && f.r > 0)) continue;
                MTE_PROF(PF_SPLIT);
                // ensureIntervalBoundary: split slot f.slot at f.r (BaseSegment.splitAt, :524-568)
                Seg left = load_u(f.blk, (u32)f.slot);
                const u32 sid = new_sid();
                if (sid == NONE) return false;
                task = left;
                const u32 r = (u32)f.r;
                task.len = left.len - r;
                // PermutationSegment.createSplitSegmentAt (permutationvector.ts:105-117): the handle
                // run continues (toff = start handle, 0 = Handle.unallocated)
                task.toff = (EXT && (left.meta & F_PERM) && left.toff == 0u) ? 0u : left.toff + r;
                const bool rm = (left.meta & F_REMOVED) != 0;  // tcap holds the overlap mask then
                task.tcap = rm ? left.tcap : ((left.toff & ARENA_BIT) ? left.tcap - r : 0u);
                task.sid = sid;
                left.len = r;
                left.tcap = rm ? left.tcap : ((left.toff & ARENA_BIT) ? r : 0u);
                if (left.meta & F_OVLHI) {  // the right piece copies removedClientOverlap (clients >= 32)
                    fence_ovl();
                    if (L == 0 && left.sid < seg_cap && sid < seg_cap) {
                        ovl[sid] = ovl[left.sid];
                        if (ovl2) ovl2[sid] = ovl2[left.sid];
                    }
                    st.gdirty = 1;
                }
                sync();
                if (L == 0) store(f.blk, (u32)f.slot, left);
                sync();
                j = (u32)f.slot + 1;
            }
            const u32 b = U(insert_slot(f.k, f.blk, f.cnt, j, task, place));
            if (st.status) return false;
            if (ins && !place) {
                // The split left piece ends exactly at pos and the right piece (visible to C)
                // starts there, so the insertingWalk re-walk (mergeTree.ts:2248-2277) lands
                // before the right piece -- except when the block split 4+4 right between the
                // two pieces: then the left block's end equals pos, blocks win ties, and the
                // new segment is appended to the left block.
                const u32 s = (u32)f.slot;  // left piece
                known.ok = true;
                known.r = 0;
                known.cum = 0;  // unused by the placement
                if (f.cnt + 1 < 8) {
                    known.k = f.k;
                    known.blk = f.blk;
                    known.cnt = f.cnt + 1;
                    known.slot = (i32)s + 1;
                } else if (s + 1 < 4) {
                    known.k = f.k;
                    known.blk = f.blk;
                    known.cnt = 4;
                    known.slot = (i32)s + 1;
                } else if (s == 3) {
                    known.k = f.k;
                    known.blk = f.blk;
                    known.cnt = 4;
                    known.slot = -1;  // append
                } else {
                    known.k = f.k + 1;
                    known.blk = U(ORD()[f.k + 1].x);
                    known.cnt = 4;
                    known.slot = (i32)s - 3;
                }
            }
            if (EXT && place && cu) {  // the inserted segment's delta range
                const u32 kb = b == f.blk ? f.k : f.k + 1;
                const u32 cntb = U(ORD()[kb].w);
                const u64 m = wave_ballot(L < cntb && L < 8 && AUX()[sidx(b, L)].w == rec.sid);
                cu_record(0, obs_prefix(kb, b, m ? (u32)__builtin_ctzll(m) : 0u), rec.len, 0, 0);
                if (st.status) return false;
            }
            if (place && collab && seq > st.minSeq) add_lru(b, rec.sid, seq);
        }
        return st.status == 0;
    }

    // markRangeRemoved / annotateRange mark pass (nodeMap, mergeTree.ts:2903-2965): positions are
    // those of the (R, C) view before the op; blocks overlapping [p1, p2) are processed in order.
    // pre: the block scan of edit() is still valid (n_lb <= 64, one chunk): pv / pincl per lane.
    MTE_DEV void range_op(bool remove, i32 p1, i32 p2, i32 R, u32 C, i32 seq, u32 propset, bool rewrite, bool pre,
                          u32 pv, u32 pincl, bool cu) {
        MTE_PROF(PF_RANGE);
        fence_ovl();
        i32 cum = 0;
        u32 memoOld = NONE, memoNew = 0;
        for (u32 base = 0; base < st.n_lb && cum < p2; base += 64) {
            const u32 k = base + L;
            const bool valid = k < st.n_lb;
            uint4 o = valid ? ORD()[k] : make_uint4(0, 0, 0, 0);
            if (pre) pre_get(pv, pincl);
            const u32 v = pre ? pv : blen_all(o, valid, R, C);
            const u32 incl = pre ? pincl : wave_scan_incl(v);
            const i32 cb = cum + (i32)(incl - v);
            u64 hm = wave_ballot(valid && v > 0 && cb < p2 && cb + (i32)v > p1);
            cum += (i32)wave_read(incl, 63);
            while (hm) {
                const u32 j = (u32)__builtin_ctzll(hm);
                hm &= hm - 1;
                const u32 kj = base + j;
                const u32 blk = wave_read(o.x, j);
                const u32 cnt = wave_read(o.w, j);
                const i32 cbj = wave_read(cb, j);
                // per slot (lanes 0..7)
                const u32 s = L;
                const u32 idx = sidx(blk, s);
                uint4 q = VIS()[idx];
                const u32 z = AUX()[idx].z;
                const u32 oby = remove ? ORD()[kj].y : 0u, obz = remove ? ORD()[kj].z : 0u;  // beside the slots
                const bool in = s < cnt && s < 8;
                const u32 sv = in ? vis_len(q, z, idx, R, C, C == 0 ? 1u : 0u) : 0u;
                const u32 si = group8_scan(sv);
                const i32 ex = cbj + (i32)(si - sv);
                const bool mark = s < cnt && s < 8 && sv > 0 && ex < p2 && ex + (i32)sv > p1;
                const u64 mm = wave_ballot(mark);
                if (!mm) continue;
                const u32 sid = mark ? AUX()[idx].w : NONE;
                if (remove) {
                    u32 fresh = 0;
                    if (mark) {
                        if (q.w & F_REMOVED) {  // addOverlappingClient (:2544-2552)
                            if (C < 32) {
                                AUX()[idx].z = AUX()[idx].z | (1u << C);
                            } else if (sid < seg_cap) {
                                // F_OVLHI's first setting writes every word (stale from an earlier pass)
                                const bool had = (q.w & F_OVLHI) != 0;
                                if (C < 64) {
                                    ovl[sid] = (had ? ovl[sid] : 0ull) | (1ull << C);
                                    if (ovl2 && !had) ovl2[sid] = 0ull;
                                } else if (ovl2) {
                                    ovl2[sid] = (had ? ovl2[sid] : 0ull) | (1ull << (C - 64));
                                    if (!had) ovl[sid] = 0ull;
                                }
                                q.w |= F_OVLHI;
                            }
                            q.w |= F_OVL;
                            VIS()[idx].w = q.w;
                        } else {
                            q.w = (q.w & ~0xff00u) | (C << 8) | F_REMOVED;
                            VIS()[idx] = make_uint4(q.x, q.y, (u32)seq, q.w);
                            AUX()[idx].z = 0;  // overlap mask starts empty
                            fresh = q.x;
                        }
                    }
                    if (C >= 32 && wave_ballot(mark && !fresh)) st.gdirty = 1;
                    const u32 gone = wave_read(group8_scan(fresh), 7);
                    if (L == 0) {
                        ORD()[kj].y = oby - gone;
                        if (gone && seq > (i32)obz) ORD()[kj].z = (u32)seq;
                    }
                    if (EXT && cu) {  // removedSegments (mergeTree.ts:2639): the segments this op removed
                        for (u64 fm = wave_ballot(fresh != 0); fm && !st.status; fm &= fm - 1) {
                            const u32 sl = (u32)__builtin_ctzll(fm);
                            cu_record(1, obs_prefix(kj, blk, sl), wave_read(fresh, sl), 0, 0);
                        }
                        if (st.status) return;
                    }
                } else {
                    const u32 props = mark ? AUX()[idx].x : 0u;
                    u64 pending = mm;
                    while (pending) {
                        const u32 leader = (u32)__builtin_ctzll(pending);
                        const u32 old = wave_read(props, leader);
                        u32 nid;
                        if (old == memoOld) {
                            nid = memoNew;
                        } else {
                            nid = build_map(old, propset, rewrite);
                            if (st.status) return;
                            memoOld = old;
                            memoNew = nid;
                        }
                        const bool same = mark && props == old && ((pending >> L) & 1ull);
                        if (same) AUX()[idx].x = nid;
                        pending &= ~wave_ballot(same);
                    }
                    if (EXT && cu) {  // deltaSegments with their propertyDeltas (maps before / after)
                        for (u64 am = mm; am && !st.status; am &= am - 1) {
                            const u32 sl = (u32)__builtin_ctzll(am);
                            sync();
                            const u32 nmap = U(AUX()[sidx(blk, sl)].x);
                            cu_record(2, obs_prefix(kj, blk, sl), wave_read(q.x, sl), nmap, wave_read(props, sl));
                        }
                        if (st.status) return;
                    }
                }
                sync();
                // addToLRUSet: only the first marked slot of a block can enqueue (needsScour)
                if (collab) {
                    const u32 lead = (u32)__builtin_ctzll(mm);
                    add_lru(blk, wave_read(sid, lead), seq);
                    if (st.status) return;
                }
            }
        }
    }

    // ---------------------------------------------------------------- resume from a summary
    // SnapshotLoader (snapshotLoader.ts:113-216) as records (include/mte.h MTE_OP_LOAD_*), applied
    // outside the op path (replay_run dispatches them). LOAD_SEG fills the leaf blocks in document
    // order (a new block at MTE_F_LOAD_LEAF); LOAD_END links the interior levels described by the
    // LOAD_NODE records before it (the shape of reloadFromSegments + loadBody's appends, computed by
    // the builder and checked against the oracle's insertingWalk) and opens the collaboration window.
    MTE_DEV void load_record(const mte_op& op, u64 i) {
        if (!collab || op.type > MTE_OP_LOAD_APPEND) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        if (op.type == MTE_OP_LOAD_NODE) return;  // consumed by LOAD_END
        if (op.type == MTE_OP_LOAD_APPEND) {  // applied by apply() (one edit call site)
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        if (op.type == MTE_OP_LOAD_END) {
            load_link(op, i);
            return;
        }
        if (st.root == NONE) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        const bool mk = (op.flags & MTE_F_LOAD_MARKER) != 0;
        const bool rm = (op.flags & MTE_F_LOAD_REMOVED) != 0;
        if (op.client >= MTE_MAX_CLIENTS || (rm && (u32)op.pos1 >= MTE_MAX_CLIENTS)) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        Seg rec;
        rec.len = mk ? 1u : op.b;
        rec.props = op.props ? build_map(0, op.props, false) : 0u;
        if (st.status) return;
        rec.toff = (u32)op.a;  // text offset, or the marker's refType
        rec.tcap = 0;          // (the overlap mask of a removed segment: empty)
        rec.seq = op.seq;
        rec.rseq = rm ? op.ref_seq : 0;
        rec.meta = (op.client & 0xffu) | (mk ? F_MARKER : 0u) | (rm ? ((((u32)op.pos1 & 0xffu) << 8) | F_REMOVED) : 0u) |
                   ((EXT && (op.flags & MTE_F_PERM)) ? F_PERM : 0u);  // a loaded run: its start handle in toff
        rec.sid = new_sid();
        if (rec.sid == NONE) return;
        u32 k = st.n_lb - 1;
        uint4 o = ord_u(k);
        if (op.flags & MTE_F_LOAD_LEAF) {
            if (st.n_lb + 1 > ord_cap()) {
                fail_cap();
                return;
            }
            const u32 nb = alloc_lb();
            if (nb == NONE) return;
            k = st.n_lb++;
            stat_max(ST_MAXLB, st.n_lb);
            o = make_uint4(nb, 0, 0, 0);
        } else if (o.w >= 7) {  // a block holds <= 7 children between ops
            fail(MTE_DOC_CAPACITY, op.seq);
            return;
        }
        if (L == 0) {
            store(o.x, o.w, rec);
            o.y += obs_len(rec.len, rec.meta);
            const i32 hi = seq_hi(rec.seq, rec.rseq, rec.meta);
            if (hi > (i32)o.z) o.z = (u32)hi;
            o.w += 1;
            ORD()[k] = o;
        }
        sync();
    }
    // buildMergeBlock (mergeTree.ts:1202-1230) generalised to the recorded child counts, then
    // startOrUpdateCollaboration(minSeq, currentSeq) (snapshotLoader.ts:126-140).
    MTE_DEV void load_link(const mte_op& end, u64 i) {
        const u64 nn = (u64)(u32)end.a;
        const u64 b0 = p.docs[doc].op_begin;
        if (end.msn > end.seq || st.heapSize != 0 || st.inUsed != 0 || st.inFree != NONE || i < b0 + nn) {
            fail(MTE_DOC_SEQ_ORDER, end.seq);
            return;
        }
        u32 lvl = 1, below = NONE, nBelow = st.n_lb, cur = 0, first = NONE, made = 0, last = NONE;
        for (u64 j = i - nn; j < i; j++) {
            const mte_op nd = read_op(p.ops + j);
            const u32 cnt = nd.b;
            if (nd.type != MTE_OP_LOAD_NODE || cnt == 0 || cnt > 7) {
                fail(MTE_DOC_CAPACITY, end.seq);
                return;
            }
            if ((u32)nd.a != lvl) {  // next level up: its children are the nodes just made
                if ((u32)nd.a != lvl + 1 || cur != nBelow) {
                    fail(MTE_DOC_CAPACITY, end.seq);
                    return;
                }
                lvl++;
                below = first;
                nBelow = made;
                cur = 0;
                first = NONE;
                made = 0;
            }
            const u32 id = alloc_in();
            if (id == NONE) return;
            if (first == NONE) first = id;
            if (id != first + made || cur + cnt > nBelow) {  // a fresh document's ids are consecutive
                fail(MTE_DOC_CAPACITY, end.seq);
                return;
            }
            if (L < cnt) {
                const u32 child = below == NONE ? ORD()[cur + L].x : below + cur + L;
                INCH()[id * 8 + L] = child;
                if (below == NONE) set_bpar_lane(child, id);
                else if (child < in_cap()) INPAR()[child] = id;
            }
            if (L == 0) INCNT()[id] = cnt;
            sync();
            cur += cnt;
            made++;
            last = id;
        }
        if (nn && (cur != nBelow || made != 1)) {  // every node linked, one root
            fail(MTE_DOC_CAPACITY, end.seq);
            return;
        }
        st.root = nn ? last : U(ORD()[0].x);
        st.height = nn ? lvl + 1 : 1u;
        st.curSeq = end.seq;
        st.minSeq = end.msn;
        sync();
    }

    // Client.applyMsg for one op record (client.ts:805-836): the edit, zamboni, then
    // updateSeqNumbers / setMinSeq (client.ts:829-836, mergeTree.ts:1718-1736) and zamboni again
    // when the MSN advanced. One zamboni call site.
    // LOAD_APPEND position (snapshotLoader.ts:184-213, blockInsert mergeTree.ts:2193-2223): pos =
    // root.cachedLength (every segment not removed) at the first segment of an append call, then
    // advanced by each segment's length whether it is linked or skipped; the running position is a
    // per-document counter, so it survives a hand-off to an HBM slot between two records. A repeated
    // object (flushBatch never clears its batch, :196-199) is re-linked by the reference when its walk
    // finds pos -- one object in two places, which this engine does not model (MTE_DOC_UNSUPPORTED)
    // -- and skipped otherwise. Returns true when the segment is to be inserted at p1.
    MTE_DEV bool load_append_pos(const mte_op& op, Seg& rec, i32& p1) {
        const bool rm = (op.flags & MTE_F_LOAD_REMOVED) != 0;
        if (st.root == NONE || (rm && (u32)op.pos1 >= MTE_MAX_CLIENTS)) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return false;
        }
        // one length scan serves both questions: root.cachedLength (the observer's view) for the first
        // segment of a call, and for a repeated object whether the walk finds pos (pos <= the length
        // of the (refSeq 0, client) view)
        const bool first = (op.flags & MTE_F_APPEND_FIRST) != 0, repeat = (op.flags & MTE_F_APPEND_REPEAT) != 0;
        i32 pos = first ? 0 : (i32)stat_get(ST_APPEND);
        i32 viewLen = 0;
        for (u32 q = first ? 0u : 1u; q < (repeat ? 2u : 1u); q++) {
            const i32 n = get_length(q ? 0 : st.curSeq, q ? (u32)op.client : 0u);
            pos = q ? pos : n;
            viewLen = n;
        }
        sync();
        if (L == 0) STATS()[ST_APPEND] = (u32)(pos + (i32)rec.len);
        sync();
        if (rec.len == 0) return false;
        if (repeat) {
            if (pos <= viewLen) fail(MTE_DOC_UNSUPPORTED, op.seq);
            return false;
        }
        if (rm) {
            rec.rseq = op.ref_seq;
            rec.meta |= ((((u32)op.pos1 & 0xffu) << 8) | F_REMOVED);
        }
        p1 = pos;
        return true;
    }

    MTE_DEV void apply(const mte_op& op_in, u64 op_index) {
        MTE_PROF(PF_APPLY);
        MTE_COUNT(PF_OPS, 1);
        mte_op op = op_in;
#ifdef MTE_PROFILE
        const u64 t_op0 = (MTE_PON(PF_OP_INS) || MTE_PON(PF_OP_REM)) ? __builtin_amdgcn_s_memtime() : 0;
        struct OpScope {
            u64* acc; u64 t0; u32 L;
            MTE_DEV ~OpScope() {
                if ((MTE_PON(PF_OP_INS) || MTE_PON(PF_OP_REM)) && L == 0) atomicAdd(acc, __builtin_amdgcn_s_memtime() - t0);
            }
        } _op_scope{prof + (op.type == MTE_OP_REMOVE ? PF_OP_REM : PF_OP_INS), t_op0, L};
        MTE_COUNT(op.type == MTE_OP_REMOVE ? PN_REM : PN_INS, 1);
#endif
#ifdef MTE_PROFILE
        u64 t_pre = MTE_PON(PF_APRE) ? __builtin_amdgcn_s_memtime() : 0;
#endif
        // a loadBody append of a summary load (include/mte.h MTE_OP_LOAD_APPEND) shares the insert
        // path: insertSegments(pos, [seg], refSeq 0, client, seq) with the segment's own merge info
        const bool ld = op.type == MTE_OP_LOAD_APPEND;
        if (op.client >= MTE_MAX_CLIENTS) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        const u32 C = collab ? (u32)op.client : 0u;
        const i32 seq = collab ? op.seq : 0;
        const i32 R = collab && !ld ? op.ref_seq : 0;
        if constexpr (EXT) zseq = op.seq;  // the time of this op's UNLINKs (ht_free)
        if (collab && op.type != MTE_OP_NOOP && !ld && !(st.curSeq < op.seq)) {
            fail(MTE_DOC_SEQ_ORDER, op.seq);
            return;
        }
        if constexpr (EXT) {
            if (op.type == MTE_OP_CELL) {  // no merge-tree op, no seq / msn movement (include/mte.h)
                cell_op(op, R, C);
                return;
            }
        }
        if constexpr (FULL) {  // relative positions need marker ids, i.e. properties
            if (op.flags & MTE_F_REL) {
                if (!rel_positions(op, op_index, R, C)) return;
            }
        }
        bool edited = false;
        if (op.type <= MTE_OP_INSERT_MARKER || ld) {
            Seg rec;
            const bool mk = ld ? (op.flags & MTE_F_LOAD_MARKER) != 0 : op.type == MTE_OP_INSERT_MARKER;
            const bool ins = op.type == MTE_OP_INSERT || mk || ld;
            rec.len = mk ? 1u : op.b;
            rec.seq = seq;
            rec.rseq = 0;
            rec.meta = (C & 0xff) | (mk ? F_MARKER : 0u) | ((EXT && (op.flags & MTE_F_PERM)) ? F_PERM : 0u);
            u32 type = op.type;
            i32 p1 = op.pos1;
            if (ld && !load_append_pos(op, rec, p1)) return;  // skipped (a repeated object) or failed
            type = ld ? (mk ? (u32)MTE_OP_INSERT_MARKER : (u32)MTE_OP_INSERT) : type;
            rec.props = (ins && op.props) ? build_map(0, op.props, false) : 0u;
            if (st.status) return;
            // (a PermutationSegment run: handles unallocated on insert -- onDelta's reset -- kept when loaded)
            rec.toff = (mk && !ld) ? op.b : ((rec.meta & F_PERM) && !ld ? 0u : (u32)op.a);
            rec.tcap = 0;
            rec.sid = 0;
            const bool cu = EXT && (op.flags & MTE_F_CATCHUP) != 0 && !ld;  // EXT batches only
            if (cu) {
                sync();
                if (L == 0) STATS()[ST_CUOP] = (u32)(op_index - p.docs[doc].op_begin);
                sync();
            }
#ifdef MTE_PROFILE
            if (MTE_PON(PF_APRE) && L == 0) atomicAdd(prof + PF_APRE, __builtin_amdgcn_s_memtime() - t_pre);
#endif
            edited = edit(type, p1, op.a, R, C, seq, rec, op.props, (op.flags & MTE_F_REWRITE) != 0, cu);
            if (!ld) stat_add(ST_OPS, 1);
            if (st.status) return;
        }
#ifdef MTE_PROFILE
        MTE_PROF(PF_APOST);
#endif
        for (u32 z = 0; z < 2; z++) {
            bool run = edited;
            if (z == 1) {
                run = false;
                if (collab && (op.flags & MTE_F_END_OF_MSG)) {
                    stat_add(ST_MSGS, 1);
                    if (op.seq < st.curSeq || op.msn > op.seq || op.msn < st.minSeq) {
                        fail(MTE_DOC_SEQ_ORDER, op.seq);
                        return;
                    }
                    st.curSeq = op.seq;
                    if (op.msn > st.minSeq) {
                        st.minSeq = op.msn;
                        run = true;
                    }
                }
            }
            if (run) {
#ifdef MTE_PROFILE
                ProfScopeT<MTE_PON(PF_ZAM_EDIT) || MTE_PON(PF_ZAM_MSN)> _zs(prof + (z == 0 ? PF_ZAM_EDIT : PF_ZAM_MSN));
#endif
                zamboni();
            }
            if (st.status) return;
        }
    }

    // ---------------------------------------------------------------- driver
    MTE_DEV void init() {
        if constexpr (EXT) ht_reset();
        u32 r = alloc_lb();
        st.root = r;
        st.height = 1;
        if (r == NONE) return;
        if (L == 0) ORD()[0] = make_uint4(r, 0, 0, 0);
        st.n_lb = 1;
        stat_max(ST_MAXLB, 1);
        sync();
    }

    // LDS mode: give every leaf block this wave holds back to the CU's pool (also after an
    // abandoned replay, whose blocks need not all be linked).
    MTE_DEV void release() {
        if (!SHARED) {
            st.n_lb = 0;
            return;
        }
        u32 n = 0;
        for (u32 base = 0; base < blk_cap(); base += 64) {
            const u32 b = base + L;
            const bool mine = b < blk_cap() && OWNER()[b] == (unsigned char)wave;
            if (mine) {
                OWNER()[b] = 0xFF;
                atomicAnd(&BITMAP()[b >> 5], ~(1u << (b & 31)));
            }
            n += (u32)__builtin_popcountll(wave_ballot(mine));
        }
        n += st.credit;
        if (L == 0 && n) atomicAdd(POOLAV(), n);
        st.credit = 0;
        st.n_lb = 0;
        sync();
    }

    // Results + the final segments in doc order (walkAllSegments, mergeTree.ts:2969-2983).
    // The text of every row is gathered into the document's run of the output text pool (the
    // row's aux.y becomes its offset in that run) and its property map is copied beside it, so the
    // host reads final state only: rows, maps and text, never the op log, payload, arena or map
    // region.
    MTE_DEV u32 block_text(uint4 o) const {  // text units of the block held by this lane
        u32 t = 0;
        const u32 c = o.w > 8 ? 8u : o.w;
        for (u32 s = 0; s < c; s++) {
            const uint4 v = VIS()[o.x * 8 + s];
            t += (v.w & (F_MARKER | F_PERM)) ? 0u : v.x;
        }
        return t;
    }
    MTE_DEV void finish() {
        fence_ovl();
        u32 nseg = 0, ntext = 0;
        for (u32 base = 0; base < st.n_lb; base += 64) {
            u32 k = base + L;
            const uint4 o = k < st.n_lb ? ORD()[k] : make_uint4(0, 0, 0, 0);
            nseg += wave_sum(o.w);
            ntext += wave_sum(k < st.n_lb ? block_text(o) : 0u);
        }
        u32 off = 0, toff = 0;
        if (st.status == 0) {
            if (L == 0) {
                off = atomicAdd(&p.counters[1], nseg);
                toff = (u32)atomicAdd((unsigned long long*)&p.counters[6], (unsigned long long)ntext);
            }
            off = wave_read(off, 0);
            toff = wave_read(toff, 0);
            if ((u64)off + nseg > p.out_cap || (u64)toff + ntext > p.out_text_cap) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                nseg = 0;
            }
        } else {
            nseg = 0;
        }
        if (nseg) {
            wave_sync();  // overlap masks, merge-arena text and property maps written by other lanes
            st.gdirty = st.adirty = 0;
            u32 run = off, trun = 0;
            u16* __restrict__ tdst = p.out_text + toff;
            for (u32 base = 0; base < st.n_lb; base += 64) {
                const u32 k = base + L;
                uint4 o = k < st.n_lb ? ORD()[k] : make_uint4(0, 0, 0, 0);
                const u32 c = o.w > 8 ? 8u : o.w;
                const u32 incl = wave_scan_incl(c);
                const u32 bt = k < st.n_lb ? block_text(o) : 0u;
                const u32 tincl = wave_scan_incl(bt);
                u32 at = run + incl - c;
                u32 tat = trun + tincl - bt;
                for (u32 s = 0; s < c; s++) {
                    uint4 v = VIS()[o.x * 8 + s], a = AUX()[o.x * 8 + s];
                    if (!(v.w & (F_MARKER | F_PERM))) {  // wave-divergent copy, 8 units in flight per lane
                        const u16* __restrict__ src = text_ptr(a.y);
                        u16* __restrict__ dst = tdst + tat;
                        for (u32 i = 0; i < v.x; i += 8) {
                            u16 t[8];
#pragma unroll
                            for (u32 j = 0; j < 8; j++) t[j] = i + j < v.x ? src[i + j] : (u16)0;
#pragma unroll
                            for (u32 j = 0; j < 8; j++)
                                if (i + j < v.x) dst[i + j] = t[j];
                        }
                        a.y = tat;  // offset in the document's text run
                        tat += v.x;
                    }
                    if (a.x && p.out_maps) {  // the row's property map, indexed by row
                        const uint4* ms = (const uint4*)(maps + (u64)a.x * mw);
                        uint4* md = (uint4*)(p.out_maps + (u64)(at + s) * mw);
                        const uint4 m0 = ms[0], m1 = ms[1], m2 = ms[2], m3 = ms[3];
                        md[0] = m0;
                        md[1] = m1;
                        md[2] = m2;
                        md[3] = m3;
                        for (u32 q = 4; q < mw / 4; q++) md[q] = ms[q];  // wider records
                    }
                    p.out_vis[at + s] = v;
                    p.out_aux[at + s] = a;
                    u64 m = (v.w & F_OVL) ? (u64)a.z : 0ull;
                    if ((v.w & F_OVLHI) && a.w < seg_cap) m |= ovl[a.w] & 0xFFFFFFFF00000000ull;
                    p.out_ovl[at + s] = m;
                    if (p.out_ovl2) p.out_ovl2[at + s] = (ovl2 && (v.w & F_OVLHI) && a.w < seg_cap) ? ovl2[a.w] : 0ull;
                }
                run += wave_read(incl, 63);
                trun += wave_read(tincl, 63);
            }
        }
        const u32 fseq = stat_get(ST_FAILSEQ), ops = stat_get(ST_OPS), msgs = stat_get(ST_MSGS);
        const u32 ngc = stat_get(ST_GC), maxlb = stat_get(ST_MAXLB), ncu = stat_get(ST_CU);
        if (L == 0) {
            DocRes& o = p.res[doc];
            o.status = st.status;
            o.failing_seq = (i32)fseq;
            o.ops = ops;
            o.msgs = msgs;
            o.min_seq = st.minSeq;
            o.cur_seq = st.curSeq;
            o.height = st.height;
            o.n_lb = st.n_lb;
            o.arena_sel = st.arenaSel;
            o.arena_top = st.arenaTop;
            o.map_next = st.mapNext;
            o.seg_next = st.segNext;
            o.heap_size = st.heapSize;
            o.n_gc = ngc;
            o.out_off = off;
            o.n_segs = nseg;
            o.text_off = toff;
            o.max_lb = maxlb;
            o.cu_n = ncu;
            o.mode = SOLO ? 3u : (LDSM ? 0u : (from_rows ? 6u : continued ? 2u : 1u));
        }
    }

    MTE_DEV void mark_spilled() {
        const u32 maxlb = stat_get(ST_MAXLB);
        if (L == 0) {
            DocRes& o = p.res[doc];
            o.status = DOC_SPILL;
            o.failing_seq = st.curSeq;
            o.n_segs = 0;
            o.max_lb = maxlb;
            o.mode = 0;
            o.spill_why = (st.n_lb << 8) | (st.heapSize << 20) | (st.inUsed & 0xff);
            atomicAdd(&p.counters[2], 1u);
        }
    }

    // One op record from the LDS ring, made wave-uniform (SGPRs).
    MTE_DEV static mte_op read_op(const mte_op* rp) {
        const uint4* q = (const uint4*)rp;
        const uint4 a = q[0], b = q[1];
        u32 w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        for (int i = 0; i < 8; i++) w[i] = wave_first(w[i]);
        mte_op op;
        __builtin_memcpy(&op, w, sizeof op);
        return op;
    }

    // Replay ops [i, end) of the doc's log. Returns the index of the first op not applied:
    // end when done; earlier when the LDS plan ran out of room before that op (the document then
    // continues HBM-resident from there) or on a failure (st.status).
    MTE_DEV u64 replay_run(u64 i) {
#ifdef MTE_PROFILE
        MTE_PROF(PF_TOTAL);
#endif
        const u64 e = p.docs[doc].op_end;
        // summary records (resume from a summary) precede the op log: a cold prefix loop, so the op
        // loops below carry no branch for them
        for (; i < e && !st.status; i++) {
            const mte_op op = read_op(p.ops + i);
            if (op.type < MTE_OP_LOAD_SEG || op.type >= MTE_OP_LOAD_APPEND) break;
            if (!room()) return i;
            load_record(op, i);
        }
        const u64 b = i;
        if (LDSM) {
            // op records are staged RING_OPS at a time through LDS; the next batch is prefetched
            // into registers one batch ahead (lane l holds 16 B of record l/2 of the batch).
            const uint4* src = (const uint4*)(p.ops);
            uint4* dst = (uint4*)RING();
            uint4 nxt = make_uint4(0, 0, 0, 0);
            if (b + (L >> 1) < e) nxt = src[b * 2 + L];
            for (; i < e && !st.status; i++) {
                const u32 r = (u32)((i - b) & (RING_OPS - 1));
                if (r == 0) {
                    sync();
                    dst[L] = nxt;
                    sync();
                    const u64 nb = i + RING_OPS;
                    if (nb + (L >> 1) < e) nxt = src[nb * 2 + L];
                }
                mte_op op;
                {
                    MTE_PROF(PF_FETCH);
                    op = read_op(RING() + r);
                }
                {
                    MTE_PROF(PF_LOOP);
                    if (!room()) break;
                }
                apply(op, i);
            }
        } else {
            for (; i < e && !st.status; i++) {
                mte_op op = p.ops[i];
                apply(op, i);
            }
        }
        return i;
    }

    // ---------------------------------------------------------------- continue HBM-resident
    // Engine<false>: copy an LDS-resident document's state (block ids, interior nodes, heap and
    // counters unchanged; fresh block ids start above the LDS pool's).
    template <class E>
    MTE_DEV void adopt(const E& e) {
        st = e.st;
        st.lbBump = e.blk_cap();
        st.lbFree = NONE;
        st.credit = 0;
        const u32 g = L >> 3, s = L & 7;
        for (u32 base = 0; base < st.n_lb; base += 8) {
            const u32 k = base + g;
            if (k < st.n_lb) {
                const u32 blk = e.ORD()[k].x;
                m_vis[blk * 8 + s] = e.VIS()[blk * 8 + s];
                m_aux[blk * 8 + s] = e.AUX()[blk * 8 + s];
                if (s == 0) m_bmeta[blk] = e.BMETA()[blk];
            }
        }
        for (u32 k = L; k < st.n_lb; k += 64) m_ord[k] = e.ORD()[k];
        for (u32 q = L; q < st.inBump * 8; q += 64) m_in_child[q] = e.INCH()[q];
        for (u32 n = L; n < st.inBump; n += 64) {
            m_in_cnt[n] = e.INCNT()[n];
            m_in_par[n] = e.INPAR()[n];
        }
        for (u32 h = 1 + L; h <= st.heapSize; h += 64) m_heap[h] = e.HEAP()[h];
        if (L < ST_WORDS) m_stats[L] = e.STATS()[L];
        wave_sync();
    }

    // Synthetic workload generator: simulated writers draw valid ops from their own
    // view (getLength(refSeq, client)); each op is recorded into the doc's op/payload slots and
    // applied immediately, so the recorded log is exactly what a replay will see. The writers'
    // state lives in GenState so a document that leaves the LDS plan continues HBM-resident.
    MTE_DEV void gen_init(GenState& g) const {
        // seeded by the GLOBAL document id, so a document is the same whichever rank generates it
        const u64 sx = 0xF1D0C0DEull ^ (u64)p.docs[doc].gid ^ (p.gen_seed * 0x9E3779B97F4A7C15ull);
        g.rng.seed(sx);
        for (u32 c = 0; c < GEN_MAX_CLIENTS; c++) {
            g.ref[c] = 0;
            g.sid_of[c] = 0;
        }
        g.nextShort = 1;
        g.pay = 0;
        g.lastC = -1;
        g.lastR = 0;
        g.lastPos = 0;
        g.step = 0;
    }
    // Returns true when every op was generated (or the doc failed), false when the LDS plan ran out
    // of room before op g.step.
    MTE_DEV bool generate_run(GenState& g) {
        const u32 nc = p.gen_nclients;
        u32* firstSeen = p.gen_first_seen + (u64)doc * GEN_MAX_CLIENTS;
        const u64 op0 = p.docs[doc].op_begin;
        const u64 nops = p.docs[doc].op_end - op0;
        for (; g.step < nops && !st.status; g.step++) {
            if (!room()) return false;
            const u64 step = g.step;
            const i32 seq = (i32)step + 1;
            const i32 cur = seq - 1;
            // the draws below consume the generator in a fixed order (no early outs)
            Rng rng = g.rng;
            const u32 c = rng.below(nc);
            if (rng.below(4) == 0) g.ref[c] = cur;
            else {
                i32 nr = g.ref[c] + (i32)rng.below(5);
                g.ref[c] = nr < cur ? nr : cur;
            }
            if (p.gen_kind == 5 && g.ref[c] < cur - 64) g.ref[c] = cur - 64;
            bool forced = false;
            if (p.gen_kind == 3 && g.lastC >= 0 && (u32)g.lastC != c && rng.below(100) < 15 && g.lastR >= g.ref[c]) {
                g.ref[c] = g.lastR;  // replay a recent other-client op's refSeq and position
                forced = true;
            }
            if (g.sid_of[c] == 0) {
                g.sid_of[c] = g.nextShort++;
                if (L == 0) firstSeen[g.sid_of[c]] = c;
            }
            const u32 C = g.sid_of[c];
            const i32 R = g.ref[c];
            const i32 len = get_length(R, C);
            const u32 roll = rng.below(100);
            u32 type;
            if (len == 0) type = MTE_OP_INSERT;
            else if (p.gen_kind == 3) type = roll < 45 ? MTE_OP_INSERT : (roll < 80 ? MTE_OP_REMOVE : MTE_OP_ANNOTATE);
            else type = roll < (len < 2048 ? 60u : 40u) ? MTE_OP_INSERT : MTE_OP_REMOVE;
            mte_op op;
            op.seq = seq;
            op.ref_seq = R;
            op.client = (uint8_t)C;
            op.flags = MTE_F_END_OF_MSG;
            op.props = 0;
            op.b = 0;
            op.type = (uint8_t)type;
            if (type == MTE_OP_INSERT) {
                const i32 pos = forced ? (g.lastPos < len ? g.lastPos : len) : (i32)rng.below((u32)len + 1);
                const u32 n = 1 + rng.below(8);
                op.pos1 = pos;
                op.a = (i32)g.pay;
                op.b = n;
                for (u32 i = 0; i < n; i++) {
                    const u16 ch = (u16)(u'a' + rng.below(26));
                    if (L == 0) payload[g.pay + i] = ch;
                }
                g.pay += n;
                st.adirty = 1;  // later cross-lane text copies read these chars
                if (p.gen_kind == 3 && rng.below(4) == 0) op.props = 1 + rng.below(p.gen_n_propsets);
            } else {
                const i32 a = forced ? (g.lastPos < len ? g.lastPos : len - 1) : (i32)rng.below((u32)len);
                const i32 n = 1 + (i32)rng.below(16);
                op.pos1 = a;
                op.a = a + n < len ? a + n : len;
                if (type == MTE_OP_ANNOTATE) op.props = 1 + rng.below(p.gen_n_propsets);
            }
            i32 msn = g.ref[0];
            for (u32 q = 1; q < nc; q++) msn = g.ref[q] < msn ? g.ref[q] : msn;
            op.msn = msn;
            g.lastC = (i32)c;
            g.lastR = R;
            g.lastPos = op.pos1;
            g.rng = rng;
            if (L == 0) p.ops[op0 + step] = op;
            apply(op, 0);
        }
        wave_sync();  // op records and payload visible before the replay kernel
        return true;
    }
};

}  // namespace mte
