// reg_engine.hpp — the row-vectorised replay engine for critical-path documents (k_solo).
//
// Same observer replay as engine.hpp (@fluidframework/merge-tree 0.31.0; paths relative to
// packages/dds/merge-tree/src), same B-tree shape and lazy zamboni schedule, restructured so that one
// op is a short run of wave-wide instructions with few dependent memory round trips:
//   * leaf blocks in DOCUMENT ORDER, 8 per "row": block k's slot s is lane 8*(k&7)+s of row k>>3.
//     A row is 64 slots = 64 lanes, held in LDS exactly where the LDS engine's SoloPlan keeps slots
//     (vis = len, seq, removedSeq, meta; aux = -, text offset, text capacity / overlap mask,
//     segment id): one ds_read_b128 per lane fetches a whole row's visibility fields. An empty slot
//     has len 0 (segments are never empty), so a block's child count is a popcount of one ballot;
//   * position resolution (insertingWalk + nodeLength, mergeTree.ts:2345-2474,1659-1699): per row
//     ONE predicate evaluation for 64 slots and ONE DPP prefix scan; the first block whose
//     cumulative end reaches pos wins (blocks win ties, :2274-2276), then the slot inside it
//     (breakTie, :2248-2277) from the same registers. No per-block summaries to maintain;
//   * edits of a block are lane-parallel on its row (DPP shifts inside the 8-lane group); a block
//     split or pack moves the blocks after it as one LDS memmove;
//   * interior B-tree levels as child-COUNT vectors in VGPRs (lane = node at that level, document
//     order): a parent is a prefix-sum lookup, a split 8 -> 4+4 a one-lane shift (mergeTree.ts:
//     2446-2489, 1876-1887), pack a redistribution of counts (:1368-1420);
//   * needsScour tri-state (mergeTree.ts:63,1279) in spare meta bits of every slot of its block, so
//     it moves with the block;
//   * the LRU heap (collections.ts:213-265) in 2 x 8 VGPRs, positions 1..511;
//   * op records prefetched 8 per VGPR, decoded with v_readlane.
// Text stays in HBM (the op payload and the merge arena), as in engine.hpp. Live segments carry
// removedSeq RSEQ_LIVE and removedClient RCL_LIVE so the visibility predicate needs no removed test.
// A document whose state outgrows this plan, or that reaches an op this engine does not implement
// (annotate, summary load records, relative positions, legacy catch-up, permutation runs), hands its
// state to the LDS engine between two ops (reg_handoff.hpp) and continues there.
// The same source also builds for the CPU (wave_simd.hpp MTE_CPU): the CPU suite checks it against
// the oracle (tests/test_reg_engine_cpu.py); the product runs the device build only.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "engine_types.hpp"
#include "wave_simd.hpp"

namespace mte {

constexpr u32 RG_ROWS = 32;               // slot rows
constexpr u32 RG_BLOCKS = RG_ROWS * 8;    // leaf blocks
constexpr u32 RG_LEVELS = 8;              // interior levels (height <= RG_LEVELS + 1)
constexpr u32 RG_HEAP = 511;              // LRU heap positions 1..511
constexpr u32 RSEQ_LIVE = 0x7FFFFFFFu;    // removedSeq of a live segment (never <= a refSeq)
constexpr u32 RCL_LIVE = 0xFFu;           // removedClient byte of a live segment (never a client)
constexpr i32 REG_HANDOFF = 101;          // internal: continue in the LDS engine from the current op
constexpr u32 ROWS_POOL_WORDS = 3;         // k_rows' pool row mask (mte_solo.hip RowsGeom): <= 96 rows
constexpr u32 ROWS_WAIT_TRIES = 20000;     // a wave finding the pool full retries this often (s_sleep 8)
// needsScour (mergeTree.ts:63) in meta bits 24..25 of every slot lane of a block
constexpr u32 NS_SHIFT = 24, NS_MASK = 3u << NS_SHIFT;
static_assert(RG_BLOCKS <= SOLO_POOL, "the rows live in the SoloPlan's slot arrays");

// Phase profile of the row engine (MTE_PROFILE device builds, `make prof`): inclusive s_memtime
// cycles and event counts accumulated in registers and written once per document by finish(), in
// the LDS engine's slot numbering (engine.hpp ProfSlot, mte.PROF_NAMES).
enum RgProf : u32 {
    RP_TOTAL, RP_FETCH, RP_APPLY, RP_RESOLVE, RP_INSERT_SLOT, RP_SPLIT, RP_RANGE, RP_ZAMBONI, RP_SCOUR,
    RP_HEAP, RP_FIND_SEG, RP_PACK, RP_LRU, RP_OPS, RP_N_RESOLVE, RP_N_SCOUR, RP_N_SCOUR_CHANGED,
    RP_N_PACK, RP_N_POP, RP_N_SPLIT_BLK, RP_N_MOVE, RP_SPLIT_AT, RP_INS, RP_REM, RP_MSN, RP_ZAM_EDIT, RP_N
};
#if defined(MTE_PROFILE) && !defined(MTE_CPU)
// RG_PROF_ONLY=<slot>: time that one scope only (each s_memtime pair costs a lone wave ~100 cycles,
// which a full profile charges to the enclosing scopes); RP_TOTAL and the event counts stay on
#ifdef RG_PROF_ONLY
#define RG_ON(slot) ((slot) == RG_PROF_ONLY || (slot) == RP_TOTAL)
#else
#define RG_ON(slot) true
#endif
template <bool ON>
struct RgScope {
    u64& acc;
    u64 t0;
    __device__ __forceinline__ RgScope(u64& a) : acc(a), t0(ON ? __builtin_amdgcn_s_memtime() : 0) {}
    __device__ __forceinline__ ~RgScope() {
        if (ON) acc += __builtin_amdgcn_s_memtime() - t0;
    }
};
#define RG_PROF(slot) RgScope<RG_ON(slot)> _rg_scope_##slot(pf[slot])
#define RG_COUNT(slot, n) (pf[slot] += (u64)(n))
#elif defined(MTE_MARKERS) && !defined(MTE_CPU)
// static code inspection: row-engine scopes as assembly comments "MTE_BEGIN 100+slot"
template <u32 S>
struct RgMark {
    __device__ __forceinline__ RgMark() { asm volatile("; MTE_BEGIN %0" ::"i"(S + 100)); }
    __device__ __forceinline__ ~RgMark() { asm volatile("; MTE_END %0" ::"i"(S + 100)); }
};
#define RG_PROF(slot) RgMark<slot> _rg_mark_##slot
#define RG_COUNT(slot, n) \
    do {                  \
    } while (0)
#else
#define RG_PROF(slot) \
    do {              \
    } while (0)
#define RG_COUNT(slot, n) \
    do {                  \
    } while (0)
#endif

// Event statistics of the CPU build (MTE_CPU_STATS, tools/rg_stats.py only): what the critical
// document's ops do (rows a resolve scans, heap sizes at a pop, scour outcomes), to size the device
// code paths. Nothing in a device build.
#if defined(MTE_CPU) && defined(MTE_CPU_STATS)
enum RgStat : u32 {
    RS_OPS, RS_RESOLVE, RS_RES_ROWS, RS_RES_NROWS, RS_POP, RS_POP_BIG, RS_POP_HEAP, RS_FIND_ROWS, RS_SCOUR,
    RS_SCOUR_NOP, RS_SCOUR_SERIAL, RS_SCOUR_COPY, RS_PACK, RS_SPLIT_BLK, RS_MOVE_SLOTS, RS_SPLIT_AT,
    RS_ZAM_CALLS, RS_ZAM_POPS, RS_LRU_PUSH, RS_RANGE_ROWS, RS_N
};
inline u64 g_rg_stats[RS_N + 64];
#define RG_STAT(i, n) (g_rg_stats[i] += (u64)(n))
#else
#define RG_STAT(i, n) \
    do {              \
    } while (0)
#endif

#ifndef MTE_CPU
extern __shared__ uint4 g_lds_dyn[];
#endif

struct RSeg {
    u32 len;
    i32 seq;
    u32 rseq;
    u32 meta;
    u32 toff;
    u32 cap;  // owned merge-arena capacity from toff (0 for payload text)
    u32 rm;   // removers: bit c for removedClient c and every client in removedClientOverlap
    u32 sid;
    u32 props = 0;  // property map id (PROPS engines; 0 = no properties)
    u32 rm2 = 0;    // removers 32..63 (WIDE engines)
};
// the extra slot fields of a PROPS engine's rows (the property map id) and of a WIDE one's (removers
// 32..63); absent otherwise: the lean rows stay eight registers
template <bool P, bool W>
struct RowProps {};
template <>
struct RowProps<true, false> {
    simd::V props;
};
template <>
struct RowProps<false, true> {
    simd::V rm2;
};
template <>
struct RowProps<true, true> {
    simd::V props, rm2;
};
struct RFound {
    bool ok;
    u32 k;     // leaf block (document order)
    u32 cnt;   // its child count
    i32 slot;  // first qualifying slot, -1 => append at the block end
    i32 r;     // pos - cumBefore(slot)
    u32 row;   // the row of block k
    u32 carry; // visible length before that row
};

// PAGED (k_rows): logical row r of the document lives in pool row ptab[r] of a pool the CU's waves
// share (rows_pool_*), taken as the document grows and given back as it shrinks or ends; a document
// the pool cannot grow is spilled (REG_HANDOFF, re-run by the host). Otherwise row r is slot row r.
// PROPS (k_rows of property-carrying batches): a ninth slot field, the segment's property map id
// (immutable maps in the document's HBM map table, SegmentPropertiesManager.addProperties), annotate
// ops, and merges that require matching properties.
// WIDE (k_solo's property-carrying instantiation): clients 32..63 too, a second removers word per slot.
template <int NR = (int)RG_ROWS, bool PAGED = false, bool PROPS = false, bool WIDE = false>
struct RegEngine {
    static constexpr bool kProps = PROPS, kWide = WIDE;
    static constexpr u32 MAXC = WIDE ? 64u : 32u;  // client ids below this (rm, rm2)
    typedef simd::V V;
    typedef simd::B B;
    static constexpr u32 NBLK = (u32)NR * 8;
    // One row of slots: vis = (len, seq, rseq, meta), aux = (cap, toff, rm, sid). A live segment has
    // rm 0, so nodeLength's removal test is one bit test of rm (no separate overlap-set lookup).
    struct Row : RowProps<PROPS, WIDE> {
        V len, seq, rseq, meta, cap, toff, rm, sid;
    };

    // ---------------------------------------------------------------- state
    simd::VA<RG_LEVELS> LV;  // LV[i] lane j: child count of node j of level i+1 (0 beyond the last)
    // Heap positions q at lane q&63 of register q>>6. Registers 0 and 1 (positions 1..127, every pop
    // of a heap that size) are plain values; 2..7 an indexed array touched only by larger heaps (one
    // 8-register array made every pop copy all eight registers at its merge points).
    struct HeapRegs {
        V r0, r1, x2, x3, x4, x5, x6, x7;  // named registers: no access is ever indexed at run time
        SD V get(u32 i) const {
            switch (i) {
                case 0: return r0;
                case 1: return r1;
                case 2: return x2;
                case 3: return x3;
                case 4: return x4;
                case 5: return x5;
                case 6: return x6;
                default: return x7;
            }
        }
        SD void set(u32 i, V v) {
            switch (i) {
                case 0: r0 = v; break;
                case 1: r1 = v; break;
                case 2: x2 = v; break;
                case 3: x3 = v; break;
                case 4: x4 = v; break;
                case 5: x5 = v; break;
                case 6: x6 = v; break;
                default: x7 = v; break;
            }
        }
        SD void zero() { r0 = r1 = x2 = x3 = x4 = x5 = x6 = x7 = simd::splat(0); }
    };
    HeapRegs HK, HS;         // heap keys (maxSeq) / segment ids
    u32 n_lb, height, heapSize, segNext, arenaTop, arenaSel;
    i32 minSeq, curSeq, heapTop, status, failSeq;
    u32 n_gc, max_lb;
    u32 n_ops, n_msgs;
    SD u32 ops_n() const { return n_ops; }
    SD u32 msgs_n() const { return n_msgs; }
    SD void set_counts(u32 o, u32 m) {
        n_ops = o;
        n_msgs = m;
    }
    SD void count_op() { n_ops++; }
    SD void count_msg() { n_msgs++; }
    u32 lb_lim;  // leaf-block limit of room() (Params::reg_lb_limit, read once)
    bool adirty;
#if defined(MTE_PROFILE) && !defined(MTE_CPU)
    u64 pf[RP_N];
#endif
    // per document
    const Params& p;
    u32 doc;
    u16* payload;
    u16* arena0;
    u32 seg_cap, arena_cap, payload_len;

    // ---------------------------------------------------------------- slot rows (LDS)
    // ---------------------------------------------------------------- paged rows
    V ptab = simd::splat(0);  // lane r: pool row of logical row r (PAGED)
    u32 n_rows = 0;           // logical rows taken from the pool (PAGED)
    SD u32 prow(u32 r) const {
        if constexpr (PAGED) return simd::readlane(ptab, r);
        else return r;
    }
#ifdef MTE_CPU
    u32 mem_vis[RG_ROWS * 64][4], mem_aux[RG_ROWS * 64][4];
    u32 mem_props[RG_ROWS * 64], mem_rm2[RG_ROWS * 64];
    u64 pool_mask = 0;           // PAGED: pool rows in use (this engine's own pool on the CPU)
    u32 pool_rows = RG_ROWS, pool_takes = 0;
    SD u32 pslot(u32 s) const { return PAGED ? prow(s >> 6) * 64 + (s & 63) : s; }
    SD bool take_row(u32& row) {  // a scattered order, so logical and pool rows differ
        for (u32 t = 0; t < pool_rows; t++) {
            const u32 c = (pool_takes * 7 + 3 + t) % pool_rows;
            if (!((pool_mask >> c) & 1)) {
                pool_mask |= 1ull << c;
                pool_takes++;
                row = c;
                return true;
            }
        }
        return false;
    }
    SD void give_row(u32 row) { pool_mask &= ~(1ull << row); }
    SD void zero_prow(u32 row) {
        memset(mem_vis[row * 64], 0, 64 * 16);
        memset(mem_aux[row * 64], 0, 64 * 16);
        memset(&mem_props[row * 64], 0, 64 * 4);
        memset(&mem_rm2[row * 64], 0, 64 * 4);
    }
    SD Row ldrow(u32 r) const {
        Row w;
        const u32 pr = prow(r);
        for (u32 l = 0; l < 64; l++) {
            const u32* v = mem_vis[pr * 64 + l];
            const u32* a = mem_aux[pr * 64 + l];
            w.len.x[l] = v[0], w.seq.x[l] = v[1], w.rseq.x[l] = v[2], w.meta.x[l] = v[3];
            w.cap.x[l] = a[0], w.toff.x[l] = a[1], w.rm.x[l] = a[2], w.sid.x[l] = a[3];
            if constexpr (PROPS) w.props.x[l] = mem_props[pr * 64 + l];
            if constexpr (WIDE) w.rm2.x[l] = mem_rm2[pr * 64 + l];
        }
        return w;
    }
    SD void strow(u32 r, const Row& w) {
        const u32 pr = prow(r);
        for (u32 l = 0; l < 64; l++) {
            u32* v = mem_vis[pr * 64 + l];
            u32* a = mem_aux[pr * 64 + l];
            v[0] = w.len.x[l], v[1] = w.seq.x[l], v[2] = w.rseq.x[l], v[3] = w.meta.x[l];
            a[0] = w.cap.x[l], a[1] = w.toff.x[l], a[2] = w.rm.x[l], a[3] = w.sid.x[l];
            if constexpr (PROPS) mem_props[pr * 64 + l] = w.props.x[l];
            if constexpr (WIDE) mem_rm2[pr * 64 + l] = w.rm2.x[l];
        }
    }
    SD V ldf(u32 r, u32 aux, u32 c) const {  // one field of a row
        V x;
        const u32 pr = prow(r);
        for (u32 l = 0; l < 64; l++) x.x[l] = aux ? mem_aux[pr * 64 + l][c] : mem_vis[pr * 64 + l][c];
        return x;
    }
    SD void stf(u32 r, u32 aux, u32 c, V x, B m) {
        const u32 pr = prow(r);
        for (u32 l = 0; l < 64; l++)
            if ((m.m >> l) & 1) (aux ? mem_aux[pr * 64 + l] : mem_vis[pr * 64 + l])[c] = x.x[l];
    }
    // slot-index memmove (blocks move as whole 8-slot groups)
    SD void mv_slots(u32 dst, u32 src, u32 n) {
        cr = NONE;
        if (!PAGED) {
            memmove(mem_vis[dst], mem_vis[src], (size_t)n * 16);
            memmove(mem_aux[dst], mem_aux[src], (size_t)n * 16);
            memmove(&mem_props[dst], &mem_props[src], (size_t)n * 4);
            memmove(&mem_rm2[dst], &mem_rm2[src], (size_t)n * 4);
            return;
        }
        for (u32 t = 0; t < n; t++) {  // slot by slot in the memmove's safe direction
            const u32 i = dst > src ? n - 1 - t : t;
            memcpy(mem_vis[pslot(dst + i)], mem_vis[pslot(src + i)], 16);
            memcpy(mem_aux[pslot(dst + i)], mem_aux[pslot(src + i)], 16);
            mem_props[pslot(dst + i)] = mem_props[pslot(src + i)];
            mem_rm2[pslot(dst + i)] = mem_rm2[pslot(src + i)];
        }
    }
    SD void zero_slots(u32 at, u32 n) {
        cr = NONE;
        for (u32 i = 0; i < n; i++) {
            memset(mem_vis[pslot(at + i)], 0, 16);
            memset(mem_aux[pslot(at + i)], 0, 16);
            mem_props[pslot(at + i)] = 0;
            mem_rm2[pslot(at + i)] = 0;
        }
    }
#else
    // the rows' two LDS arrays (byte offsets into the dynamic LDS): the SoloPlan's slot arrays for
    // k_solo (so the LDS engine finds them in place after a handoff), a per-wave share for k_rows
    u32 vbase = (u32)offsetof(SoloPlan, vis), abase = (u32)offsetof(SoloPlan, aux);
    SD uint4* VISP() const { return reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(g_lds_dyn) + vbase); }
    SD uint4* AUXP() const { return reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(g_lds_dyn) + abase); }
    u32 pbase = 0;  // PROPS: byte offset of the slots' property map ids (one u32 per slot)
    SD u32* PROPP() const { return reinterpret_cast<u32*>(reinterpret_cast<unsigned char*>(g_lds_dyn) + pbase); }
    u32 r2base = 0;  // WIDE: byte offset of the slots' removers 32..63 (one u32 per slot)
    SD u32* RM2P() const { return reinterpret_cast<u32*>(reinterpret_cast<unsigned char*>(g_lds_dyn) + r2base); }
    u32 pool_off = 0;  // PAGED: byte offset of the pool's row mask (ROWS_POOL_WORDS words)
    SD u32* pool_words() const { return reinterpret_cast<u32*>(reinterpret_cast<unsigned char*>(g_lds_dyn) + pool_off); }
    SD bool take_row(u32& row) {  // lane 0 claims a free pool row with an LDS atomic or
        u32 got = NONE;
        if (__lane_id() == 0) {
            u32* m = pool_words();
            for (u32 wd = 0; wd < ROWS_POOL_WORDS && got == NONE; wd++) {
                u32 cur = __hip_atomic_load(m + wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                while (~cur) {
                    const u32 bit = 1u << __builtin_ctz(~cur);
                    const u32 old = atomicOr(m + wd, bit);
                    if (!(old & bit)) {
                        got = wd * 32 + (u32)__builtin_ctz(bit);
                        break;
                    }
                    cur = old | bit;
                }
            }
        }
        got = simd::readlane(simd::V{got}, 0);
        row = got;
        return got != NONE;
    }
    // A full pool is usually full for a moment (the other waves' documents shrink and end all the
    // time): wait up to ~4 ms for a row before giving the document up (a bounded wait, so waves
    // that all wait cannot deadlock: they spill; ~0.4 ms still let one C2 document in five steps
    // spill into a 100 ms HBM re-run).
    SD bool take_row_wait(u32& row) {
        for (u32 t = 0; t < ROWS_WAIT_TRIES; t++) {
            if (take_row(row)) return true;
            __builtin_amdgcn_s_sleep(8);  // ~512 cycles
        }
        return take_row(row);
    }
    SD void give_row(u32 row) {
        if (__lane_id() == 0) atomicAnd(pool_words() + (row >> 5), ~(1u << (row & 31)));
    }
    SD void zero_prow(u32 row) {
        VISP()[row * 64 + __lane_id()] = make_uint4(0, 0, 0, 0);
        AUXP()[row * 64 + __lane_id()] = make_uint4(0, 0, 0, 0);
        if constexpr (PROPS) PROPP()[row * 64 + __lane_id()] = 0u;
        if constexpr (WIDE) RM2P()[row * 64 + __lane_id()] = 0u;
        simd::lds_order();
    }
    // physical slot of logical slot s, per lane (PAGED: a block range can cross pool rows)
    SD u32 pslot(u32 s) const {
        if constexpr (PAGED) return simd::bperm(ptab, simd::V{s >> 6}).x * 64u + (s & 63u);
        else return s;
    }
    SD Row ldrow(u32 r) const {
        const u32 i = prow(r) * 64 + __lane_id();
        const uint4 v = VISP()[i], a = AUXP()[i];
        Row w;
        w.len = V{v.x}, w.seq = V{v.y}, w.rseq = V{v.z}, w.meta = V{v.w};
        w.cap = V{a.x}, w.toff = V{a.y}, w.rm = V{a.z}, w.sid = V{a.w};
        if constexpr (PROPS) w.props = V{PROPP()[i]};
        if constexpr (WIDE) w.rm2 = V{RM2P()[i]};
        return w;
    }
    SD void strow(u32 r, const Row& w) {
        const u32 i = prow(r) * 64 + __lane_id();
        VISP()[i] = make_uint4(w.len.x, w.seq.x, w.rseq.x, w.meta.x);
        AUXP()[i] = make_uint4(w.cap.x, w.toff.x, w.rm.x, w.sid.x);
        if constexpr (PROPS) PROPP()[i] = w.props.x;
        if constexpr (WIDE) RM2P()[i] = w.rm2.x;
        simd::lds_order();
    }
    SD V ldf(u32 r, u32 aux, u32 c) const {
        const u32* b = reinterpret_cast<const u32*>(aux ? AUXP() : VISP());
        return V{b[(prow(r) * 64 + __lane_id()) * 4 + c]};
    }
    SD void stf(u32 r, u32 aux, u32 c, V x, B m) {
        u32* b = reinterpret_cast<u32*>(aux ? AUXP() : VISP());
        if (simd::lane_of(m)) b[(prow(r) * 64 + __lane_id()) * 4 + c] = x.x;
        simd::lds_order();
    }
    // Overlapping slot move, one 64-slot chunk per LDS round trip; the lean engines overlap each
    // chunk's writes with the next chunk's reads (-0.3 % on the lone 10^6-op document, profiles/r05/
    // r05x). (Issuing eight chunks' reads before their writes measured 7 % SLOWER: 4.25 vs 3.93 us/op.)
    SD void mv_slots(u32 dst, u32 src, u32 n) {
        cr = NONE;
        uint4* V4 = VISP();
        uint4* A4 = AUXP();
        const u32 L = __lane_id();
        if constexpr (PAGED) {  // the same chunks, each lane's slots mapped through ptab
            const bool up = dst > src;
            for (u32 c = 0; c < n; c += 64) {
                const i32 i = up ? (i32)(n - c) - 64 + (i32)L : (i32)(c + L);
                const bool ok = i >= 0 && (u32)i < n;
                const u32 ii = ok ? (u32)i : 0u;
                const u32 ps = pslot(src + ii), pd = pslot(dst + ii);
                uint4 v = make_uint4(0, 0, 0, 0), a = v;
                u32 pp = 0, q2 = 0;
                if (ok) {
                    v = V4[ps];
                    a = A4[ps];
                    if constexpr (PROPS) pp = PROPP()[ps];
                    if constexpr (WIDE) q2 = RM2P()[ps];
                }
                simd::lds_order();
                if (ok) {
                    V4[pd] = v;
                    A4[pd] = a;
                    if constexpr (PROPS) PROPP()[pd] = pp;
                    if constexpr (WIDE) RM2P()[pd] = q2;
                }
                simd::lds_order();
            }
            return;
        }
        if constexpr (!PROPS && !WIDE) {
            // two stages: the next chunk's reads go out before this chunk's writes. The ranges never
            // meet: the walk runs away from the destination (down the slots when moving up, up them
            // when moving down), so every read still sees the slots before the move.
            const uint4 z = make_uint4(0, 0, 0, 0);
            if (dst > src) {
                i32 i = (i32)n - 64 + (i32)L;
                uint4 v = z, a = z;
                if (i >= 0) {
                    v = V4[src + (u32)i];
                    a = A4[src + (u32)i];
                }
                for (i32 b = (i32)n - 64; b > -64; b -= 64) {
                    const i32 j = i - 64;
                    uint4 v2 = z, a2 = z;
                    if (b - 64 > -64 && j >= 0) {
                        v2 = V4[src + (u32)j];
                        a2 = A4[src + (u32)j];
                    }
                    simd::lds_order();
                    if (i >= 0) {
                        V4[dst + (u32)i] = v;
                        A4[dst + (u32)i] = a;
                    }
                    simd::lds_order();
                    v = v2;
                    a = a2;
                    i = j;
                }
            } else {
                u32 i = L;
                uint4 v = z, a = z;
                if (i < n) {
                    v = V4[src + i];
                    a = A4[src + i];
                }
                for (u32 b = 0; b < n; b += 64) {
                    const u32 j = i + 64;
                    uint4 v2 = z, a2 = z;
                    if (b + 64 < n && j < n) {
                        v2 = V4[src + j];
                        a2 = A4[src + j];
                    }
                    simd::lds_order();
                    if (i < n) {
                        V4[dst + i] = v;
                        A4[dst + i] = a;
                    }
                    simd::lds_order();
                    v = v2;
                    a = a2;
                    i = j;
                }
            }
            return;
        }
        if (dst > src) {
            for (i32 b = (i32)n - 64; b > -64; b -= 64) {
                const i32 i = b + (i32)L;
                uint4 v = make_uint4(0, 0, 0, 0), a = v;
                u32 pp = 0, q2 = 0;
                if (i >= 0) {
                    v = V4[src + (u32)i];
                    a = A4[src + (u32)i];
                    if constexpr (PROPS) pp = PROPP()[src + (u32)i];
                    if constexpr (WIDE) q2 = RM2P()[src + (u32)i];
                }
                simd::lds_order();
                if (i >= 0) {
                    V4[dst + (u32)i] = v;
                    A4[dst + (u32)i] = a;
                    if constexpr (PROPS) PROPP()[dst + (u32)i] = pp;
                    if constexpr (WIDE) RM2P()[dst + (u32)i] = q2;
                }
                simd::lds_order();
            }
        } else {
            for (u32 b = 0; b < n; b += 64) {
                const u32 i = b + L;
                uint4 v = make_uint4(0, 0, 0, 0), a = v;
                u32 pp = 0, q2 = 0;
                if (i < n) {
                    v = V4[src + i];
                    a = A4[src + i];
                    if constexpr (PROPS) pp = PROPP()[src + i];
                    if constexpr (WIDE) q2 = RM2P()[src + i];
                }
                simd::lds_order();
                if (i < n) {
                    V4[dst + i] = v;
                    A4[dst + i] = a;
                    if constexpr (PROPS) PROPP()[dst + i] = pp;
                    if constexpr (WIDE) RM2P()[dst + i] = q2;
                }
                simd::lds_order();
            }
        }
    }
    SD void zero_slots(u32 at, u32 n) {
        cr = NONE;
        if constexpr (!PAGED && !PROPS && !WIDE) {
            for (u32 b = __lane_id(); b < n; b += 64) {
                VISP()[at + b] = make_uint4(0, 0, 0, 0);
                AUXP()[at + b] = make_uint4(0, 0, 0, 0);
            }
            simd::lds_order();
            return;
        }
        for (u32 c = 0; c < n; c += 64) {
            const u32 b = c + __lane_id();
            const u32 ps = pslot(at + (b < n ? b : 0u));
            if (b < n) {
                VISP()[ps] = make_uint4(0, 0, 0, 0);
                AUXP()[ps] = make_uint4(0, 0, 0, 0);
                if constexpr (PROPS) PROPP()[ps] = 0u;
                if constexpr (WIDE) RM2P()[ps] = 0u;
            }
        }
        simd::lds_order();
    }
#endif
    SD V ld_len(u32 r) const { return ldf(r, 0, 0); }
    SD V ld_meta(u32 r) const { return ldf(r, 0, 3); }
    SD V ld_sid(u32 r) const { return ldf(r, 1, 3); }
    // The row an op is working on stays in registers between its steps (resolve -> split -> insert ->
    // LRU; heap pop -> scour -> needsScour): row(r) reads LDS only when r is not the cached row,
    // putrow writes through. Anything that moves blocks (mv_slots / zero_slots) drops the cache.
    Row cw;
    u32 cr = NONE;
    SD Row row(u32 r) {
        if (r != cr) {
            cw = ldrow(r);
            cr = r;
        }
        return cw;
    }
    SD void putrow(u32 r, const Row& w) {
        strow(r, w);
        cw = w;
        cr = r;
    }
    // the cached row itself, for edits in place (no working copy of its eight registers); pair with
    // writeback(r) before anything else touches the cache
    SD Row& rowref(u32 r) {
        if (r != cr) {
            cw = ldrow(r);
            cr = r;
        }
        return cw;
    }
    SD void writeback(u32 r) { strow(r, cw); }

    // PAGED: logical rows [n_rows, need) from the pool, zeroed (rows past the last block stay zero)
    bool pool_full = false;  // PAGED: the last grow found the pool full (not the logical row limit)
    SD bool grow_rows(u32 need) {
        while (n_rows < need) {
            u32 row;
#ifdef MTE_CPU
            if (n_rows >= (u32)NR || !take_row(row)) return false;
#else
            if (n_rows >= (u32)NR) return false;
            if (!take_row_wait(row)) {
                pool_full = true;
                return false;
            }
#endif
            zero_prow(row);
            ptab = simd::writelane(ptab, n_rows, row);
            n_rows++;
        }
        return true;
    }
    SD void shrink_rows(u32 keep) {
        cr = NONE;
        while (n_rows > keep) give_row(prow(--n_rows));
    }
    SD void release_rows() {
        if constexpr (PAGED) shrink_rows(0);
    }
    // every row the state uses is held (a PAGED engine whose first row the pool never gave has none)
    SD bool rows_whole() const {
        if constexpr (PAGED) return n_rows * 8 >= n_lb;
        else return true;
    }
    // Room for leaf blocks [0, nb): PAGED takes pool rows (none left: spill the document, the host
    // re-runs it); otherwise the fixed rows must hold them.
    SD bool ensure_blocks(u32 nb) {
        if constexpr (PAGED) {
            if (grow_rows((nb + 7) >> 3)) return true;
            fail(REG_HANDOFF, curSeq);
        } else {
            if (nb <= NBLK) return true;
            fail(MTE_DOC_CAPACITY, curSeq);
        }
        return false;
    }

    SD RegEngine(const Params& p_, u32 doc_) : p(p_), doc(doc_) { setup(); }
#ifndef MTE_CPU
    // rows in another LDS region (k_rows: one share of the CU's LDS per wave)
    SD RegEngine(const Params& p_, u32 doc_, u32 vb, u32 ab, u32 mode, u32 pool = 0, u32 pb = 0, u32 r2b = 0)
        : p(p_), doc(doc_) {
        vbase = vb;
        abase = ab;
        pbase = pb;
        r2base = r2b;
        pool_off = pool;
        res_mode = mode;
        setup();
    }
#endif
    u32 res_mode = 4;  // DocRes::mode of a document this engine finishes (4: k_solo, 5: k_rows)
    SD void setup() {
        const DocCfg& c = p.docs[doc];
        payload = p.payload + c.payload_off;
        arena0 = p.arena + c.arena_off;
        seg_cap = c.seg_cap;
        arena_cap = c.arena_cap;
        payload_len = c.payload_len;
        init();
        if constexpr (PROPS) {
            mw = p.map_words;
            maps = p.maps + c.map_off * mw;
            map_cap = c.map_cap;
            mapNext = 1;  // map id 0 == no properties
            // TextSegment.canAppend reads the last character when the text has '\n': not modelled here
            if (c.has_nl) status = REG_HANDOFF;
        }
    }

    // ---------------------------------------------------------------- property maps (PROPS, HBM)
    // A map record is [n, key 0, value 0, key 1, value 1, ...] (mw words) in the document's map
    // table, immutable once built; id 0 = no properties. Lane i holds pair i.
    u32* maps = nullptr;
    u32 map_cap = 0, mw = 0, mapNext = 1;
    // lanes below each lane set in m (mbcnt)
    SD static V rank_below(u64 m) {
#ifdef MTE_CPU
        V r;
        for (u32 l = 0; l < 64; l++) r.x[l] = (u32)__builtin_popcountll(m & ((1ull << l) - 1ull));
        return r;
#else
        return V{__builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u))};
#endif
    }
    // matchProperties on one value, b uniform (properties.ts:72-80): equal ids, or b an object value
    // that a's deep-equality bits name
    SD B val_match(V a, u32 b) const {
        const B eq = a == simd::splat(b);
        if (!(p.val_flags[b] & 2u)) return eq;
        const u32 j = p.val_objidx[b];
        if (j == NONE) return eq;
        const V om = simd::ld(reinterpret_cast<const u32*>(p.val_objmatch), a * 2u + (j >> 5), simd::mk_all());
        return eq | (((om >> (j & 31u)) & 1u) != 0u);
    }
    // matchProperties of two maps (properties.ts:62-93)
    SD bool match_props(u32 a, u32 b) {
        if (a == b) return true;
        if (a == 0 || b == 0 || a >= map_cap || b >= map_cap) return false;
        fence_arena();  // map records are written lane-parallel (build_map)
        const u32* ma = maps + (u64)a * mw;
        const u32* mb = maps + (u64)b * mw;
        const u32 na = ma[0], nb = mb[0];
        if (na != nb) return false;
        const B in = L() < na;
        const V Ka = simd::ld(ma + 1, L() * 2u, in), Va = simd::ld(ma + 2, L() * 2u, in);
        const V Kb = simd::ld(mb + 1, L() * 2u, in), Vb = simd::ld(mb + 2, L() * 2u, in);
        B ok = ~in;
        for (u32 q = 0; q < nb; q++) {
            const u32 kq = simd::readlane(Kb, q), vq = simd::readlane(Vb, q);
            const B hit = in & (Ka == kq);
            if (simd::ballot(hit)) ok = ok | (hit & val_match(Va, vq));
        }
        return simd::ballot(~ok) == 0;
    }
    // SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111) on an immutable map:
    // a fresh map id (the LDS engine's build_map, engine.hpp, lane for lane)
    SD u32 build_map(u32 old, u32 propset, bool rewrite) {
        if (mapNext >= map_cap) {  // the load-time estimate was short: the host re-runs it with the worst case
            fail(res_mode == 4 ? DOC_SPILL : REG_HANDOFF, curSeq);  // (k_solo cannot hand over mid-op)
            return 0;
        }
        fence_arena();
        const u32 maxp = (mw - 1) / 2 < MTE_MAX_PROPS ? (mw - 1) / 2 : MTE_MAX_PROPS;
        u32 n = 0;
        V K = simd::splat(0), Vv = simd::splat(0);
        if (old && old < map_cap) {
            const u32* mo = maps + (u64)old * mw;
            n = mo[0];
            if (n > maxp) n = maxp;
            K = simd::ld(mo + 1, L() * 2u, L() < n);
            Vv = simd::ld(mo + 2, L() * 2u, L() < n);
        }
        const mte_propset ps = p.propsets[propset];
        const u32 pc = ps.count, pf = ps.first;
        if (rewrite) {  // delete keys whose new value is falsy / absent (:65-78); order kept
            B keep = simd::mk_none();
            for (u32 q = 0; q < pc; q++) {
                const u32 k = p.prop_keys[pf + q];
                const bool falsy = (p.val_flags[p.prop_vals[pf + q]] & 1u) != 0;
                const B hit = (L() < n) & (K == k);
                keep = falsy ? simd::andn(keep, hit) : (keep | hit);
            }
            keep = keep & (L() < n);
            const u64 km = simd::ballot(keep);
            const u32 nk = (u32)__builtin_popcountll(km);
            const V below = rank_below(km);
            const V dst = simd::sel(keep, below, (L() - below) + nk);  // a permutation of the lanes
            K = simd::push(K, dst);
            Vv = simd::push(Vv, dst);
            n = nk;
        }
        for (u32 q = 0; q < pc; q++) {
            const u32 k = p.prop_keys[pf + q], v = p.prop_vals[pf + q];
            const u64 hm = simd::ballot((L() < n) & (K == k));
            if (v == 0) {  // null deletes (:98-100): the pairs after it move down one lane
                if (hm) {
                    const u32 at = (u32)__builtin_ctzll(hm);
                    const V nxt = (L() + 1u) & 63u;
                    const V K1 = simd::bperm(K, nxt), V1 = simd::bperm(Vv, nxt);
                    const B mvd = L() >= at;
                    K = simd::sel(mvd, K1, K);
                    Vv = simd::sel(mvd, V1, Vv);
                    n--;
                }
            } else if (hm) {
                Vv = simd::sel(L() == (u32)__builtin_ctzll(hm), v, Vv);
            } else if (n < maxp) {
                K = simd::sel(L() == n, k, K);
                Vv = simd::sel(L() == n, v, Vv);
                n++;
            } else {
                fail(MTE_DOC_UNSUPPORTED, curSeq);
                return 0;
            }
        }
        const u32 id = mapNext++;
        u32* m = maps + (u64)id * mw;
        simd::st(m + 1, L() * 2u, K, L() < n);
        simd::st(m + 2, L() * 2u, Vv, L() < n);
        simd::st(m, L(), simd::splat(n), L() == 0u);
        adirty = true;  // read back later (match_props, build_map): fence_arena first
        return id;
    }
    SD void init() {
        if constexpr (PAGED) {
            n_rows = 0;
            ptab = simd::splat(0);
        } else {
            zero_slots(0, NBLK * 8);  // every slot empty: rows past the last block stay zero
        }
        LV.zero();
        HK.zero();
        HS.zero();
        n_lb = 1;
        height = 1;
        heapSize = segNext = arenaTop = arenaSel = 0;
        minSeq = curSeq = heapTop = 0;
        status = 0;
        midop = false;
        failSeq = -1;
        set_counts(0, 0);
        n_gc = 0;
        max_lb = 1;
        lb_lim = p.reg_lb_limit && p.reg_lb_limit < NBLK ? p.reg_lb_limit : NBLK;
        adirty = false;
#if defined(MTE_PROFILE) && !defined(MTE_CPU)
        for (u32 i = 0; i < RP_N; i++) pf[i] = 0;
#endif
        if constexpr (PAGED)
            if (!grow_rows(1)) status = REG_HANDOFF;
    }

    SD static V L() { return simd::lanes(); }
    // a REG_HANDOFF raised INSIDE an op (a pool row or a map record it could not get) leaves the op
    // half applied: only a restart from op 0 may continue such a document
    bool midop = false;
    SD void fail(i32 code, i32 seq) {
        if (status == 0) {
            status = code;
            failSeq = seq;
            midop = code == REG_HANDOFF;
        }
    }
    // Segment ids are 1-based in the rows (an empty slot holds 0), the LDS engine's id + 1: the
    // heap's segment lookup compares ids alone. finish() and the handoff write id - 1.
    SD u32 new_sid() {
        if (segNext >= seg_cap) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return NONE;
        }
        return ++segNext;
    }

    // ---------------------------------------------------------------- blocks
    SD static u32 gbase(u32 k) { return (k & 7u) * 8u; }
    SD static B in_group(u32 k) { return (L() >> 3) == (k & 7u); }
    SD static u32 group_bits(u64 m, u32 k) { return (u32)((m >> gbase(k)) & 0xFFull); }
    SD static u32 count_in(const Row& w, u32 k) { return (u32)__builtin_popcount(group_bits(simd::ballot(w.len != 0u), k)); }
    SD static u32 ns_in(const Row& w, u32 k) { return (simd::readlane(w.meta, gbase(k)) >> NS_SHIFT) & 3u; }
    SD static void ns_put(Row& w, u32 k, u32 sc) { w.meta = simd::sel(in_group(k), (w.meta & ~NS_MASK) | (sc << NS_SHIFT), w.meta); }
    SD u32 count(u32 k) { return count_in(row(k >> 3), k); }
    SD u32 ns_get(u32 k) { return ns_in(row(k >> 3), k); }
    SD void ns_set(u32 k, u32 sc) {
        ns_put(rowref(k >> 3), k, sc);
        writeback(k >> 3);
    }

    // nodeLength of every slot of a row for (refSeq R, client C) (mergeTree.ts:1659-1699):
    //   ins = client == C || seq <= R;  rem = removed && (removedClient == C || removedSeq <= R
    //   || C in removedClientOverlap);  visible = ins && !rem ? len : 0.
    // (live: rseq RSEQ_LIVE and rm 0; removed: bit C of rm covers removedClient and the overlap set)
    SD static V vis(const Row& w, i32 R, u32 C) {
        const B ins = simd::sle(w.seq, R) | (simd::bfe(w.meta, 0, 8) == C);
        B rem;
        if constexpr (WIDE) rem = simd::sle(w.rseq, R) | (((C < 32 ? w.rm : w.rm2) & (1u << (C & 31u))) != 0u);
        else rem = simd::sle(w.rseq, R) | ((w.rm & (1u << C)) != 0u);
        return simd::sel(simd::andn(ins, rem), w.len, 0u);
    }

    // insertingWalk's target for `pos` in the (R, C) view: the first leaf block whose cumulative
    // visible end is >= pos, then inside it the first slot with pos < its end, or a zero-length slot
    // at pos that wins breakTie (skip tombstones already seen at R, mergeTree.ts:2257-2261).
    // The scan starts at row r0 with the visible length before it, carry0 (a previous resolve of
    // the same op found its block in r0: rows before it are unchanged by the splits since).
    SD RFound resolve(i32 pos, i32 R, u32 C, u32 r0 = 0, u32 carry0 = 0) {
        RG_PROF(RP_RESOLVE);
        RFound f;
        f.ok = false;
        f.k = 0;
        f.cnt = 0;
        f.slot = -1;
        f.r = 0;
        f.row = 0;
        f.carry = 0;
        const u32 nrows = (n_lb + 7) >> 3;
        RG_STAT(RS_RESOLVE, 1);
        RG_STAT(RS_RES_NROWS, nrows);
        u32 carry = carry0;
        // Block ends are the lanes 8g+7; blocks past n_lb are empty (rows past the last block stay
        // zero), so their ends never reach pos before a real block's end does.
        const B end = (L() & 7u) == 7u;
        // the hit row: the block and slot from the registers of the scan
        auto hit_row = [&](const Row& w, u32 r, u64 hit, const V& v, const V& incl) MTE_LI {
            const u32 g = (u32)__builtin_ctzll(hit) >> 3;
            const u32 k = r * 8 + g, gb = g * 8;
            const V rr = (u32)pos - (incl - v);
            const B valid = w.len != 0u;
            const B seen = simd::sle(w.rseq, R) & (w.rseq != 0u);
            const B cand = in_group(k) & valid & (simd::slt(rr, v) | ((rr == 0u) & (v == 0u) & ~seen));
            const u64 cm = simd::ballot(cand);
            f.ok = true;
            f.k = k;
            f.cnt = (u32)__builtin_popcount(group_bits(simd::ballot(valid), k));
            f.row = r;
            f.carry = carry;
            cw = w;
            cr = r;
            if (cm) {
                const u32 l = (u32)__builtin_ctzll(cm);
                f.slot = (i32)(l - gb);
                f.r = (i32)simd::readlane(rr, l);
            }
        };
        const u32 last = nrows - 1;
        // two row buffers, each refilled (unconditionally: the last row again at the end, so the
        // LDS counter wait stays exact) while the other one is scanned; the loop only finds the hit
        // row (no state written in it, so no per-row register copies)
        Row a = row(r0), b;
        V v, incl;
        u64 hit = 0;
        bool inb = false;
        u32 r = r0;
        for (;;) {
            b = ldrow(r + 1 < last ? r + 1 : last);
            RG_COUNT(RP_N_RESOLVE, 1);
            v = vis(a, R, C);
            RG_STAT(RS_RES_ROWS, 1);
            incl = simd::scan_incl(v) + carry;
            hit = simd::ballot(end & simd::sge(incl, pos));
            if (hit) break;
            carry = simd::readlane(incl, 63);
            if (++r >= nrows) break;
            a = ldrow(r + 1 < last ? r + 1 : last);
            RG_COUNT(RP_N_RESOLVE, 1);
            v = vis(b, R, C);
            RG_STAT(RS_RES_ROWS, 1);
            incl = simd::scan_incl(v) + carry;
            hit = simd::ballot(end & simd::sge(incl, pos));
            if (hit) {
                inb = true;
                break;
            }
            carry = simd::readlane(incl, 63);
            if (++r >= nrows) break;
        }
        if (!hit) return f;
        if (inb) a = b;
        hit_row(a, r, hit, v, incl);
        return f;
    }

    // ---------------------------------------------------------------- interior levels
    // Parent (node index at level lv+1) of node c at level lv, and its first child.
    SD u32 parent_of(u32 lv, u32 c, u32& first) const {
        const V cnt = LV.get(lv);
        const V incl = simd::scan_incl(cnt);
        const u64 m = simd::ballot(incl > c);
        const u32 pi = m ? (u32)__builtin_ctzll(m) : 0u;
        first = simd::readlane(incl, pi) - simd::readlane(cnt, pi);
        return pi;
    }
    // A new node was placed right after node c at level lv (its parent gains a child): split
    // parents that reach 8 children 4+4, grow the root (insertingWalk / split / updateRoot,
    // mergeTree.ts:2446-2489, 1876-1887).
    SD void insert_after(u32 c, u32 lv) {
        for (u32 guard = 0; guard <= RG_LEVELS; guard++) {
            if (lv + 1 >= height) {  // c is the root: a new root [c, new]
                if (lv >= RG_LEVELS) break;
                LV.set(lv, simd::sel(L() == 0u, 2u, simd::splat(0)));
                height++;
                return;
            }
            u32 first;
            const u32 pi = parent_of(lv, c, first);
            V P = LV.get(lv);
            const u32 nc = simd::readlane(P, pi) + 1;
            if (nc < 8) {
                LV.set(lv, simd::writelane(P, pi, nc));
                return;
            }
            // split node pi: it keeps 4 children, a new node right after it takes 4
            P = simd::sel(L() > pi, simd::wave_shr1(P), P);
            P = simd::sel((L() == pi) | (L() == pi + 1), 4u, P);
            LV.set(lv, P);
            c = pi;
            lv++;
        }
        fail(MTE_DOC_CAPACITY, curSeq);
    }

    // ---------------------------------------------------------------- block edits
    // Blocks [from, n_lb) move to [from + d, n_lb + d); the 8*d slots this opens (d > 0) are left
    // for the caller, the ones it frees at the end (d < 0) are zeroed.
    SD void shift_blocks(u32 from, i32 d) {
        if (d == 0) return;
        RG_COUNT(RP_N_MOVE, n_lb - from);
        const u32 n = (n_lb - from) * 8;
        RG_STAT(RS_MOVE_SLOTS, n);
        if (d > 0) {
            mv_slots((from + (u32)d) * 8, from * 8, n);
        } else {
            mv_slots((from - (u32)(-d)) * 8, from * 8, n);
            zero_slots((n_lb - (u32)(-d)) * 8, (u32)(-d) * 8);
        }
    }

    // Insert `rec` at slot j of block k (child count cnt); a block reaching 8 children splits 4+4,
    // the new block right after it in document order (needsScour undefined). With `upd`, slot j-1
    // first takes (len ul, cap uc) (the left piece of a split). Returns the block holding rec.
    SD u32 insert_slot(u32 k, u32 cnt, u32 j, const RSeg& rec, bool upd, u32 ul, u32 uc) {
        RG_PROF(RP_INSERT_SLOT);
        if (cnt >= 8 || j > cnt) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return NONE;
        }
        const u32 r = k >> 3, gb = gbase(k);
        Row& w = rowref(r);
        const V sl = L() & 7u;
        const B ing = in_group(k);
        const B mv = ing & (sl > j);
        const B at = L() == gb + j;
        const u32 ns = (simd::readlane(w.meta, gb) >> NS_SHIFT) & 3u;
        if (upd) {
            const B lf = L() == gb + j - 1;
            w.len = simd::sel(lf, ul, w.len);
            w.cap = simd::sel(lf, uc, w.cap);
        }
        auto put = [&](V& x, u32 val) MTE_LI {
            x = simd::sel(mv, simd::row_shr1(x), x);
            x = simd::sel(at, val, x);
        };
        put(w.len, rec.len);
        put(w.seq, (u32)rec.seq);
        put(w.rseq, rec.rseq);
        put(w.meta, (rec.meta & ~NS_MASK) | (ns << NS_SHIFT));
        put(w.toff, rec.toff);
        put(w.cap, rec.cap);
        put(w.rm, rec.rm);
        put(w.sid, rec.sid);
        if constexpr (PROPS) put(w.props, rec.props);
        if constexpr (WIDE) put(w.rm2, rec.rm2);
        writeback(r);
        if (cnt + 1 < 8) return k;
        split_block(k);
        return j < 4 ? k : k + 1;
    }
    // Block k holds 8 children: a new block k+1 takes slots 4..7 (mergeTree.ts:2476-2489).
    SD void split_block(u32 k) {
        RG_PROF(RP_SPLIT);
        RG_COUNT(RP_N_SPLIT_BLK, 1);
        RG_STAT(RS_SPLIT_BLK, 1);
        if (!ensure_blocks(n_lb + 1)) return;
        shift_blocks(k + 1, 1);
        const u32 r = k >> 3, r2 = (k + 1) >> 3;
        const V sl = L() & 7u;
        const B lo = in_group(k + 1) & (sl < 4u), hi2 = in_group(k + 1) & (sl >= 4u), hi = in_group(k) & (sl >= 4u);
        const V src = (L() + (r2 == r ? 0u : 64u) - 4u) & 63u;  // new slot s <- old slot 4+s of block k
        Row w = row(r);
        const u32 nsk = simd::readlane(w.meta, gbase(k)) & NS_MASK;
        Row w2 = r2 == r ? w : ldrow(r2);
        auto mv = [&](V& x, V& y, u32 keepHi) MTE_LI {  // x: row r, y: row r2
            const V moved = simd::bperm(x, src);
            if (r2 == r) {
                x = simd::sel(lo, moved, x);
                x = simd::sel(hi2, 0u, x);
                x = simd::sel(hi, keepHi, x);
            } else {
                y = simd::sel(lo, moved, simd::sel(hi2, 0u, y));
                x = simd::sel(hi, keepHi, x);
            }
        };
        mv(w.len, w2.len, 0u);
        mv(w.seq, w2.seq, 0u);
        mv(w.rseq, w2.rseq, 0u);
        mv(w.meta, w2.meta, nsk);  // block k keeps its needsScour in every lane
        mv(w.toff, w2.toff, 0u);
        mv(w.cap, w2.cap, 0u);
        mv(w.rm, w2.rm, 0u);
        mv(w.sid, w2.sid, 0u);
        if constexpr (PROPS) mv(w.props, w2.props, 0u);
        if constexpr (WIDE) mv(w.rm2, w2.rm2, 0u);
        // the new block's needsScour is undefined
        if (r2 == r) {
            w.meta = simd::sel(in_group(k + 1), w.meta & ~NS_MASK, w.meta);
            putrow(r, w);
        } else {
            w2.meta = simd::sel(in_group(k + 1), w2.meta & ~NS_MASK, w2.meta);
            strow(r2, w2);
            putrow(r, w);
        }
        n_lb++;
        if (n_lb > max_lb) max_lb = n_lb;
        insert_after(k, 0);
    }

    // ---------------------------------------------------------------- LRU heap (collections.ts:213-265)
    // Position q lives in register q >> 6, lane q & 63. A walk unrolled by heap level names its
    // registers statically (level d <= 5: register 0; 6: 1; 7: 2..3; 8: 4..7): a VA indexed by a
    // run-time register number compiles to a v_cndmask chain over all eight registers per access.
    template <int D>
    SD static u32 hrd(const HeapRegs& A, u32 q) {
        const u32 l = q & 63u;
        if constexpr (D <= 5) {
            return simd::readlane(A.get(0), l);
        } else if constexpr (D == 6) {
            return simd::readlane(A.get(1), l);
        } else if constexpr (D == 7) {
            const u32 a = simd::readlane(A.get(2), l), b = simd::readlane(A.get(3), l);
            return (q >> 6) & 1u ? b : a;
        } else {
            const u32 a = simd::readlane(A.get(4), l), b = simd::readlane(A.get(5), l);
            const u32 c = simd::readlane(A.get(6), l), d = simd::readlane(A.get(7), l);
            const u32 r = (q >> 6) & 3u;
            return r == 0 ? a : r == 1 ? b : r == 2 ? c : d;
        }
    }
    template <int D>
    SD static void hwr(HeapRegs& A, u32 q, u32 v) {
        const u32 l = q & 63u;
        if constexpr (D <= 5) {
            A.set(0, simd::writelane(A.get(0), l, v));
        } else if constexpr (D == 6) {
            A.set(1, simd::writelane(A.get(1), l, v));
        } else if constexpr (D == 7) {
            if ((q >> 6) & 1u) A.set(3, simd::writelane(A.get(3), l, v));
            else A.set(2, simd::writelane(A.get(2), l, v));
        } else {
            switch ((q >> 6) & 3u) {
                case 0: A.set(4, simd::writelane(A.get(4), l, v)); break;
                case 1: A.set(5, simd::writelane(A.get(5), l, v)); break;
                case 2: A.set(6, simd::writelane(A.get(6), l, v)); break;
                default: A.set(7, simd::writelane(A.get(7), l, v)); break;
            }
        }
    }
    SD static u32 hlevel(u32 q) { return 31u - (u32)__builtin_clz(q); }
    SD u32 hkey(u32 q) const {  // any position (run-time level)
        const u32 d = hlevel(q);
        return d <= 5 ? hrd<0>(HK, q) : d == 6 ? hrd<6>(HK, q) : d == 7 ? hrd<7>(HK, q) : hrd<8>(HK, q);
    }
    SD u32 hsid(u32 q) const {
        const u32 d = hlevel(q);
        return d <= 5 ? hrd<0>(HS, q) : d == 6 ? hrd<6>(HS, q) : d == 7 ? hrd<7>(HS, q) : hrd<8>(HS, q);
    }
    SD void hset(u32 q, u32 sid, u32 key) {
        const u32 d = hlevel(q);
        if (d <= 5) {
            hwr<0>(HK, q, key);
            hwr<0>(HS, q, sid);
        } else if (d == 6) {
            hwr<6>(HK, q, key);
            hwr<6>(HS, q, sid);
        } else if (d == 7) {
            hwr<7>(HK, q, key);
            hwr<7>(HS, q, sid);
        } else {
            hwr<8>(HK, q, key);
            hwr<8>(HS, q, sid);
        }
    }
    // push: keys are op seqs, strictly increasing across messages, so the sift-up never moves an
    // entry (collections.ts:241-250 moves strictly larger parents only): an append
    SD void heap_push(u32 sid, i32 key) {
        if (heapSize + 1 >= RG_HEAP) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return;
        }
        const u32 n = ++heapSize;
        RG_STAT(RS_LRU_PUSH, 1);
        if (n == 1) heapTop = key;
        hset(n, sid, (u32)key);
    }
    // pop: sift-down of collections.ts:252-264 (smaller child, left on ties, moves up while
    // strictly below the moved last entry (lk, ls)); node k sits at level D, m entries remain
    template <int D>
    SD void sift(u32 k, u32 m, u32 lk, u32 ls, i32& newTop) {
        if constexpr (D < 8) {
            u32 j = k << 1;
            if (j <= m) {
                u32 kj = hrd<D + 1>(HK, j);
                if (j < m) {
                    const u32 kj1 = hrd<D + 1>(HK, j + 1);
                    if ((i32)kj - (i32)kj1 > 0) {
                        j++;
                        kj = kj1;
                    }
                }
                if ((i32)lk - (i32)kj > 0) {
                    if (D == 0) newTop = (i32)kj;
                    hwr<D>(HK, k, kj);
                    hwr<D>(HS, k, hrd<D + 1>(HS, j));
                    sift<D + 1>(j, m, lk, ls, newTop);
                    return;
                }
            }
        }
        hwr<D>(HK, k, lk);
        hwr<D>(HS, k, ls);
    }
    // The same sift-down, lane-parallel while the heap fits positions 1..127 (registers 0 and 1):
    // every node k of register 0 (lane k) picks its child c(k) and whether the moved entry goes
    // below it (lk > K[c(k)]) at once; the path from the root then follows two ballots of those
    // decisions, and every node on it above the stop node takes its child's entry in one select.
    SD void pop_fast(u32 m, u32 lk, u32 ls, i32& newTop) {
        const V K0 = HK.get(0), K1 = HK.get(1), S0 = HS.get(0), S1 = HS.get(1);
        const V cl = L() * 2u, cr = cl + 1u;
        // both children's keys AND segment ids in one round of crossbar gathers (register 1 only
        // when the heap reaches it)
        V kL, kR, sL, sR;
        if (m < 64u) {
            kL = simd::bperm(K0, cl & 63u);
            kR = simd::bperm(K0, cr & 63u);
            sL = simd::bperm(S0, cl & 63u);
            sR = simd::bperm(S0, cr & 63u);
        } else {
            const B l0 = cl < 64u, r0 = cr < 64u;
            kL = simd::sel(l0, simd::bperm(K0, cl & 63u), simd::bperm(K1, cl & 63u));
            kR = simd::sel(r0, simd::bperm(K0, cr & 63u), simd::bperm(K1, cr & 63u));
            sL = simd::sel(l0, simd::bperm(S0, cl & 63u), simd::bperm(S1, cl & 63u));
            sR = simd::sel(r0, simd::bperm(S0, cr & 63u), simd::bperm(S1, cr & 63u));
        }
        const B right = (cr < m + 1u) & simd::slt(kR, kL);  // smaller child, the left one on ties
        const V c = simd::sel(right, cr, cl);
        const V kc = simd::sel(right, kR, kL);
        const V sc = simd::sel(right, sR, sL);
        const B go = (cl < m + 1u) & simd::slt(kc, (i32)lk);  // the moved entry goes below k
        u32 k = 1;
        u64 path = 0;  // nodes of register 0 that take their child's entry
        // G bit k: node k takes its chosen child's entry (the moved entry goes below k); Rt bit k:
        // that child is the right one. The path from the root follows them in scalar registers
        // (one crossbar round trip fewer than gathering each child's parent decision); nodes
        // 32..63 continue into register 1.
        const u64 G = simd::ballot(go), Rt = simd::ballot(right);
        while (k < 64u) {
            if (!((G >> k) & 1u)) break;
            path |= 1ull << k;
            k = 2 * k + (u32)((Rt >> k) & 1u);
        }
        const B mv = simd::ballot_mask(path);
        V N0 = simd::sel(mv, kc, K0), T0 = simd::sel(mv, sc, S0);
        if (path & 2u) newTop = (i32)simd::readlane(kc, 1);
        if (k < 64u) {
            N0 = simd::writelane(N0, k, lk);
            T0 = simd::writelane(T0, k, ls);
        } else {
            HK.set(1, simd::writelane(K1, k & 63u, lk));
            HS.set(1, simd::writelane(S1, k & 63u, ls));
        }
        HK.set(0, N0);
        HS.set(0, T0);
    }
    SD u32 heap_pop() {
        RG_PROF(RP_HEAP);
        RG_COUNT(RP_N_POP, 1);
        const u32 n = heapSize, m = n - 1;
        RG_STAT(RS_POP, 1);
        RG_STAT(RS_POP_BIG, m >= 128u);
        RG_STAT(RS_POP_HEAP, n);
#if defined(MTE_CPU) && defined(MTE_CPU_STATS)
        if (n > g_rg_stats[RS_N]) g_rg_stats[RS_N] = n;  // the largest heap at a pop
        if (n_lb > g_rg_stats[RS_N + 1]) g_rg_stats[RS_N + 1] = n_lb;
#endif
        const u32 top = hrd<0>(HS, 1);
        const u32 lk = hkey(n), ls = hsid(n);
        i32 newTop = (i32)lk;
        if (m >= 1) {
            if (m < 128u) pop_fast(m, lk, ls, newTop);
            else sift<0>(1, m, lk, ls, newTop);
        }
        heapTop = newTop;
        heapSize = m;
        return top;
    }
    // addToLRUSet (mergeTree.ts:1273-1283) for a segment of block k
    SD void add_lru(u32 k, u32 sid, i32 seq) {
        RG_PROF(RP_LRU);
        if (ns_get(k) != SC_TRUE && seq > curSeq) {
            ns_set(k, SC_TRUE);
            heap_push(sid, seq);
        }
    }
    // the leaf block holding segment sid (segment.parent), NONE when unlinked. Segment ids are
    // unique, so each batch of eight rows needs one per-lane select per row and ONE ballot (no
    // branch per row): the hit lane's row index comes back with one readlane.
    SD u32 find_seg(u32 sid) {
        RG_PROF(RP_FIND_SEG);
        const u32 nrows = (n_lb + 7) >> 3;
        RG_STAT(RS_FIND_ROWS, nrows);
        for (u32 r0 = 0; r0 < nrows; r0 += 8) {  // eight rows' reads in flight per round
            V s8[8];
            for (u32 i = 0; i < 8; i++) s8[i] = ld_sid(r0 + i < nrows ? r0 + i : r0);
            V hr = simd::splat(NONE);
            for (u32 i = 8; i-- > 0;) hr = simd::sel(s8[i] == sid, r0 + i, hr);  // rows past nrows re-read r0: i = 0 wins
            const u64 m = simd::ballot(hr != NONE);
            if (m) {
                const u32 l = (u32)__builtin_ctzll(m);
                return simd::readlane(hr, l) * 8 + (l >> 3);
            }
        }
        return NONE;
    }

    // ---------------------------------------------------------------- text (HBM)
    SD u16* arena_cur() const { return arena0 + (u64)arenaSel * arena_cap; }
    SD void fence_arena() {
        if (adirty) {
            simd::wave_fence();
            adirty = false;
        }
    }
    // copy n units from text offset src (payload or arena) to offset dst of dbase (lanes in parallel)
    SD void copy_text(u32 dst, u32 src, u32 n, u16* dbase) {
        const u16* sb = (src & ARENA_BIT) ? arena_cur() : payload;
        const u32 so = src & ~ARENA_BIT, d0 = dst & ~ARENA_BIT;
        for (u32 b = 0; b < n; b += 64) {
            const V i = L() + b;
            const B m = i < n;
            const V t = simd::ld(sb, i + so, m);
            simd::st(dbase, i + d0, t, m);
        }
    }
    // Semispace compaction of the merge arena: every live arena-resident text, document order.
    SD void arena_gc() {
        fence_arena();
        const u32 other = arenaSel ^ 1u;
        u16* dst = arena0 + (u64)other * arena_cap;
        u32 top = 0;
        for (u32 k = 0; k < n_lb; k++) {
            const u32 r = k >> 3, gb = gbase(k);
            Row w = ldrow(r);
            const u32 cnt = (u32)__builtin_popcount(group_bits(simd::ballot(w.len != 0u), k));
            bool dirty = false;
            for (u32 s = 0; s < cnt; s++) {
                const u32 l = gb + s;
                const u32 meta = simd::readlane(w.meta, l), toff = simd::readlane(w.toff, l);
                if ((meta & F_MARKER) || !(toff & ARENA_BIT)) continue;
                const u32 len = simd::readlane(w.len, l), oc = simd::readlane(w.cap, l);
                const bool rm = simd::readlane(w.rseq, l) != RSEQ_LIVE;
                const u32 cap = (rm || oc < len) ? len : oc;
                if ((toff & ~ARENA_BIT) + len > arena_cap || top + cap > arena_cap) {
                    fail(MTE_DOC_CAPACITY, curSeq);
                    return;
                }
                copy_text(top, toff, len, dst);
                w.toff = simd::writelane(w.toff, l, top | ARENA_BIT);
                w.cap = simd::writelane(w.cap, l, cap);
                dirty = true;
                top += cap;
            }
            if (dirty) putrow(r, w);
        }
        simd::wave_fence();
        arenaSel = other;
        arenaTop = top;
        n_gc++;
    }

    // ---------------------------------------------------------------- zamboni (mergeTree.ts:1289-1478)
    // scourNode on block k (cnt children): tombstones at or below the MSN are dropped and reset the
    // merge chain, settled live text appends to the chain head under TextSegment.canAppend
    // (textSegment.ts:63-85; no '\n' in these documents, no properties); kept slots are compacted.
    // Returns the new child count.
    //
    // Lane-parallel form: in the lean documents this engine replays (no properties, no '\n'), a
    // settled slot joins the run of the settled slot before it exactly when both are text (a removed
    // or unsettled slot resets the chain; a marker head or marker slot starts a new one), unless
    // TextSegment.canAppend's granularity test fails, which needs the run's accumulated length: a
    // block where a joining slot is longer than GRANULARITY takes the serial walk (scour_serial).
    // Each run becomes its head with the run's text: already contiguous (no copy), appended into the
    // head's arena chunk when it has the capacity, or else copied into a fresh chunk of
    // max(32, 2 * total) units; all copies of the block run as one flattened gather.
    bool scoured = false;  // the last scour rewrote its block's row, needsScour already false
    SD u32 scour(u32 k, u32 cnt) {
        RG_PROF(RP_SCOUR);
        scoured = false;
        RG_COUNT(RP_N_SCOUR, 1);
        if (cnt > 8) cnt = 8;
        const u32 r = k >> 3, gb = gbase(k);
        const B ing = in_group(k);
        Row w = row(r);
        const B act = ing & (w.len != 0u);
        const B rem = act & (w.rseq != RSEQ_LIVE);
        const u32 mDROP = group_bits(simd::ballot(rem & simd::sle(w.rseq, minSeq)), k);
        const u32 mSET = group_bits(simd::ballot(simd::andn(act, rem) & simd::sle(w.seq, minSeq)), k);
        const u32 mTXT = group_bits(simd::ballot(act & ((w.meta & F_MARKER) == 0u)), k);
        const u32 mST = mSET & mTXT;
        u32 mJOIN = mST & (mST << 1) & 0xFFu;  // slot s joins the run of slot s-1
        if constexpr (PROPS) {  // ... when its properties match slot s-1's (matchProperties)
            const u32 mSAME = group_bits(simd::ballot(w.props == simd::row_shr1(w.props)), k);
            for (u32 c = mJOIN & ~mSAME; c; c &= c - 1) {
                const u32 sb = (u32)__builtin_ctz(c);
                if (!match_props(simd::readlane(w.props, gb + sb - 1), simd::readlane(w.props, gb + sb))) mJOIN &= ~(1u << sb);
            }
        }
        RG_STAT(RS_SCOUR, 1);
        if (!mDROP && !mJOIN) {  // nothing dropped, nothing merged
            RG_STAT(RS_SCOUR_NOP, 1);
            return cnt;
        }
        if (mJOIN & group_bits(simd::ballot(w.len > (u32)GRANULARITY), k)) {
            RG_STAT(RS_SCOUR_SERIAL, 1);
            return scour_serial(k, cnt);
        }
        RG_COUNT(RP_N_SCOUR_CHANGED, 1);
        fence_arena();
        const V sl = L() & 7u;
        V jdst = simd::splat(0), jlen = jdst, jsrc = jdst;  // per slot lane: jlen units from jsrc to jdst
        for (u32 attempt = 0; attempt < 2; attempt++) {
            // offsets inside a run: exclusive prefix sum of the block's lengths
            const V gl = simd::sel(ing, w.len, 0u);
            const V ex = simd::scan_incl(gl) - gl;
            const B cont = w.toff == simd::row_shr1(w.toff + w.len);  // text starts where slot s-1's ends
            const u32 mCONT = group_bits(simd::ballot(cont), k);
            jdst = jlen = simd::splat(0);
            u32 top = arenaTop, need = 0;
            Row nw = w;
            for (u32 heads = mST & ~mJOIN & (mJOIN >> 1); heads; heads &= heads - 1) {
                const u32 h = (u32)__builtin_ctz(heads);
                const u32 run = (u32)__builtin_ctz(~(mJOIN >> (h + 1)));  // joining slots after h
                const u32 e = h + run, rb = ((2u << e) - 1u) & ~((2u << h) - 1u);  // bits h+1..e
                const u32 lh = gb + h, le = gb + e;
                const u32 off = simd::readlane(w.toff, lh), cap = simd::readlane(w.cap, lh);
                const u32 exh = simd::readlane(ex, lh);
                const u32 total = simd::readlane(ex, le) + simd::readlane(w.len, le) - exh;
                u32 noff = off, ncap = cap, cbits = 0;
                if ((mCONT & rb) == rb) {  // the run's text is one contiguous range already
                    if (off & ARENA_BIT) ncap = simd::readlane(w.toff, le) + simd::readlane(w.cap, le) - off;
                } else if ((off & ARENA_BIT) && total <= cap) {  // append into the head's chunk
                    cbits = rb;
                } else {  // a fresh chunk
                    ncap = 2 * total < 32 ? 32u : 2 * total;
                    noff = top | ARENA_BIT;
                    top += ncap;
                    need += ncap;
                    cbits = rb | (1u << h);
                }
                if (cbits) {
                    const B cp = ing & (((simd::splat(cbits) >> sl) & 1u) != 0u);
                    jdst = simd::sel(cp, ex + (noff - exh), jdst);
                    jlen = simd::sel(cp, w.len, jlen);
                }
                nw.len = simd::writelane(nw.len, lh, total);
                nw.toff = simd::writelane(nw.toff, lh, noff);
                nw.cap = simd::writelane(nw.cap, lh, ncap);
            }
            if (arenaTop + need <= arena_cap) {
                arenaTop = top;
                jsrc = w.toff;  // the slots' text before the runs' heads move
                w = nw;
                break;
            }
            if (attempt == 1) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return cnt;
            }
            arena_gc();  // moves every arena text: re-read the slots and redo the runs
            if (status) return cnt;
            w = row(r);
            fence_arena();
        }
        copy_runs(jdst, jsrc, jlen);
        // compaction: kept slots (not dropped, not joined) in order at the front of the group, the
        // rest behind them; a push permutation (ds_permute) inside the group
        const u32 mKEEP = group_bits(simd::ballot(act), k) & ~mDROP & ~mJOIN;
        const u32 nkeep = (u32)__builtin_popcount(mKEEP);
        const V below = (simd::shl(simd::splat(1), sl) - 1u);
        const B kp = ((simd::splat(mKEEP) >> sl) & 1u) != 0u;
        const V dst = simd::sel(ing, simd::sel(kp, simd::bcnt(simd::splat(mKEEP) & below),
                                               simd::bcnt(simd::splat(~mKEEP & 0xFFu) & below) + nkeep) + gb,
                                L());
        const B tail = ing & (sl >= nkeep);
        auto cmp = [&](V& x, u32 keepEmpty) MTE_LI {
            const V nv = simd::push(x, dst);
            x = simd::sel(tail, nv & keepEmpty, nv);
        };
        cmp(w.len, 0u);
        cmp(w.seq, 0u);
        cmp(w.rseq, 0u);
        cmp(w.meta, NS_MASK);  // the block's needsScour stays in every lane
        cmp(w.cap, 0u);
        cmp(w.toff, 0u);
        cmp(w.rm, 0u);
        cmp(w.sid, 0u);
        if constexpr (PROPS) cmp(w.props, 0u);
        if constexpr (WIDE) cmp(w.rm2, 0u);
        ns_put(w, k, SC_FALSE);  // scourNode's caller clears needsScour (mergeTree.ts:1457): same write
        putrow(r, w);
        scoured = true;
        return nkeep;
    }
    // The runs' text copies of one block as one flattened gather: slot lane l copies jlen units from
    // its text src to jdst (sources are never destinations of the same scour).
    SD void copy_runs(V jdst, V jsrc, V jlen) {
        const V jinc = simd::scan_incl(jlen);
        const u32 total = simd::readlane(jinc, 63);
        if (!total) return;
        RG_STAT(RS_SCOUR_COPY, 1);
        const V jstart = jinc - jlen;
        u64 jm = simd::ballot(jlen != 0u);
        u16* ar = arena_cur();
        for (u32 base = 0; base < total; base += 64) {
            const V f = L() + base;
            V j = simd::splat(0);
            for (u64 m = jm; m; m &= m - 1) {
                const u32 q = (u32)__builtin_ctzll(m);
                j = simd::sel(f >= simd::readlane(jstart, q), q, j);
            }
            const V s0 = simd::bperm(jstart, j), d = simd::bperm(jdst, j), sr = simd::bperm(jsrc, j);
            const B m = f < total;
            const V o = f - s0;
            const B fa = (sr & ARENA_BIT) != 0u;
            const V so = (sr & ~ARENA_BIT) + o;
            const V t = simd::sel(fa, simd::ld(ar, so, m & fa), simd::ld(payload, so, simd::andn(m, fa)));
            simd::st(ar, (d & ~ARENA_BIT) + o, t, m);
        }
        adirty = true;
    }
    // The serial walk of scourNode (any lengths): the granularity test needs the run's accumulated
    // length.
    SD u32 scour_serial(u32 k, u32 cnt) {
        fence_arena();
        const u32 r = k >> 3, gb = gbase(k);
        const B ing = in_group(k);
        Row w = row(r);
        const B act = ing & (w.len != 0u);
        const B rem = act & (w.rseq != RSEQ_LIVE);
        const u32 mREM = group_bits(simd::ballot(rem), k);
        const u32 mKEPT = group_bits(simd::ballot(rem & simd::sgt(w.rseq, minSeq)), k);
        const u32 mSET = group_bits(simd::ballot(simd::andn(act, rem) & simd::sle(w.seq, minSeq)), k);
        if (!(mREM & ~mKEPT) && !(mSET & (mSET << 1))) return cnt;  // nothing dropped, nothing to merge
        const u32 mTXT = group_bits(simd::ballot(act & ((w.meta & F_MARKER) == 0u)), k);
        u32 nkeep = 0, jn = 0;
        V kSrc = simd::splat(0), kLen = kSrc, kOff = kSrc, kCap = kSrc;  // lane i: kept slot i
        V jdst = kSrc, jsrc = kSrc, jlen = kSrc;                          // lane j: copy job j
        for (u32 attempt = 0; attempt < 2; attempt++) {
            nkeep = jn = 0;
            jdst = jsrc = jlen = simd::splat(0);
            u32 top = arenaTop, need = 0;
            i32 prev = -1;
            u32 pLen = 0, pOff = 0, pCap = 0, pMat = 0, pProps = 0;
            bool pText = false, pFresh = false;
            auto job = [&](u32 d, u32 s, u32 n) MTE_LI {
                if (jn < 64) {
                    jdst = simd::writelane(jdst, jn, d);
                    jsrc = simd::writelane(jsrc, jn, s);
                    jlen = simd::writelane(jlen, jn, n);
                }
                jn++;
            };
            for (u32 s = 0; s < cnt; s++) {
                const u32 bit = 1u << s;
                bool keep = true;
                if (mREM & bit) {
                    keep = (mKEPT & bit) != 0;
                    prev = -1;
                } else if (mSET & bit) {
                    const u32 ln = simd::readlane(w.len, gb + s), to = simd::readlane(w.toff, gb + s);
                    const u32 tc = simd::readlane(w.cap, gb + s);
                    u32 sp = 0;
                    if constexpr (PROPS) sp = simd::readlane(w.props, gb + s);
                    const bool ok = prev >= 0 && pText && (mTXT & bit) && (pLen <= (u32)GRANULARITY || ln <= (u32)GRANULARITY) &&
                                    (!PROPS || match_props(pProps, sp));
                    if (ok) {  // TextSegment.append
                        if ((pOff & ARENA_BIT) && pLen + ln <= pCap) {
                            job(pOff + pLen, to, ln);
                        } else if (pOff + pLen == to && pMat == pLen) {  // text already contiguous
                            if (pOff & ARENA_BIT) pCap = to + tc - pOff;
                            pMat += ln;
                        } else {
                            u32 ncap = 2 * (pLen + ln);
                            if (ncap < 32) ncap = 32;
                            const u32 dst = top | ARENA_BIT;
                            top += ncap;
                            need += ncap;
                            // pending jobs into the head's chunk follow it to the new one; the
                            // materialised prefix (none for a chunk built by this batch) is copied
                            const u32 m0 = pFresh ? 0u : pMat;
                            const B mvj = (L() < jn) & (jdst >= pOff + m0) & (jdst < pOff + pLen);
                            jdst = simd::sel(mvj, jdst - pOff + dst, jdst);
                            if (m0) job(dst, pOff, m0);
                            job(dst + pLen, to, ln);
                            pOff = dst;
                            pCap = ncap;
                            pFresh = true;
                        }
                        pLen += ln;
                        kLen = simd::writelane(kLen, (u32)prev, pLen);
                        kOff = simd::writelane(kOff, (u32)prev, pOff);
                        kCap = simd::writelane(kCap, (u32)prev, pCap);
                        keep = false;
                    } else {
                        prev = (i32)nkeep;
                        pLen = ln;
                        pMat = ln;
                        pOff = to;
                        pCap = tc;
                        pText = (mTXT & bit) != 0;
                        pFresh = false;
                        pProps = sp;
                    }
                } else {
                    prev = -1;
                }
                if (keep) {
                    kSrc = simd::writelane(kSrc, nkeep, s);
                    kLen = simd::writelane(kLen, nkeep, simd::readlane(w.len, gb + s));
                    kOff = simd::writelane(kOff, nkeep, simd::readlane(w.toff, gb + s));
                    kCap = simd::writelane(kCap, nkeep, simd::readlane(w.cap, gb + s));
                    nkeep++;
                }
            }
            if (nkeep == cnt) return cnt;
            if (arenaTop + need <= arena_cap && jn <= 64) {
                arenaTop = top;
                break;
            }
            if (attempt == 1) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return cnt;
            }
            arena_gc();  // moves every arena text: re-read the slots and redo the chain
            if (status) return cnt;
            w = row(r);
        }
        if (jn) run_jobs(jn, jdst, jsrc, jlen);
        // compaction: group lane gb+i takes kept slot i
        const V sl = L() & 7u;
        const B kp = ing & (sl < nkeep);
        const V src = simd::bperm(kSrc, sl) + gb;
        auto cmp = [&](V& x, const V* over, u32 keepEmpty) MTE_LI {  // empty lanes keep only `keepEmpty` bits
            const V nv = over ? simd::bperm(*over, sl) : simd::bperm(x, src);
            x = simd::sel(kp, nv, simd::sel(ing, x & keepEmpty, x));
        };
        cmp(w.len, &kLen, 0u);
        cmp(w.toff, &kOff, 0u);
        cmp(w.cap, &kCap, 0u);
        cmp(w.rm, nullptr, 0u);
        cmp(w.seq, nullptr, 0u);
        cmp(w.rseq, nullptr, 0u);
        cmp(w.meta, nullptr, NS_MASK);  // the block's needsScour stays in every lane
        cmp(w.sid, nullptr, 0u);
        if constexpr (PROPS) cmp(w.props, nullptr, 0u);
        if constexpr (WIDE) cmp(w.rm2, nullptr, 0u);
        ns_put(w, k, SC_FALSE);
        putrow(r, w);
        scoured = true;
        return nkeep;
    }
    // The recorded copies as one flattened gather (sources are never destinations of one scour).
    SD void run_jobs(u32 jn, V jdst, V jsrc, V jlen) {
        const V jl = simd::sel(L() < jn, jlen, 0u);
        const V jinc = simd::scan_incl(jl);
        const u32 total = simd::readlane(jinc, 63);
        const V jstart = jinc - jl;
        u16* ar = arena_cur();
        for (u32 base = 0; base < total; base += 64) {
            const V f = L() + base;
            V j = simd::splat(0);
            for (u32 q = 1; q < jn; q++) j = simd::sel(f >= simd::readlane(jstart, q), q, j);
            const V s0 = simd::bperm(jstart, j), d = simd::bperm(jdst, j), sr = simd::bperm(jsrc, j);
            const B m = f < total;
            const V o = f - s0;
            const B fa = (sr & ARENA_BIT) != 0u;
            const V so = (sr & ~ARENA_BIT) + o;
            const V t = simd::sel(fa, simd::ld(ar, so, m & fa), simd::ld(payload, so, simd::andn(m, fa)));
            simd::st(ar, (d & ~ARENA_BIT) + o, t, m);
        }
        adirty = true;
    }

    // pack (mergeTree.ts:1368-1420), leaf level: the m children [k0, k0+m) of level-1 node pi
    // (already re-scoured; lane i of cn = child i's count) become max(1, min(7, T/4)) fresh blocks.
    SD void pack_leaves(u32 pi, u32 m, u32 k0, V cn) {
        RG_PROF(RP_PACK);
        RG_COUNT(RP_N_PACK, 1);
        RG_STAT(RS_PACK, 1);
        const u32 T = simd::readlane(simd::scan_incl(simd::sel(L() < m, cn, 0u)), 63);
        u32 kk = T / 4;
        if (kk > 7) kk = 7;
        if (kk < 1) kk = 1;
        const u32 base = T / kk, extra = T % kk;
        if (!ensure_blocks(n_lb + kk - m)) return;
        // item t (lane t < T) of the concatenated children: block k0 + sib, slot q
        V sib = simd::splat(0), q = L();
        for (u32 i = 0; i < m; i++) {
            const u32 n = simd::readlane(cn, i);
            const B adv = (q >= n) & (sib == i);
            q = simd::sel(adv, q - n, q);
            sib = simd::sel(adv, i + 1, sib);
        }
        const V sg = (sib + k0) * 8u + q;  // source slot (global)
        const u32 r0 = k0 >> 3, r1 = r0 + 1 < (u32)NR ? r0 + 1 : r0;
        const B inr0 = (sg >> 6) == r0;
        Row a = ldrow(r0), b = ldrow(r1);
        auto gather = [&](const V& x0, const V& x1) MTE_LI {
            return simd::sel(inr0, simd::bperm(x0, sg & 63u), simd::bperm(x1, sg & 63u));
        };
        Row t;
        t.len = gather(a.len, b.len);
        t.seq = gather(a.seq, b.seq);
        t.rseq = gather(a.rseq, b.rseq);
        t.meta = gather(a.meta, b.meta) & ~NS_MASK;  // packed blocks: needsScour undefined
        t.toff = gather(a.toff, b.toff);
        t.cap = gather(a.cap, b.cap);
        t.rm = gather(a.rm, b.rm);
        t.sid = gather(a.sid, b.sid);
        if constexpr (PROPS) t.props = gather(a.props, b.props);
        if constexpr (WIDE) t.rm2 = gather(a.rm2, b.rm2);
        const i32 d = (i32)kk - (i32)m;
        shift_blocks(k0 + m, d);
        // destination: block k0 + dj slot dq <- item dj*base + min(dj, extra) + dq
        const u32 rA = k0 >> 3, rB = (k0 + kk - 1) >> 3;
        for (u32 rr = rA; rr <= rB; rr++) {
            const V G = L() + rr * 64;
            const V blk = G >> 3;
            const B inb = (blk >= k0) & (blk < k0 + kk);
            const V dj = blk - k0, dq = G & 7u;
            const V big = simd::sel(dj < extra, dj, simd::splat(extra));
            const V nB = simd::sel(dj < extra, base + 1, simd::splat(base));
            const B have = inb & (dq < nB);
            const V ti = (dj * base + big + dq) & 63u;
            Row w = ldrow(rr);
            auto put = [&](V& x, const V& tv) MTE_LI { x = simd::sel(have, simd::bperm(tv, ti), simd::sel(inb, 0u, x)); };
            put(w.len, t.len);
            put(w.seq, t.seq);
            put(w.rseq, t.rseq);
            put(w.meta, t.meta);
            put(w.toff, t.toff);
            put(w.cap, t.cap);
            put(w.rm, t.rm);
            put(w.sid, t.sid);
            if constexpr (PROPS) put(w.props, t.props);
            if constexpr (WIDE) put(w.rm2, t.rm2);
            strow(rr, w);
        }
        cr = NONE;
        n_lb = (u32)((i32)n_lb + d);
        if (n_lb > max_lb) max_lb = n_lb;
        LV.set(0, simd::writelane(LV.get(0), pi, kk));
        if (kk < 4 && height > 2) pack_internal(pi, 1);
    }
    // pack on an interior level: node pi of level lv underflowed; the children of its parent are
    // redistributed into max(1, min(7, T/4)) nodes, T their total child count.
    SD void pack_internal(u32 pi, u32 lv) {
        for (u32 guard = 0; guard < RG_LEVELS + 2; guard++) {
            u32 i0;
            const u32 qi = parent_of(lv, pi, i0);  // parent at level lv+1
            const V Q = LV.get(lv);
            const u32 m = simd::readlane(Q, qi);
            V C = LV.get(lv - 1);  // child counts of the level-lv nodes
            const u32 T = simd::readlane(simd::scan_incl(simd::sel((L() >= i0) & (L() < i0 + m), C, 0u)), 63);
            u32 kk = T / 4;
            if (kk > 7) kk = 7;
            if (kk < 1) kk = 1;
            const u32 base = T / kk, extra = T % kk;
            const i32 d = (i32)kk - (i32)m;
            // lanes after the old range move by d
            const V src = L() - (u32)d;
            const V moved = simd::bperm(C, src & 63u);
            C = simd::sel(L() >= i0 + kk, simd::sel(src < 64u, moved, 0u), C);
            const V dj = L() - i0;
            C = simd::sel((L() >= i0) & (L() < i0 + kk), simd::sel(dj < extra, base + 1, simd::splat(base)), C);
            LV.set(lv - 1, C);
            LV.set(lv, simd::writelane(Q, qi, kk));
            if (kk < 4 && lv + 2 < height) {
                pi = qi;
                lv++;
                continue;
            }
            return;
        }
        fail(MTE_DOC_CAPACITY, curSeq);
    }

    // zamboniSegments (mergeTree.ts:1422-1478): up to 2 heap entries with maxSeq <= minSeq.
    SD void zamboni() {
        RG_PROF(RP_ZAMBONI);
        RG_STAT(RS_ZAM_CALLS, 1);
        for (int i = 0; i < 2 && !status; i++) {
            if (heapSize == 0 || heapTop > minSeq) break;
            RG_STAT(RS_ZAM_POPS, 1);
            const u32 sid = heap_pop();
            const u32 k = find_seg(sid);
            if (k == NONE) continue;  // no longer linked
            if (ns_get(k) == SC_FALSE) continue;
            const u32 cnt = count(k);
            const u32 nc = scour(k, cnt);
            if (status) return;
            if (!scoured) ns_set(k, SC_FALSE);
            if (!(nc < cnt && nc < 4 && height > 1)) continue;
            u32 k0;
            const u32 pi = parent_of(0, k, k0);
            const u32 m = simd::readlane(LV.get(0), pi);
            if (m == 0 || m > 8 || k0 + m > n_lb) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return;
            }
            V cn = simd::splat(0);
            for (u32 idx = 0; idx < m; idx++) {
                const u32 c = scour(k0 + idx, count(k0 + idx));
                if (status) return;
                cn = simd::writelane(cn, idx, c);
            }
            pack_leaves(pi, m, k0, cn);
        }
    }

    // ---------------------------------------------------------------- ops
    // ensureIntervalBoundary at the resolved slot (BaseSegment.splitAt, mergeTree.ts:524-568): the
    // right piece copies everything and follows the left one. Returns the insert_slot result.
    SD u32 split_at(const RFound& f) {
        RG_PROF(RP_SPLIT_AT);
        RG_STAT(RS_SPLIT_AT, 1);
        const u32 r = f.k >> 3, l = gbase(f.k) + (u32)f.slot;
        const Row w = row(r);
        RSeg t;
        t.len = simd::readlane(w.len, l);
        t.seq = (i32)simd::readlane(w.seq, l);
        t.rseq = simd::readlane(w.rseq, l);
        t.meta = simd::readlane(w.meta, l);
        t.toff = simd::readlane(w.toff, l);
        t.cap = simd::readlane(w.cap, l);
        t.rm = simd::readlane(w.rm, l);
        if constexpr (PROPS) t.props = simd::readlane(w.props, l);  // the right piece shares the map
        if constexpr (WIDE) t.rm2 = simd::readlane(w.rm2, l);
        const u32 sid = new_sid();
        if (sid == NONE) return NONE;
        const u32 rr = (u32)f.r;
        const bool ar = (t.toff & ARENA_BIT) != 0;  // arena text: cap >= len, split between the pieces
        const u32 lc = ar ? rr : 0u;
        RSeg right = t;
        right.len = t.len - rr;
        right.toff = t.toff + rr;
        right.cap = ar ? t.cap - rr : 0u;
        right.sid = sid;
        return insert_slot(f.k, f.cnt, (u32)f.slot + 1, right, true, rr, lc);
    }

    // insertSegments (mergeTree.ts:1968-1998): split at pos, then place the new segment.
    SD bool op_insert(i32 pos, i32 R, u32 C, i32 seq, RSeg rec) {
        RG_PROF(RP_INS);
        RFound f = resolve(pos, R, C);
        if (!f.ok) {
            fail(MTE_DOC_INSERT_FAILED, seq);
            return false;
        }
        u32 k = f.k, j;
        if (f.slot >= 0 && f.r > 0) {
            if (split_at(f) == NONE || status) return false;
            // the insertion point follows from the split: before the right piece, except when the
            // block split 4+4 right between the two pieces (blocks win ties: append to the left)
            const u32 s = (u32)f.slot;
            if (f.cnt + 1 < 8 || s + 1 < 4) {
                j = s + 1;
                f.cnt = f.cnt + 1 < 8 ? f.cnt + 1 : 4;
            } else if (s == 3) {
                j = 4;
                f.cnt = 4;
            } else {
                k = f.k + 1;
                j = s - 3;
                f.cnt = 4;
            }
        } else {
            j = f.slot >= 0 ? (u32)f.slot : f.cnt;
        }
        if (rec.len == 0) return false;  // blockInsert skips empty segments (:2196)
        rec.sid = new_sid();
        if (rec.sid == NONE) return false;
        const u32 b = insert_slot(k, f.cnt, j, rec, false, 0, 0);
        if (status) return false;
        if (seq > minSeq) add_lru(b, rec.sid, seq);
        return status == 0;
    }

    // markRangeRemoved (mergeTree.ts:2607-2719): split at p1 and p2, then mark [p1, p2) of the
    // (R, C) view before the op: first remover wins, later ones join removedClientOverlap.
    SD bool op_remove(i32 p1, i32 p2, i32 R, u32 C, i32 seq) {
        RG_PROF(RP_REM);
        // the p2 resolve and the marking start at p1's row: nothing before it moves or changes
        // visible length (a split keeps the lengths, a block split shifts only later blocks)
        u32 r1 = 0, c1 = 0;
        for (u32 ph = 0; ph < 2; ph++) {
            const RFound f = resolve(ph ? p2 : p1, R, C, r1, c1);
            if (ph == 0 && f.ok) {
                r1 = f.row;
                c1 = f.carry;
            }
            if (!f.ok || !(f.slot >= 0 && f.r > 0)) continue;
            if (split_at(f) == NONE || status) return false;
        }
        RG_PROF(RP_RANGE);
        const u32 nrows = (n_lb + 7) >> 3;
        u32 carry = c1;
        const u32 cbit = WIDE ? 1u << (C & 31u) : 1u << C;
        for (u32 r = r1; r < nrows && (i32)carry < p2; r++) {
            Row& w = rowref(r);
            const V v = vis(w, R, C);
            const V incl = simd::scan_incl(v) + carry;
            const V ex = incl - v;
            const B mark = (v != 0u) & simd::slt(ex, p2) & simd::sgt(incl, p1);
            carry = simd::readlane(incl, 63);
            const u64 mm = simd::ballot(mark);
            if (!mm) continue;
            const B was = mark & (w.rseq != RSEQ_LIVE);  // already removed: addOverlappingClient
            const B fresh = simd::andn(mark, was);
            if (WIDE && C >= 32) {
                if constexpr (WIDE) w.rm2 = simd::sel(mark, w.rm2 | cbit, w.rm2);
            } else {
                w.rm = simd::sel(mark, w.rm | cbit, w.rm);
            }
            w.meta = simd::sel(was, w.meta | F_OVL, simd::sel(fresh, (w.meta & ~0xFF00u) | (C << 8) | F_REMOVED, w.meta));
            w.rseq = simd::sel(fresh, (u32)seq, w.rseq);
            writeback(r);
            // addToLRUSet per block, document order: the first marked slot of each block
            for (u64 gm = mm; gm;) {
                const u32 l = (u32)__builtin_ctzll(gm);
                const u32 g = l >> 3;
                gm &= ~(0xFFull << (g * 8));
                add_lru(r * 8 + g, simd::readlane(w.sid, l), seq);
                if (status) return false;
            }
        }
        return status == 0;
    }

    // annotateRange (mergeTree.ts:2565-2605; PROPS): split at p1 and p2 like a remove, then every
    // segment of [p1, p2) visible in the (R, C) view takes a new map, addProperties of the op's set on
    // its old one (one map per distinct old map: the LDS engine's memo of the last one built).
    SD bool op_annotate(i32 p1, i32 p2, i32 R, u32 C, i32 seq, u32 propset, bool rewrite) {
        RG_PROF(RP_REM);
        u32 r1 = 0, c1 = 0;
        for (u32 ph = 0; ph < 2; ph++) {
            const RFound f = resolve(ph ? p2 : p1, R, C, r1, c1);
            if (ph == 0 && f.ok) {
                r1 = f.row;
                c1 = f.carry;
            }
            if (!f.ok || !(f.slot >= 0 && f.r > 0)) continue;
            if (split_at(f) == NONE || status) return false;
        }
        RG_PROF(RP_RANGE);
        const u32 nrows = (n_lb + 7) >> 3;
        u32 carry = c1, memoOld = NONE, memoNew = 0;
        for (u32 r = r1; r < nrows && (i32)carry < p2; r++) {
            Row& w = rowref(r);
            const V v = vis(w, R, C);
            const V incl = simd::scan_incl(v) + carry;
            const V ex = incl - v;
            const B mark = (v != 0u) & simd::slt(ex, p2) & simd::sgt(incl, p1);
            carry = simd::readlane(incl, 63);
            const u64 mm = simd::ballot(mark);
            if (!mm) continue;
            for (u64 pending = mm; pending;) {
                const u32 old = simd::readlane(w.props, (u32)__builtin_ctzll(pending));
                u32 nid;
                if (old == memoOld) {
                    nid = memoNew;
                } else {
                    nid = build_map(old, propset, rewrite);
                    if (status) return false;
                    memoOld = old;
                    memoNew = nid;
                }
                const B same = simd::ballot_mask(pending) & (w.props == old);
                w.props = simd::sel(same, nid, w.props);
                pending &= ~simd::ballot(same);
            }
            writeback(r);
            for (u64 gm = mm; gm;) {  // addToLRUSet per block, document order
                const u32 l = (u32)__builtin_ctzll(gm);
                const u32 g = l >> 3;
                gm &= ~(0xFFull << (g * 8));
                add_lru(r * 8 + g, simd::readlane(w.sid, l), seq);
                if (status) return false;
            }
        }
        return status == 0;
    }

    // Room for one more op (margins for the splits, packs and heap pushes an op can cause);
    // false => hand the document to the LDS engine before this op.
    SD bool room() {
        // level-1 nodes hold >= 1 leaf block each, so fewer than 57 blocks cannot reach lane 56 (and
        // the readlane, a VALU -> SALU round trip, is skipped)
        if constexpr (PAGED) {
            // rows are taken as blocks appear (ensure_blocks), so no block margin; pool rows past
            // the last block's row go back at once (a spare per wave, twelve per CU, had made the
            // pool run out on C2's peaks)
            const u32 keep = (n_lb + 7) >> 3;
            if (n_rows > keep) shrink_rows(keep);
            return n_lb + 4 <= lb_lim && heapSize + n_lb + 8 < RG_HEAP && height + 2 <= RG_LEVELS &&
                   (n_lb < 57 || simd::readlane(LV.get(0), 56) == 0u);
        }
        return n_lb + 16 <= lb_lim && heapSize + n_lb + 8 < RG_HEAP && height + 2 <= RG_LEVELS &&
               (n_lb < 57 || simd::readlane(LV.get(0), 56) == 0u);
    }

    // Client.applyMsg for one op record (client.ts:805-836); false => not applied, hand off.
    SD bool apply(const mte_op& op) {
        RG_PROF(RP_APPLY);
        RG_STAT(RS_OPS, 1);
        const u32 type = op.type;
        const bool ins = type == MTE_OP_INSERT || type == MTE_OP_INSERT_MARKER;
        const bool ann = PROPS && type == MTE_OP_ANNOTATE;
        if (!(ins || ann || type == MTE_OP_REMOVE || type == MTE_OP_NOOP)) return false;
        // (MTE_F_CATCHUP only asks for delta records, which only a legacy-format replay reads: that one
        // runs the EXT kernels, so here the flag is ignored like the lean LDS kernels do)
        if ((op.flags & (MTE_F_REL | MTE_F_PERM)) || (!PROPS && op.props)) return false;
        if (type != MTE_OP_NOOP && (op.client == 0 || op.client >= MAXC)) return false;
        if (!room()) return false;
        const u32 C = op.client;
        const i32 seq = op.seq, R = op.ref_seq;
        if (type != MTE_OP_NOOP && !(curSeq < seq)) {
            fail(MTE_DOC_SEQ_ORDER, seq);
            return true;
        }
        bool edited = false;
        if (ins) {
            RSeg rec;
            const bool mk = type == MTE_OP_INSERT_MARKER;
            rec.len = mk ? 1u : op.b;
            rec.seq = seq;
            rec.rseq = RSEQ_LIVE;
            rec.meta = (C & 0xFFu) | (RCL_LIVE << 8) | (mk ? F_MARKER : 0u);
            rec.toff = mk ? op.b : (u32)op.a;
            rec.cap = 0;
            rec.rm = 0;
            rec.sid = 0;
            if constexpr (PROPS) {
                rec.props = op.props ? build_map(0, op.props, false) : 0u;
                if (status) return true;
            }
            edited = op_insert(op.pos1, R, C, seq, rec);
            count_op();
        } else if (type == MTE_OP_REMOVE) {
            edited = op_remove(op.pos1, op.a, R, C, seq);
            count_op();
        } else if (ann) {
            if constexpr (PROPS) edited = op_annotate(op.pos1, op.a, R, C, seq, op.props, (op.flags & MTE_F_REWRITE) != 0);
            count_op();
        }
        if (status) return true;
        if (edited) {
            RG_PROF(RP_ZAM_EDIT);
            zamboni();
        }
        if (status) return true;
        if (op.flags & MTE_F_END_OF_MSG) {
            count_msg();
            if (op.seq < curSeq || op.msn > op.seq || op.msn < minSeq) {
                fail(MTE_DOC_SEQ_ORDER, op.seq);
                return true;
            }
            curSeq = op.seq;
            if (op.msn > minSeq) {
                RG_PROF(RP_MSN);
                minSeq = op.msn;
                zamboni();
            }
        }
        return true;
    }

    // Replay ops [i, e): returns the first op not applied (e when done or failed; earlier when the
    // document hands over to the LDS engine). Records are prefetched 8 per VGPR (lane 8*r + w holds
    // word w of record r), four chunks ahead.
    SD u64 replay(u64 i0, u64 e) {
        if (!p.docs[doc].collab) {  // local, non-collaborative edits: the LDS engine's path
            status = REG_HANDOFF;
            return i0;
        }
        RG_PROF(RP_TOTAL);
        // this document's records from one base pointer, indexed by 32-bit op numbers (a 64-bit
        // global op index in the loop held three more SGPR pairs in a kernel that spills SGPRs)
        const u32* src = (const u32*)p.ops + i0 * 8;
        const u32 n = (u32)(e - i0);
        auto load_chunk = [&](u32 c0) MTE_LI {  // records [c0, c0+8)
            const u32 left = n > c0 ? n - c0 : 0u;
            const u32 nw = left >= 8 ? 64u : left * 8u;
            return simd::ld(src + (u64)c0 * 8, L(), L() < nw);
        };
        // Two chunk registers: CUR holds the records being decoded, NXT the next eight. At a chunk's
        // first op CUR = NXT (loaded eight ops earlier), the op is decoded, and only THEN is NXT
        // refilled: the compiler waits for the whole vector-memory counter before a decode, so the
        // newest load outstanding there must be an op old. (Loading before the decode, or a
        // four-register ring indexed by a switch, made every chunk wait for a fresh HBM load.)
        V CUR = load_chunk(0), NXT = load_chunk(8);
#ifndef MTE_CPU
        // wait for the first chunk here, once: CUR then enters the loop with no load outstanding, so
        // the decodes need no vector-memory wait at all (stores of the merge arena included)
        asm volatile("" ::"v"(CUR.x));
#endif
        u32 k = 0;
        for (; k < n && !status; k++) {
            const u32 r = k & 7u;
            const bool first = r == 0 && k != 0;
            if (first) {
                CUR = NXT;
#ifndef MTE_CPU
                asm volatile("");  // keep this a branch: a select would read NXT (and wait) every op
#endif
            }
            mte_op op;
            {
                RG_PROF(RP_FETCH);
                u32 w[8];
                for (u32 x = 0; x < 8; x++) w[x] = simd::readlane(CUR, r * 8 + x);
                __builtin_memcpy(&op, w, sizeof op);
            }
            if (first) NXT = load_chunk(k + 8);
            RG_COUNT(RP_OPS, 1);
            if (!apply(op)) {
                status = REG_HANDOFF;
                return i0 + k;
            }
        }
        return i0 + k;
    }

    // ---------------------------------------------------------------- results
    // The final segments in document order (walkAllSegments, mergeTree.ts:2969-2983) in the LDS
    // engine's row format (removedSeq 0 and removedClient 0 for live segments), text gathered into
    // the document's run of the output text pool, and the per-document result record.
    SD u32 atomic_reserve(u32* ctr, u32 n) const {
#ifdef MTE_CPU
        const u32 o = *ctr;
        *ctr += n;
        return o;
#else
        u32 o = 0;
        if (simd::lane0()) o = atomicAdd(ctr, n);
        return __builtin_amdgcn_readfirstlane(o);
#endif
    }
    SD u64 atomic_reserve64(u64* ctr, u64 n) const {
#ifdef MTE_CPU
        const u64 o = *ctr;
        *ctr += n;
        return o;
#else
        u64 o = 0;
        if (simd::lane0()) o = atomicAdd((unsigned long long*)ctr, (unsigned long long)n);
        const u32 lo = __builtin_amdgcn_readfirstlane((u32)o), hi = __builtin_amdgcn_readfirstlane((u32)(o >> 32));
        return ((u64)hi << 32) | lo;
#endif
    }
    // the document leaves this engine unfinished (k_rows has no LDS plan to hand it to): the host
    // re-runs it HBM-resident from its first op (engine.hpp mark_spilled)
    SD void mark_spilled() {
        fence_arena();
        if (simd::lane0()) {
            DocRes& o = p.res[doc];
            o.status = DOC_SPILL;
            o.failing_seq = curSeq;
            o.n_segs = 0;
            o.max_lb = max_lb;
            o.mode = 0;
            o.spill_why = (n_lb << 8) | (heapSize << 20);
#ifndef MTE_CPU
            atomicAdd(&p.counters[2], 1u);
#endif
        }
    }
    SD void finish() {
        fence_arena();
        const u32 nrows = (n_lb + 7) >> 3;
        u32 nseg = 0, ntext = 0;
        for (u32 r = 0; r < nrows; r++) {
            const V len = ld_len(r);
            const B txt = (len != 0u) & ((ld_meta(r) & F_MARKER) == 0u);
            nseg += (u32)__builtin_popcountll(simd::ballot(len != 0u));
            ntext += simd::readlane(simd::scan_incl(simd::sel(txt, len, 0u)), 63);
        }
        u32 off = 0, toff = 0;
        if (status == 0) {
            off = atomic_reserve(&p.counters[1], nseg);
            toff = (u32)atomic_reserve64((u64*)&p.counters[6], ntext);
            if ((u64)off + nseg > p.out_cap || (u64)toff + ntext > p.out_text_cap) {
                fail(MTE_DOC_CAPACITY, curSeq);
                nseg = 0;
            }
        } else {
            nseg = 0;
        }
        if (nseg) {
            u32 run = off, trun = 0;
            u16* tdst = p.out_text + toff;
            u32* ov = (u32*)p.out_vis;
            u32* oa = (u32*)p.out_aux;
            u32* oo = (u32*)p.out_ovl;
            for (u32 r = 0; r < nrows; r++) {
                const Row w = ldrow(r);
                const B have = w.len != 0u;
                const B txt = have & ((w.meta & F_MARKER) == 0u);
                const V one = simd::sel(have, 1u, simd::splat(0));
                const V at = simd::scan_incl(one) - one + run;
                const V tl = simd::sel(txt, w.len, 0u);
                const V tat = simd::scan_incl(tl) - tl + trun;
                const B live = w.rseq == RSEQ_LIVE;
                const B hasov = (w.meta & F_OVL) != 0u;
                const V m2 = simd::sel(live, w.meta & ~0xFF00u, w.meta) & ~NS_MASK;
                // removedClientOverlap = the removers but removedClient (the LDS engine's format)
                V ovm, ovh = simd::splat(0);
                if constexpr (WIDE) {  // removedClient may be 32..63: its bit is in rm2 then
                    const V rc = simd::bfe(w.meta, 8, 8);
                    const V rcb = simd::shl(simd::splat(1), rc);  // bit rc & 31
                    const B rclo = rc < 32u;
                    ovm = w.rm & (simd::sel(rclo, rcb, 0u) ^ 0xFFFFFFFFu);
                    ovh = simd::sel(hasov, w.rm2 & (simd::sel(rclo, 0u, rcb) ^ 0xFFFFFFFFu), 0u);
                } else {
                    ovm = w.rm & (simd::shl(simd::splat(1), simd::bfe(w.meta, 8, 8)) ^ 0xFFFFFFFFu);
                }
                const V ovl = simd::sel(hasov, ovm, 0u);
                const V z2 = simd::sel(live, w.cap, ovl);
                const V t4 = at * 4u;
                simd::st(ov, t4, w.len, have);
                simd::st(ov, t4 + 1u, w.seq, have);
                simd::st(ov, t4 + 2u, simd::sel(live, 0u, w.rseq), have);
                simd::st(ov, t4 + 3u, m2, have);
                V pm = simd::splat(0);
                if constexpr (PROPS) pm = w.props;
                simd::st(oa, t4, pm, have);
                if constexpr (PROPS) {  // the row's property map, indexed by row (emission reads it)
                    const B hp = have & (w.props != 0u);
                    if (p.out_maps && simd::ballot(hp)) {
                        fence_arena();
                        for (u32 q = 0; q < mw; q++)
                            simd::st(p.out_maps, at * mw + q, simd::ld(maps, w.props * mw + q, hp), hp);
                    }
                }
                simd::st(oa, t4 + 1u, simd::sel(txt, tat, w.toff), have);
                simd::st(oa, t4 + 2u, z2, have);
                simd::st(oa, t4 + 3u, w.sid - 1u, have);
                simd::st(oo, at * 2u, ovl, have);
                simd::st(oo, at * 2u + 1u, ovh, have);
                if (p.out_ovl2) {  // clients 64..127: never on the rows (their first op hands over)
                    simd::st((u32*)p.out_ovl2, at * 2u, simd::splat(0), have);
                    simd::st((u32*)p.out_ovl2, at * 2u + 1u, simd::splat(0), have);
                }
                // text, one segment at a time, 64 units per step
                for (u64 tm = simd::ballot(txt); tm; tm &= tm - 1) {
                    const u32 l = (u32)__builtin_ctzll(tm);
                    copy_text(simd::readlane(tat, l), simd::readlane(w.toff, l), simd::readlane(w.len, l), tdst);
                }
                run += (u32)__builtin_popcountll(simd::ballot(have));
                trun += simd::readlane(simd::scan_incl(tl), 63);
            }
        }
        DocRes& o = p.res[doc];
        if (simd::lane0()) {
            o.status = status;
            o.failing_seq = status ? failSeq : -1;
            o.ops = ops_n();
            o.msgs = msgs_n();
            o.min_seq = minSeq;
            o.cur_seq = curSeq;
            o.height = height;
            o.n_lb = n_lb;
            o.arena_sel = arenaSel;
            o.arena_top = arenaTop;
            o.map_next = PROPS ? mapNext : 1u;
            o.seg_next = segNext;
            o.heap_size = heapSize;
            o.n_gc = n_gc;
            o.out_off = off;
            o.n_segs = nseg;
            o.text_off = toff;
            o.max_lb = max_lb;
            o.cu_n = 0;
            o.mode = res_mode;  // row-vectorised engine: 4 on k_solo, 5 on k_rows
            o.spill_why = 0;
        }
#if defined(MTE_PROFILE) && !defined(MTE_CPU)
        if (simd::lane0()) {
            static constexpr u32 map[RP_N] = {PF_TOTAL, PF_FETCH, PF_APPLY, PF_RESOLVE, PF_INSERT_SLOT, PF_SPLIT,
                                              PF_RANGE, PF_ZAMBONI, PF_SCOUR, PF_HEAP, PF_FIND_SEG, PF_PACK,
                                              PF_LRU, PF_OPS, PN_RESOLVE, PN_SCOUR, PN_SCOUR_CHANGED, PN_PACK,
                                              PN_POP, PN_SPLIT_BLK, PN_DIRTY, PF_ALLOC, PF_OP_INS, PF_OP_REM,
                                              PF_ZAM_MSN, PF_ZAM_EDIT};
            u64* o2 = p.prof + (u64)doc * PROF_SLOTS;
            for (u32 i = 0; i < RP_N; i++) o2[map[i]] += pf[i];
        }
#endif
    }

    // ---------------------------------------------------------------- checkpoints (incremental replay)
    // Client.applyMsg is incremental (client.ts:805-836): a reader interleaves getText with messages.
    // With Params::ck_out set, a document this engine finishes also leaves its whole replay state in
    // its checkpoint region (DocCfg::ck_out_off, ck_cap words); a later pass over a log that extends
    // this one (the host checks the prefix, mte_host.cpp ck_match) starts from that state at op
    // ck_at instead of op 0. The state is the engine's own: rows, interior levels, heap, scalars, the
    // live merge-arena semispace and the property maps -- nothing the replay does depends on where it
    // started, so the continued replay is the full one, op for op.
    // Region (words): header [0, CK_HDR), rows (NF fields of 64 words each, row by row), LV / HK / HS
    // (8 registers each), the arena semispace's [0, arenaTop) units, the map records [0, mapNext).
    static constexpr u32 CK_MAGIC = 0x434B5031u, CK_HDR = CK_HDR_WORDS;
    static_assert(RG_ROWS <= CK_MAX_ROWS, "checkpoint regions hold the whole row plan");
    enum : u32 { CK_VALID, CK_AT_LO, CK_AT_HI, CK_FLAGS, CK_NLB, CK_HEIGHT, CK_HEAPSIZE, CK_HEAPTOP, CK_MINSEQ,
                 CK_CURSEQ, CK_SEGNEXT, CK_ARENATOP, CK_ARENASEL, CK_MAPNEXT, CK_NOPS, CK_NMSGS, CK_NGC, CK_MAXLB,
                 CK_MW, CK_N };
    static constexpr u32 CK_NF = 8 + (PROPS ? 1u : 0u) + (WIDE ? 1u : 0u);
    // words a checkpoint of a document with these capacities can take (the host sizes regions by it)
    SD static u64 ck_words(u32 arena_cap, u32 map_cap, u32 map_words) { return ck_region_words(arena_cap, map_cap, map_words); }
    SD void ckpt_save(u64 at) {
        const DocCfg& c = p.docs[doc];
        if (!p.ck_out || !c.ck_cap || status || !rows_whole()) return;
        fence_arena();
        u32* base = p.ck_out + c.ck_out_off;
        const u32 nrows = (n_lb + 7) >> 3;
        const u64 rows_end = CK_HDR + (u64)nrows * CK_NF * 64, regs_end = rows_end + 24 * 64;
        const u64 ar_end = regs_end + ((u64)arenaTop + 1) / 2;
        const u64 end = ar_end + (PROPS ? (u64)mapNext * mw : 0);
        if (end > c.ck_cap) return;  // (the region stays invalid: the next pass replays from op 0)
        const V Lv = L();
        for (u32 rr = 0; rr < nrows; rr++) {
            const Row w = ldrow(rr);
            u32* o = base + CK_HDR + (u64)rr * CK_NF * 64;
            simd::st(o, Lv, w.len, simd::mk_all());
            simd::st(o + 64, Lv, w.seq, simd::mk_all());
            simd::st(o + 128, Lv, w.rseq, simd::mk_all());
            simd::st(o + 192, Lv, w.meta, simd::mk_all());
            simd::st(o + 256, Lv, w.cap, simd::mk_all());
            simd::st(o + 320, Lv, w.toff, simd::mk_all());
            simd::st(o + 384, Lv, w.rm, simd::mk_all());
            simd::st(o + 448, Lv, w.sid, simd::mk_all());
            if constexpr (PROPS) simd::st(o + 512, Lv, w.props, simd::mk_all());
            if constexpr (WIDE) simd::st(o + 64 * (CK_NF - 1), Lv, w.rm2, simd::mk_all());
        }
        u32* g = base + rows_end;
#pragma unroll
        for (u32 i = 0; i < 8; i++) {
            simd::st(g + 64 * i, Lv, LV.get(i), simd::mk_all());
            simd::st(g + 64 * (8 + i), Lv, HK.get(i), simd::mk_all());
            simd::st(g + 64 * (16 + i), Lv, HS.get(i), simd::mk_all());
        }
        copy_text(0, ARENA_BIT, arenaTop, reinterpret_cast<u16*>(base + regs_end));
        if constexpr (PROPS)
            for (u64 q = 0; q < (u64)mapNext * mw; q += 64) {
                const V i = Lv + (u32)q;
                const B m = i < (u32)((u64)mapNext * mw);
                simd::st(base + ar_end, i, simd::ld(maps, i, m), m);
            }
        const u32 flags = (PROPS ? 1u : 0u) | (WIDE ? 2u : 0u);
        const u32 hv[CK_N] = {0u, (u32)at, (u32)(at >> 32), flags, n_lb, height, heapSize, (u32)heapTop, (u32)minSeq,
                              (u32)curSeq, segNext, arenaTop, arenaSel, PROPS ? mapNext : 1u, ops_n(), msgs_n(), n_gc,
                              max_lb, PROPS ? mw : 0u};
        V h = simd::splat(0);
        for (u32 i = 1; i < CK_N; i++) h = simd::sel(Lv == i, hv[i], h);
        simd::st(base, Lv, h, Lv < (u32)CK_N);
        // the valid word last, after every other word of the region is out
        simd::wave_fence();
        simd::st(base, Lv, simd::splat(CK_MAGIC), Lv == 0u);
    }
    // Continue from the checkpoint of the previous pass (DocCfg::ck_at ops in, region ck_in_off of
    // Params::ck_in): returns the op to go on from, or i0 (state untouched: replay from the start)
    // when there is none or it does not fit this engine.
    SD u64 ckpt_resume(u64 i0) {
        const DocCfg& c = p.docs[doc];
        if (!p.ck_in || !c.ck_at || status) return i0;
        const u32* base = p.ck_in + c.ck_in_off;
        const V Lv = L();
        const V h = simd::ld(base, Lv, Lv < (u32)CK_N);
        auto hw = [&](u32 i) MTE_LI { return simd::readlane(h, i); };
        const u64 at = (u64)hw(CK_AT_LO) | ((u64)hw(CK_AT_HI) << 32);
        const u32 flags = hw(CK_FLAGS), nlb = hw(CK_NLB);
        const bool cprops = flags & 1u, cwide = (flags & 2u) != 0;
        // (a lean checkpoint continues on a PROPS / WIDE engine -- no maps, no high removers -- not the
        // other way round; a map table narrower than the records written is refused too)
        if (hw(CK_VALID) != CK_MAGIC || at != c.ck_at || (cprops && !PROPS) || (cwide && !WIDE) || nlb == 0 ||
            nlb > NBLK || hw(CK_HEIGHT) > RG_LEVELS + 1 || hw(CK_ARENATOP) > arena_cap || hw(CK_SEGNEXT) > seg_cap ||
            (cprops && (hw(CK_MW) != mw || hw(CK_MAPNEXT) > map_cap)))
            return i0;
        const u32 nrows = (nlb + 7) >> 3;
        if constexpr (PAGED) {
            if (!grow_rows(nrows)) {  // the pool is full now: k_rows restarts it or the host re-runs it
                status = REG_HANDOFF;
                return i0;
            }
        }
        const u32 cnf = 8 + (cprops ? 1u : 0u) + (cwide ? 1u : 0u);
        for (u32 rr = 0; rr < nrows; rr++) {
            const u32* o = base + CK_HDR + (u64)rr * cnf * 64;
            Row w;
            w.len = simd::ld(o, Lv, simd::mk_all());
            w.seq = simd::ld(o + 64, Lv, simd::mk_all());
            w.rseq = simd::ld(o + 128, Lv, simd::mk_all());
            w.meta = simd::ld(o + 192, Lv, simd::mk_all());
            w.cap = simd::ld(o + 256, Lv, simd::mk_all());
            w.toff = simd::ld(o + 320, Lv, simd::mk_all());
            w.rm = simd::ld(o + 384, Lv, simd::mk_all());
            w.sid = simd::ld(o + 448, Lv, simd::mk_all());
            if constexpr (PROPS) w.props = cprops ? simd::ld(o + 512, Lv, simd::mk_all()) : simd::splat(0);
            if constexpr (WIDE) w.rm2 = cwide ? simd::ld(o + 64 * (cnf - 1), Lv, simd::mk_all()) : simd::splat(0);
            strow(rr, w);
        }
        cr = NONE;
        const u64 rows_end = CK_HDR + (u64)nrows * cnf * 64, regs_end = rows_end + 24 * 64;
        const u32* g = base + rows_end;
#pragma unroll
        for (u32 i = 0; i < 8; i++) {
            LV.set(i, simd::ld(g + 64 * i, Lv, simd::mk_all()));
            HK.set(i, simd::ld(g + 64 * (8 + i), Lv, simd::mk_all()));
            HS.set(i, simd::ld(g + 64 * (16 + i), Lv, simd::mk_all()));
        }
        n_lb = nlb;
        height = hw(CK_HEIGHT);
        heapSize = hw(CK_HEAPSIZE);
        heapTop = (i32)hw(CK_HEAPTOP);
        minSeq = (i32)hw(CK_MINSEQ);
        curSeq = (i32)hw(CK_CURSEQ);
        segNext = hw(CK_SEGNEXT);
        arenaTop = hw(CK_ARENATOP);
        arenaSel = hw(CK_ARENASEL) & 1u;
        set_counts(hw(CK_NOPS), hw(CK_NMSGS));
        n_gc = hw(CK_NGC);
        max_lb = hw(CK_MAXLB);
        // the arena text into this pass's semispace arenaSel (offsets kept: the rows' toff stay valid)
        {
            const u16* src = reinterpret_cast<const u16*>(base + regs_end);
            u16* dst = arena_cur();
            for (u32 b = 0; b < arenaTop; b += 64) {
                const V i = Lv + b;
                const B m = i < arenaTop;
                simd::st(dst, i, simd::ld(src, i, m), m);
            }
        }
        if constexpr (PROPS) {
            mapNext = cprops ? hw(CK_MAPNEXT) : 1u;
            const u32* src = base + regs_end + ((u64)arenaTop + 1) / 2;
            const u32 nw = cprops ? mapNext * mw : 0u;
            for (u32 q = 0; q < nw; q += 64) {
                const V i = Lv + q;
                const B m = i < nw;
                simd::st(maps, i, simd::ld(src, i, m), m);
            }
        }
        adirty = true;  // arena and map words written lane-parallel: fence before they are read
        if (simd::lane0()) {  // counters[12] / [13]: documents and op records resumed this pass
#ifdef MTE_CPU
            p.counters[12] += 1;
            p.counters[13] += (u32)at;
#else
            atomicAdd(&p.counters[12], 1u);
            atomicAdd(&p.counters[13], (u32)at);
#endif
        }
        return i0 + at;
    }
};

}  // namespace mte
