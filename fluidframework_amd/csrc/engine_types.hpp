// engine_types.hpp — plain data shared by the HIP kernels and the host side of the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mte.h"

#define MTE_HOSTDEV_ __host__ __device__ inline

namespace mte {

typedef uint32_t u32;
typedef int32_t i32;
typedef uint64_t u64;
typedef uint16_t u16;

constexpr u32 NONE = 0xFFFFFFFFu;
constexpr u32 ARENA_BIT = 0x80000000u;
constexpr u32 SC_UNDEF = 0, SC_TRUE = 1, SC_FALSE = 2;   // needsScour tri-state (mergeTree.ts:63)
constexpr u32 F_REMOVED = 1u << 16, F_MARKER = 1u << 17;  // slot meta flags
constexpr u32 F_OVL = 1u << 18;    // removedClientOverlap non-empty: clients 0..31 in aux.z (dead tcap)
constexpr u32 F_OVLHI = 1u << 19;  // ... and clients 32..63 in the HBM mask by segment id
constexpr u32 F_PERM = 1u << 20;   // PermutationSegment run (SharedMatrix row / col vector): no text
constexpr u32 MAP_WORDS = 16;  // the narrowest map record: [0] = count, then 7 (key, val) pairs; a batch
                               // whose documents carry more distinct keys gets wider records
                               // (Params::map_words = 1 + 2 * keys, rounded up to 4, <= 128)
constexpr i32 GRANULARITY = 256;                         // TextSegmentGranularity (mergeTree.ts:1059)

// Per output row, the emission's view of its text (EmitParams::esc, written by k_emit_count for k_emit_write):
// the bytes JSON.stringify writes for the row's text alone, quotes excluded (UTF-8, '"' '\\' and control
// characters escaped, an unpaired surrogate as \uXXXX), and the flags the SnapshotV1 writer needs
// without reading the text or the aux row: the text starts with a low / ends with a high surrogate (a
// pair joined across two rows of a run is 4 bytes, not 6 + 6), ends with '\n' (TextSegment.canAppend),
// and the row has a property map. Markers and permutation runs: 0 bytes, the props flag only.
constexpr u32 ESC_LEN = 0x0FFFFFFFu, ESC_NL = 1u << 28, ESC_PROPS = 1u << 29, ESC_LO = 1u << 30, ESC_HI = 1u << 31;
MTE_HOSTDEV_ bool esc_is_hi(u32 c) { return c >= 0xD800u && c < 0xDC00u; }
MTE_HOSTDEV_ bool esc_is_lo(u32 c) { return c >= 0xDC00u && c < 0xE000u; }
// bytes of one UTF-16 unit c after `prev` inside one JSON string (emit.hip put_quoted): a high surrogate
// counts 6 and its low partner -2, so a joined pair totals 4 (6 + 6 for unpaired units)
MTE_HOSTDEV_ i32 esc_unit(u32 c, u32 prev) {
    if (c == '"' || c == '\\') return 2;
    if (c < 0x20u) return (c == '\b' || c == '\f' || c == '\n' || c == '\r' || c == '\t') ? 2 : 6;
    if (esc_is_hi(c)) return 6;
    if (esc_is_lo(c)) return esc_is_hi(prev) ? -2 : 6;
    return c < 0x80u ? 1 : c < 0x800u ? 2 : 3;
}

// Leaf-block metadata word: parent interior node (bits 0..29) | needsScour (bits 30..31).
constexpr u32 BM_PAR = 0x3FFFFFFFu;
constexpr u32 BM_NOPAR = 0x3FFFFFFFu;

// ------------------------------------------------------------------------------------------------
// LDS plan of the replay kernel: ONE workgroup per CU with LDS_WAVES waves; each wave replays one
// document at a time (persistent doc queue). Per-document structures live in the wave's region;
// leaf blocks (8 slots of 32 B) come from a pool shared by the CU's waves, so one large document
// can borrow blocks that the others do not need.
constexpr u32 LDS_WAVES = 8;
constexpr u32 LDS_BYTES = 163840;  // 160 KiB per CU (MI355X_MICROARCH.md), one workgroup declares all of it
constexpr u32 ORD_CAP = 128;       // leaf blocks per document while resident in LDS
#ifndef MTE_IN_CAP
#define MTE_IN_CAP 48
#endif
#ifndef MTE_HEAP_CAP
#define MTE_HEAP_CAP 255  // 191: C2 +2.6 % (A/B, profiles/ab_r03: half as many documents continue HBM-resident); 127: +11 %
#endif
constexpr u32 IN_CAP = MTE_IN_CAP;      // interior nodes per document while resident in LDS
constexpr u32 HEAP_CAP = MTE_HEAP_CAP;  // LRU heap entries per document while resident in LDS
constexpr u32 RING_OPS = 32;       // op records staged per wave (prefetched one batch ahead)
constexpr u32 OP_CREDIT = 4;       // leaf blocks a wave holds in reserve before each op

struct WaveRegion {
    uint4 ord[ORD_CAP];         // doc order: (block id, observer-visible length, max seq, child count)
    u32 in_child[IN_CAP * 8];
    u32 in_cnt[IN_CAP];
    u32 in_par[IN_CAP];
    uint2 heap[HEAP_CAP + 1];   // 1-based binary heap of (segment id, maxSeq)
    mte_op ring[RING_OPS];
    u32 scratch[64];
    u16 hint[256];              // LRU heap: segment id (mod 256) -> leaf block
    u32 stats[8];               // per-document counters (engine.hpp ST_*)
};
constexpr u32 ST_OPS = 0, ST_MSGS = 1, ST_GC = 2, ST_MAXLB = 3, ST_FAILSEQ = 4, ST_APPEND = 5, ST_CU = 6, ST_WORDS = 8;
constexpr u32 POOL_HDR = 80;  // 16-word allocation bitmap + pool_avail
constexpr u32 POOL_BLOCKS = ((LDS_BYTES - LDS_WAVES * (u32)sizeof(WaveRegion) - POOL_HDR - 16) / (8 * 32 + 4 + 1)) & ~3u;

struct LdsPlan {
    u32 bitmap[16];              // 1 = block taken (or beyond the pool)
    u32 pool_avail;              // blocks neither owned nor held as credit by any wave
    u32 pool_pad[3];
    WaveRegion wave[LDS_WAVES];
    uint4 vis[POOL_BLOCKS * 8];  // len, seq, removedSeq, client | removedClient << 8 | flags
    uint4 aux[POOL_BLOCKS * 8];  // props map id, text offset, owned text capacity, segment id
    u32 bmeta[POOL_BLOCKS];
    unsigned char owner[POOL_BLOCKS];  // wave holding the block (0xFF = free)
};
static_assert(sizeof(LdsPlan) <= LDS_BYTES, "LDS plan exceeds 160 KiB");
static_assert(POOL_BLOCKS <= 16 * 32, "bitmap too small");

// LDS plan of the solo kernel (k_solo): ONE wave owns a whole CU's LDS and replays one
// critical-path document (the Zipf heads of C4) with room for the block list, interior
// nodes and LRU heap such a long document reaches, so it never has to continue HBM-resident.
constexpr u32 SOLO_ORD = 512;
constexpr u32 SOLO_IN = 192;
constexpr u32 SOLO_HEAP = 1023;
constexpr u32 SOLO_HINTS = 1024;
struct SoloRegion {
    uint4 ord[SOLO_ORD];
    u32 in_child[SOLO_IN * 8];
    u32 in_cnt[SOLO_IN];
    u32 in_par[SOLO_IN];
    uint2 heap[SOLO_HEAP + 1];
    mte_op ring[RING_OPS];
    u32 scratch[64];
    u16 hint[SOLO_HINTS];
    u32 stats[8];
};
constexpr u32 SOLO_POOL = ((LDS_BYTES - (u32)sizeof(SoloRegion) - 64) / (8 * 32 + 4)) & ~3u;
struct SoloPlan {
    SoloRegion w;
    uint4 vis[SOLO_POOL * 8];
    uint4 aux[SOLO_POOL * 8];
    u32 bmeta[SOLO_POOL];
};
static_assert(sizeof(SoloPlan) <= LDS_BYTES, "solo LDS plan exceeds 160 KiB");
// block ids below MAX_POOL are LDS ids of a document that continued HBM-resident
constexpr u32 MAX_POOL = SOLO_POOL > POOL_BLOCKS ? SOLO_POOL : POOL_BLOCKS;

constexpr u64 OVL2_NONE = ~0ull;   // DocCfg::ovl2_off of a document whose window holds <= 64 clients
constexpr u32 GEN_MAX_CLIENTS = 64;  // the synthetic generator's writers (short ids 1..63)

// Host-computed per-document layout.
struct DocCfg {
    u64 op_begin, op_end;
    u64 payload_off;
    u64 arena_off;     // two semispaces of arena_cap units each
    u64 ovl_off;       // per segment id: removedClientOverlap mask (u64; clients 32..63 used)
    u64 ovl2_off;      // ... clients 64..127 (Params::ovl2), OVL2_NONE unless the window exceeds 64 clients
    u64 map_off;
    u64 hb_off;        // byte offset of this doc's HBM-resident state (HBM mode only)
    u64 cu_off;        // first catch-up delta record (Params::cu_rec, 2 x uint4 each) of this doc
    u32 cu_cap;        // catch-up delta records it may write (MTE_F_CATCHUP ops)
    u32 ht_cap;        // SharedMatrix vector with cell ops: HandleTable slots (cell records + 2), else 0
    u64 ht_off;        // its HandleTable in Params::htab: [length, handles[ht_cap], last free seq[ht_cap]]
    u32 payload_len;
    u32 arena_cap;
    u32 seg_cap;       // segment ids available
    u32 map_cap;
    u32 hb_blk, hb_ord, hb_in, hb_heap;  // HBM-mode capacities
    u32 collab;        // 1 = observer replay, 0 = local non-collaborative edits
    u32 has_nl;        // payload contains '\n' (TextSegment.canAppend reads last chars only then)
    u32 prio;          // critical-path document (far longer than the batch mean): high wave priority
    u32 gid;           // global document id (summary records; the generator's per-document seed)
    // incremental replay (option retain, reg_engine.hpp ckpt_*): this pass's checkpoint region in
    // Params::ck_out (ck_cap words, 0 = none) and, when the loaded log extends the previous pass's, the
    // previous region in Params::ck_in and the op records it covers (ck_at, 0 = replay from op 0)
    u64 ck_out_off, ck_cap, ck_in_off, ck_at;
};

// Per-document results written by the kernel.
struct DocRes {
    i32 status;
    i32 failing_seq;
    u32 ops;
    u32 msgs;
    i32 min_seq;
    i32 cur_seq;
    u32 height;
    u32 n_lb;
    u32 arena_sel;
    u32 arena_top;
    u32 map_next;
    u32 seg_next;
    u32 heap_size;
    u32 n_gc;
    u32 out_off;     // first row of this doc's final segments in the output pool
    u32 n_segs;
    u32 max_lb;      // peak leaf-block count
    u32 mode;        // 0 LDS-resident, 1 HBM-resident (k_hbmq / host re-run), 2 continued HBM-resident,
                     // 3 solo LDS-resident, 4 solo row engine, 5 k_rows, 6 k_rows then HBM-resident (k_rows_cont)
    u32 spill_why;   // why the LDS pass gave the doc up (engine.hpp St::spillWhy)
    u32 text_off;    // first unit of this doc's gathered final text in the output text pool
    u32 cu_n;        // catch-up delta records written (Engine::cu_record)
};

// internal status: the LDS-resident replay ran out of room (leaf-block pool, interior nodes, heap
// or block list); the doc's LDS state is dropped and the host re-runs it HBM-resident
constexpr i32 DOC_SPILL = 100;

struct Params {
    mte_op* ops;
    u16* payload;
    const mte_propset* propsets;
    const u32* prop_keys;
    const u32* prop_vals;
    const u32* val_flags;     // bit0: JS-falsy; bit1: object-typed (matchProperties recurses)
    const u64* val_objmatch;  // per value: bit j = matchProperties(value, objvalue j)
    const u32* val_objidx;    // per value: index among object-typed values (or NONE)
    u32 n_propsets;
    u32 n_vals;
    const DocCfg* docs;
    const u32* doc_list;      // docs to run, in start order (LPT)
    u32 n_list;
    u32 n_docs;
    DocRes* res;
    u16* arena;
    u64* ovl;
    u64* ovl2;                // removedClientOverlap of clients 64..127 (DocCfg::ovl2_off), or null
    u32* maps;
    unsigned char* hbm;       // HBM-mode per-doc state (DocCfg::hb_off)
    uint4* out_vis;           // final segments, doc order (output pool)
    uint4* out_aux;
    u64* out_ovl;
    u64* out_ovl2;            // ... clients 64..127 of each final row (null without such documents)
    u64 out_cap;
    u16* out_text;            // final segment texts, one run per document (Engine::finish)
    u32* out_maps;            // property map of each final row with props (MAP_WORDS per row), or null
    u64 out_text_cap;
    u32* counters;            // [0] doc queue, [1] output rows, [2] docs re-run by the host,
                              // [3] unused, [4] docs continued HBM-resident, [5] k_lds critical-path
                              // queue, [6..7] output text units (u64),
                              // [8] / [9] k_rows restarts pushed / popped, [10] k_rows documents
                              // dumped for k_rows_cont (16 words, zeroed before each pass)
    unsigned char* spill;     // per-wave HBM slots (slot_bytes each): LDS waves 0..8G-1 keep theirs for
                              // documents that outgrow the LDS plan, HBM waves use slot_hbm0 + blockIdx
    u64 slot_bytes;
    u32 slot_blk, slot_ord, slot_in, slot_heap;  // capacities of a slot (hbm_caps of the longest doc)
    u32 slot_hbm0;            // first slot of the k_hbmq waves (after the LDS waves' slots)
    u32* slot_bits;           // k_hbmq slot bitmap (n_hslots bits, 1 = held)
    u32 n_hslots;
    u32 lds_active;           // waves per k_lds workgroup that take documents (spread small batches)
    u32 n_prio;               // doc_list[0 .. n_prio): critical-path documents, taken by LDS waves only
    u32 n_solo;               // doc_list[0 .. n_solo) <= n_prio: one k_solo workgroup each
    unsigned char* solo_spill;  // per solo document: an HBM slot for continuing (solo_slot_bytes each)
    u64 solo_slot_bytes;
    u32 solo_blk, solo_ord, solo_in, solo_heap;  // capacities of a solo slot (hbm_caps of its longest doc)
    u32 pool_limit;           // test knob: LDS leaf blocks usable per CU (0 = all)
    u64* prof;                // MTE_PROFILE builds: per doc PROF_SLOTS cycle counters
    uint4* cu_rec;            // catch-up delta records: (op index in the doc, position, length, kind),
                              // (map after, map before, 0, 0); kind 0 insert, 1 remove, 2 annotate
    // synthetic workload generator
    u32* gen_first_seen;      // per doc: GEN_MAX_CLIENTS entries, writer index for each short id (1..)
    u32 gen_kind;
    u32 gen_nclients;
    u64 gen_seed;
    u32 gen_n_propsets;       // propset ids 1..gen_n_propsets are the generator's annotate sets
    u32 reg_solo;             // k_solo replays lean documents register-resident first (reg_engine.hpp)
    u32 reg_lb_limit;         // test knob: leaf blocks the register plan may hold (0 = all it has)
    u32 map_words;            // words per property-map record (a multiple of 4, >= MAP_WORDS)
    u32 map_rerun;            // 1 in the host's re-run pass: a full map table is a capacity failure
    // SharedMatrix cell ops (MTE_OP_CELL): pass 1 (cell_mode 1) writes each record's adjustPosition
    // (NONE = undefined) to cell_pos[2 * cell + col]; pass 2 (cell_mode 2) allocates the handles of the
    // cells both vectors defined and writes them to cell_h (0 = none)
    u32 cell_mode;
    u32* cell_pos;
    u32* cell_h;
    u32* htab;
    const u32* htab0;         // each HandleTable's state at document start (new, or loaded from a summary)
    u64* solo_clk;            // per solo workgroup: s_memtime / s_memrealtime at its replay's start and
                              // end (4 u64): shader cycles vs the 100 MHz reference clock; then, at
                              // [4 * SOLO_CLK_SLOTS], the bulk kernel's start (s_memrealtime)
    u32* solo_started;        // solo workgroups that have started this pass (k_solo_gate waits for n_solo)
    u32* rows_retry;          // k_rows: documents the row pool could not grow, queued to restart once
                              // (doc + 1 per slot; counters[8] pushed, counters[9] popped), or null
    u32 rows_pool_lim;        // test knob: k_rows pool rows usable per CU (0 = all of the pool)
    u32* rows_cont;           // k_rows: documents handed to an HBM slot mid-pass, ROWS_CONT_WORDS each
                              // (doc, slot, op index lo / hi, the HBM engine's St); counters[10] queued,
                              // counters[11] taken by k_rows_cont
    u32* ck_out;              // option retain: the row engines' checkpoints of this pass (DocCfg::ck_*)
    const u32* ck_in;         // ... and of the previous pass, the ones this pass continues from
};
constexpr u32 ROWS_CONT_WORDS = 32;

// A checkpoint region (option retain, reg_engine.hpp ckpt_save): header, up to CK_MAX_ROWS rows of up
// to 10 fields, 24 registers, the arena semispace (u16 units) and the map records, in words.
constexpr u32 CK_MAX_ROWS = 32, CK_HDR_WORDS = 64;
MTE_HOSTDEV_ u64 ck_region_words(u32 arena_cap, u32 map_cap, u32 map_words) {
    return CK_HDR_WORDS + (u64)CK_MAX_ROWS * 10 * 64 + 24 * 64 + ((u64)arena_cap + 1) / 2 + (u64)map_cap * map_words;
}

constexpr u32 SOLO_CLK_SLOTS = 64;  // solo workgroups with clock stamps (Params::solo_clk)

// MTE_PROFILE builds: s_memtime cycles per engine phase, per document (engine.hpp PROF_*).
constexpr u32 PROF_SLOTS = 40;

// HBM-resident capacities of a document with n ops (leaf blocks hold >= 4 segments except
// transiently; segments <= 2 per op + 1 without zamboni). Block ids below POOL_BLOCKS are the
// LDS ids of a document that continued in HBM, fresh ids start above them.
MTE_HOSTDEV_ void hbm_caps(u64 n, u32& blk, u32& ord, u32& in, u32& heap) {
    u64 b = n / 2 + 64 + MAX_POOL;
    if (b > 0x3FFFFFF0ull) b = 0x3FFFFFF0ull;
    blk = (u32)b;
    ord = (u32)b;
    u64 i = b / 2 + 64;
    in = (u32)(i > 0x3FFFFFF0ull ? 0x3FFFFFF0ull : i);
    u64 h = 2 * n + 64;
    heap = (u32)(h > 0x3FFFFFF0ull ? 0x3FFFFFF0ull : h);
}

constexpr u32 HBM_HINTS = 1024;  // HBM mode: segment id (mod 1024) -> leaf block at LRU push

// HBM-mode state layout of one document (byte offsets from DocCfg::hb_off).
struct HbmLayout {
    MTE_HOSTDEV_ static u64 a16(u64 n) { return (n + 15) & ~15ull; }
    u64 vis, aux, bmeta, ord, in_child, in_cnt, in_par, heap, scratch, hint, bytes;
    MTE_HOSTDEV_ static HbmLayout of(u32 blk, u32 ord, u32 in, u32 heap) {
        HbmLayout l;
        u64 o = 0;
        l.vis = o;
        o += a16((u64)blk * 8 * 16);
        l.aux = o;
        o += a16((u64)blk * 8 * 16);
        l.bmeta = o;
        o += a16((u64)blk * 4);
        l.ord = o;
        o += a16((u64)ord * 16);
        l.in_child = o;
        o += a16((u64)in * 8 * 4);
        l.in_cnt = o;
        o += a16((u64)in * 4);
        l.in_par = o;
        o += a16((u64)in * 4);
        l.heap = o;
        o += a16((u64)(heap + 1) * 8);
        l.scratch = o;  // 64 words of per-lane scratch, then the per-document counters (stats)
        o += 128 * 4;
        l.hint = o;
        o += HBM_HINTS * 4;
        l.bytes = o;
        return l;
    }
};

}  // namespace mte
