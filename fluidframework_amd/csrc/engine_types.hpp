// engine_types.hpp — plain data shared by the HIP kernels and the host side of the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mte.h"

namespace mte {

typedef uint32_t u32;
typedef int32_t i32;
typedef uint64_t u64;
typedef uint16_t u16;

constexpr u32 NONE = 0xFFFFFFFFu;
constexpr u32 ARENA_BIT = 0x80000000u;
constexpr u32 SC_UNDEF = 0, SC_TRUE = 1, SC_FALSE = 2;   // needsScour tri-state (mergeTree.ts:63)
constexpr u32 F_REMOVED = 1u << 16, F_MARKER = 1u << 17;  // Slot.meta flags
constexpr u32 MAP_WORDS = 16;                            // [0]=count, then 7 (key,val) pairs
constexpr i32 GRANULARITY = 256;                         // TextSegmentGranularity (mergeTree.ts:1059)

// Visibility-relevant part of a leaf slot: 16 bytes, one dwordx4 load per lane.
struct Slot {
    u32 len;
    i32 seq;
    i32 rseq;
    u32 meta;  // client | rclient << 8 | flags
};

struct SegRec {
    Slot v;
    u64 ovl;      // removedClientOverlap as a short-id mask
    u32 props;    // property-map id (0 = undefined)
    u32 toff;     // text offset (ARENA_BIT => merge arena, else doc payload); marker: refType
    u32 tcap;     // owned arena capacity from toff (0 for payload text)
    u32 sid;      // segment id (LRU heap identity)
};

// Host-computed per-document layout.
struct DocCfg {
    u64 op_begin, op_end;
    u64 payload_off;
    u64 arena_off;     // two semispaces of arena_cap units each
    u64 seg_off;
    u64 heap_off;
    u64 lbo_off;
    u64 map_off;
    u32 payload_len;
    u32 arena_cap;
    u32 seg_cap;
    u32 heap_cap;
    u32 lbo_cap;
    u32 map_cap;
    u32 collab;        // 1 = observer replay, 0 = local non-collaborative edits
    u32 pad;
};

// Per-document results written by the kernel.
struct DocRes {
    i32 status;
    i32 failing_seq;
    u32 ops;
    u32 msgs;
    i32 min_seq;
    i32 cur_seq;
    u32 root;
    u32 height;
    u32 n_lb;
    u32 arena_sel;
    u32 arena_top;
    u32 map_next;
    u32 seg_next;
    u32 heap_size;
    u32 n_gc;
    u32 lb_free;
};

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
    const u32* doc_order;
    u32 n_docs;
    u32 pad0;
    DocRes* res;
    u16* arena;
    u32* seg_parent;
    uint2* heap;
    u32* lbo;
    u32* maps;
    uint4* lb_vis;
    u64* lb_ovl;
    u32* lb_props;
    uint2* lb_txt;
    u32* lb_sid;
    u32* lb_cnt;
    u32* lb_par;
    u32* lb_scour;
    u32* in_child;
    u32* in_cnt;
    u32* in_par;
    u32* counters;  // [0] leaf-block bump, [1] internal-node bump
    u32 nlb_cap, nin_cap;
    // synthetic workload generator
    u32* gen_first_seen;  // per doc: 64 entries, writer index for each short id (1..)
    u32 gen_kind;
    u32 gen_nclients;
    u64 gen_seed;
    u32 gen_n_propsets;   // propset ids 1..gen_n_propsets are the generator's annotate sets
    u32 pad1;
};

}  // namespace mte
