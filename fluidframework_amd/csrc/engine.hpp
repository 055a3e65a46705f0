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

// Phase profiling (compile with -DMTE_PROFILE): inclusive s_memtime cycles per phase.
enum ProfSlot : u32 {
    PF_APPLY = 0, PF_RESOLVE, PF_INSERT_SLOT, PF_RANGE, PF_ZAMBONI, PF_SCOUR, PF_HEAP, PF_FIND_SEG,
    PF_MAP, PF_PACK, PF_FETCH, PF_LRU, PF_TEXT, PF_ALLOC, PF_OPS, PF_TOTAL
};
#ifdef MTE_PROFILE
struct ProfScope {
    u64& acc;
    u64 t0;
    MTE_DEV ProfScope(u64& a) : acc(a), t0(__builtin_amdgcn_s_memtime()) {}
    MTE_DEV ~ProfScope() { acc += __builtin_amdgcn_s_memtime() - t0; }
};
#define MTE_PROF(slot) ProfScope _prof_scope_##slot(prof[slot])
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

// Uniform replay state (identical in every lane).
struct St {
    u32 root, height, n_lb, max_lb;
    i32 minSeq, curSeq;
    u32 heapSize, segNext, arenaTop, arenaSel, mapNext;
    u32 lbFree, lbBump, inFree, inBump, inUsed;
    i32 status, failingSeq;
    u32 opsApplied, msgs, nGc;
    u32 adirty, gdirty;
};

template <bool LDSM>
struct Engine {
    const Params& p;
    DocCfg cfg;
    u32 doc;
    u32 L;  // lane
    St st;
    bool collab, has_nl;
#ifdef MTE_PROFILE
    u64 prof[PROF_SLOTS];
#endif
    // state arrays (LDS-resident for LDSM, else HBM-resident)
    uint4* vis;  // by block id * 8 + slot
    uint4* aux;
    u32* bmeta;  // by block id: parent | needsScour << 30
    uint4* ord;  // doc order: (block id, observer-visible length, max seq, child count)
    u32* in_child;
    u32* in_cnt;
    u32* in_par;
    uint2* heap;
    u32* scratch;
    mte_op* ring;
    u32 blk_cap, ord_cap, in_cap, heap_cap;
    u32* bitmap;             // LDS pool allocation bitmap
    unsigned char* owner;    // LDS pool block -> wave
    u32 wave;
    // doc-relative HBM bases
    u16* payload;
    u16* arena0;
    u64* ovl;
    u32* maps;

    MTE_DEV Engine(const Params& p_, u32 doc_) : p(p_), cfg(p_.docs[doc_]), doc(doc_) {
        L = lane_id();
#ifdef MTE_PROFILE
        for (u32 i = 0; i < PROF_SLOTS; i++) prof[i] = 0;
#endif
        payload = p.payload + cfg.payload_off;
        arena0 = p.arena + cfg.arena_off;
        ovl = p.ovl + cfg.ovl_off;
        maps = p.maps + cfg.map_off * MAP_WORDS;
        collab = cfg.collab != 0;
        has_nl = cfg.has_nl != 0;
        st.root = NONE;
        st.height = 1;
        st.n_lb = st.max_lb = 0;
        st.minSeq = st.curSeq = 0;
        st.heapSize = st.segNext = st.arenaTop = st.arenaSel = 0;
        st.mapNext = 1;  // map id 0 == undefined
        st.lbFree = st.inFree = NONE;
        st.lbBump = st.inBump = st.inUsed = 0;
        st.status = 0;
        st.failingSeq = -1;
        st.opsApplied = st.msgs = st.nGc = 0;
        st.adirty = st.gdirty = 0;
        bitmap = nullptr;
        owner = nullptr;
        wave = 0;
        ring = nullptr;
    }

    MTE_DEV void bind_lds(LdsPlan* lp, u32 w) {
        WaveRegion& r = lp->wave[w];
        vis = lp->vis;
        aux = lp->aux;
        bmeta = lp->bmeta;
        ord = r.ord;
        in_child = r.in_child;
        in_cnt = r.in_cnt;
        in_par = r.in_par;
        heap = r.heap;
        scratch = r.scratch;
        ring = r.ring;
        blk_cap = POOL_BLOCKS;
        ord_cap = ORD_CAP;
        in_cap = IN_CAP;
        heap_cap = HEAP_CAP;
        bitmap = lp->bitmap;
        owner = lp->owner;
        wave = w;
    }
    MTE_DEV void bind_hbm() {
        HbmLayout l = HbmLayout::of(cfg.hb_blk, cfg.hb_ord, cfg.hb_in, cfg.hb_heap);
        unsigned char* b = p.hbm + cfg.hb_off;
        vis = (uint4*)(b + l.vis);
        aux = (uint4*)(b + l.aux);
        bmeta = (u32*)(b + l.bmeta);
        ord = (uint4*)(b + l.ord);
        in_child = (u32*)(b + l.in_child);
        in_cnt = (u32*)(b + l.in_cnt);
        in_par = (u32*)(b + l.in_par);
        heap = (uint2*)(b + l.heap);
        scratch = (u32*)(b + l.scratch);
        blk_cap = cfg.hb_blk;
        ord_cap = cfg.hb_ord;
        in_cap = cfg.hb_in;
        heap_cap = cfg.hb_heap;
    }

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
            st.failingSeq = seq;
        }
    }

    // ---------------------------------------------------------------- slots
    MTE_DEV Seg load(u32 blk, u32 s) const {
        Seg g;
        if (blk >= blk_cap || s >= 8) {
            g.len = 0;
            g.seq = g.rseq = 0;
            g.meta = g.props = g.toff = g.tcap = 0;
            g.sid = NONE;
            return g;
        }
        u32 i = blk * 8 + s;
        uint4 v = vis[i], a = aux[i];
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
    MTE_DEV void store(u32 blk, u32 s, const Seg& g) const {
        if (blk >= blk_cap || s >= 8) return;
        u32 i = blk * 8 + s;
        vis[i] = make_uint4(g.len, (u32)g.seq, (u32)g.rseq, g.meta);
        aux[i] = make_uint4(g.props, g.toff, g.tcap, g.sid);
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
        if (b >= blk_cap) return NONE;
        u32 x = bmeta[b] & BM_PAR;
        return x == BM_NOPAR ? NONE : x;
    }
    MTE_DEV u32 bscour(u32 b) const { return b < blk_cap ? bmeta[b] >> 30 : SC_UNDEF; }
    MTE_DEV void set_bpar_lane(u32 b, u32 par) const {  // per-lane write
        if (b < blk_cap) bmeta[b] = (bmeta[b] & ~BM_PAR) | (par == NONE ? BM_NOPAR : (par & BM_PAR));
    }
    MTE_DEV void set_bscour(u32 b, u32 sc) const {
        if (L == 0 && b < blk_cap) bmeta[b] = (bmeta[b] & BM_PAR) | (sc << 30);
    }

    // Visible length of slot idx for (refSeq R, client C): nodeLength for a leaf
    // (mergeTree.ts:1659-1699). C == 0 is the observer / local client: localNetLength (:1161-1172).
    MTE_DEV u32 vislen(uint4 v, u32 idx, i32 R, u32 C) const {
        const u32 meta = v.w;
        const bool removed = (meta & F_REMOVED) != 0;
        if (C == 0) return removed ? 0u : v.x;
        if (!(client_of(meta) == C || (i32)v.y <= R)) return 0u;
        if (removed) {
            if (rclient_of(meta) == C || (i32)v.z <= R) return 0u;
            if (meta & F_OVL) {
                u32 sid = aux[idx].w;
                if (sid < cfg.seg_cap && ((ovl[sid] >> C) & 1ull)) return 0u;
            }
        }
        return v.x;
    }
    // breakTie for a zero-visible leaf at pos 0: skip tombstones already seen at R (mergeTree.ts:2257-2261)
    MTE_DEV static bool tie_ok(uint4 v, i32 R) {
        return !((v.w & F_REMOVED) && (i32)v.z != 0 && (i32)v.z <= R);
    }
    // Visible length of a whole leaf block (one ord entry) for (R, C).
    MTE_DEV u32 blen(uint4 o, i32 R, u32 C) const {
        if (C == 0 || (i32)o.z <= R) return o.y;  // every child settled at R: same for all clients
        u32 v = 0;
        const u32 n = o.w > 8 ? 8u : o.w;
        for (u32 s = 0; s < n; s++) v += vislen(vis[o.x * 8 + s], o.x * 8 + s, R, C);
        return v;
    }

    // Recompute (visible length, max seq) of ord[k0 .. k0+n), n <= 8, from the slots.
    MTE_DEV void refresh(u32 k0, u32 n) {
        const u32 g = L >> 3, s = L & 7;
        const bool act = g < n;
        uint4 o = act ? ord[k0 + g] : make_uint4(0, 0, 0, 0);
        u32 len = 0;
        i32 mx = 0;
        if (act && s < o.w && o.x < blk_cap) {
            uint4 v = vis[o.x * 8 + s];
            len = obs_len(v.x, v.w);
            mx = seq_hi((i32)v.y, (i32)v.z, v.w);
        }
        u32 tl = group8_scan(len);
        i32 tm = group8_max(mx);
        sync();
        if (act && s == 7) {
            ord[k0 + g].y = tl;
            ord[k0 + g].z = (u32)tm;
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
        for (u32 base = 0; base < st.n_lb; base += 64) {
            const u32 k = base + L;
            const bool valid = k < st.n_lb;
            uint4 o = valid ? ord[k] : make_uint4(0, 0, 0, 0);
            u32 v = valid ? blen(o, R, C) : 0u;
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
        // inside the block: first slot with r < vislen, or a zero-visible slot at r == 0 that wins breakTie
        const u32 s = L;
        uint4 q = make_uint4(0, 0, 0, 0);
        u32 v = 0;
        bool tie = false;
        if (s < f.cnt && s < 8) {
            q = vis[f.blk * 8 + s];
            v = vislen(q, f.blk * 8 + s, R, C);
            tie = (C == 0) ? true : tie_ok(q, R);
        }
        u32 incl = group8_scan(v);
        i32 r = pos - (f.cum + (i32)(incl - v));
        bool cand = (s < f.cnt) && (s < 8) && (r < (i32)v || (r == 0 && v == 0 && tie));
        u64 m2 = wave_ballot(cand);
        if (m2) {
            u32 l2 = (u32)__builtin_ctzll(m2);
            f.slot = (i32)l2;
            f.r = wave_read(r, l2);
        }
        return f;
    }

    MTE_DEV i32 get_length(i32 R, u32 C) {  // MergeTree.getLength (mergeTree.ts:1577-1579)
        fence_ovl();
        i32 cum = 0;
        for (u32 base = 0; base < st.n_lb; base += 64) {
            const u32 k = base + L;
            u32 v = 0;
            if (k < st.n_lb) v = blen(ord[k], R, C);
            cum += (i32)wave_sum(v);
        }
        return cum;
    }

    // ---------------------------------------------------------------- allocation
    // Out of room: in LDS mode the document leaves the LDS plan (DOC_SPILL: its LDS state is
    // dropped and the host re-runs it HBM-resident); in HBM mode it is a capacity failure.
    MTE_DEV void fail_cap() {
        if (LDSM) fail(DOC_SPILL, st.curSeq);
        else fail(MTE_DOC_CAPACITY, st.curSeq);
    }

    MTE_DEV u32 alloc_lb() {
        MTE_PROF(PF_ALLOC);
        u32 id = NONE;
        if (LDSM) {
            // claim a free bit of the CU's pool bitmap (other waves claim concurrently)
            for (int guard = 0; guard < 64; guard++) {
                u32 w = L < 16 ? bitmap[L] : 0xFFFFFFFFu;
                u64 m = wave_ballot(w != 0xFFFFFFFFu);
                if (!m) break;
                u32 wl = (u32)__builtin_ctzll(m);
                u32 word = wave_read(w, wl);
                u32 bit = (u32)__builtin_ctz(~word);
                u32 old = 0;
                if (L == 0) old = atomicOr(&bitmap[wl], 1u << bit);
                old = wave_read(old, 0);
                if (!(old & (1u << bit))) {
                    id = wl * 32 + bit;
                    break;
                }
            }
            if (id == NONE || id >= blk_cap) {
                fail_cap();
                return NONE;
            }
            if (L == 0) owner[id] = (unsigned char)wave;
        } else {
            if (st.lbFree != NONE) {
                id = st.lbFree;
                u32 nx = bmeta[id] & BM_PAR;
                st.lbFree = nx == BM_NOPAR ? NONE : nx;
            } else if (st.lbBump < blk_cap) {
                id = st.lbBump++;
            } else {
                fail_cap();
                return NONE;
            }
        }
        sync();
        if (L == 0) bmeta[id] = BM_NOPAR | (SC_UNDEF << 30);
        sync();
        return id;
    }
    MTE_DEV void free_lb(u32 id) {
        if (id >= blk_cap) return;
        if (LDSM) {
            if (L == 0) {
                owner[id] = 0xFF;
                atomicAnd(&bitmap[id >> 5], ~(1u << (id & 31)));
            }
        } else {
            if (L == 0) bmeta[id] = st.lbFree == NONE ? BM_NOPAR : st.lbFree;
            st.lbFree = id;
        }
        sync();
    }
    MTE_DEV u32 alloc_in() {
        u32 id = NONE;
        if (st.inFree != NONE) {
            id = st.inFree;
            st.inFree = in_par[id];
        } else if (st.inBump < in_cap) {
            id = st.inBump++;
        } else {
            fail_cap();
            return NONE;
        }
        st.inUsed++;
        sync();
        if (L == 0) {
            in_cnt[id] = 0;
            in_par[id] = NONE;
        }
        sync();
        return id;
    }
    MTE_DEV void free_in(u32 id) {
        if (id >= in_cap) return;
        if (L == 0) in_par[id] = st.inFree;
        st.inFree = id;
        st.inUsed--;
        sync();
    }
    MTE_DEV u32 new_sid() {
        if (st.segNext >= cfg.seg_cap) {
            fail(MTE_DOC_CAPACITY, st.curSeq);
            return NONE;
        }
        return st.segNext++;
    }

    // ---------------------------------------------------------------- doc-order block list
    MTE_DEV void ord_shift_right(u32 from, u32 d) {  // ord[from..n_lb) -> ord[from+d..)
        for (i32 end = (i32)st.n_lb; end > (i32)from; end -= 64) {
            i32 start = end - 64 < (i32)from ? (i32)from : end - 64;
            i32 idx = start + (i32)L;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (idx < end) v = ord[idx];
            sync();
            if (idx < end) ord[idx + d] = v;
            sync();
        }
    }
    MTE_DEV void ord_shift_left(u32 from, u32 d) {  // ord[from..n_lb) -> ord[from-d..)
        for (u32 start = from; start < st.n_lb; start += 64) {
            u32 idx = start + L;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (idx < st.n_lb) v = ord[idx];
            sync();
            if (idx < st.n_lb) ord[idx - d] = v;
            sync();
        }
    }
    MTE_DEV u32 ord_find(u32 blk) const {
        for (u32 base = 0; base < st.n_lb; base += 64) {
            u32 idx = base + L;
            u64 m = wave_ballot(idx < st.n_lb && ord[idx].x == blk);
            if (m) return base + (u32)__builtin_ctzll(m);
        }
        return NONE;
    }
    // Current leaf block of segment `sid` (the LRU heap entry's segment.parent), NONE if unlinked.
    MTE_DEV bool find_seg(u32 sid, u32& k, u32& blk, u32& cnt) {
        MTE_PROF(PF_FIND_SEG);
        for (u32 base = 0; base < st.n_lb; base += 8) {
            const u32 kk = base + (L >> 3), s = L & 7;
            uint4 o = kk < st.n_lb ? ord[kk] : make_uint4(NONE, 0, 0, 0);
            bool hit = kk < st.n_lb && s < o.w && o.x < blk_cap && aux[o.x * 8 + s].w == sid;
            u64 m = wave_ballot(hit);
            if (m) {
                u32 l = (u32)__builtin_ctzll(m);
                k = base + (l >> 3);
                blk = wave_read(o.x, l);
                cnt = wave_read(o.w, l);
                return true;
            }
        }
        return false;
    }

    // ---------------------------------------------------------------- tree structure
    MTE_DEV u32 parent_of(u32 node, u32 lvl) const { return lvl == 0 ? bpar(node) : (node < in_cap ? in_par[node] : NONE); }
    MTE_DEV void set_parent(u32 node, u32 lvl, u32 par) const {
        if (L == 0) {
            if (lvl == 0) set_bpar_lane(node, par);
            else if (node < in_cap) in_par[node] = par;
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
            if (par != NONE && par >= in_cap) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            if (par == NONE) {  // child is the root: updateRoot
                u32 r = alloc_in();
                if (r == NONE) return;
                if (L == 0) {
                    in_child[r * 8 + 0] = child;
                    in_child[r * 8 + 1] = nn;
                    in_cnt[r] = 2;
                    in_par[r] = NONE;
                }
                set_parent(child, lvl_child, r);
                set_parent(nn, lvl_child, r);
                sync();
                st.root = r;
                st.height++;
                return;
            }
            u32 cnt = in_cnt[par];
            if (cnt > 8) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            u32 c = (L < cnt) ? in_child[par * 8 + L] : NONE;
            u64 m = wave_ballot(L < cnt && c == child);
            if (!m) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            u32 idx = (u32)__builtin_ctzll(m);
            sync();
            if (L > idx && L < cnt && L + 1 < 8) in_child[par * 8 + L + 1] = c;
            if (L == 0) {
                in_child[par * 8 + idx + 1] = nn;
                in_cnt[par] = cnt + 1;
            }
            set_parent(nn, lvl_child, par);
            sync();
            if (cnt + 1 < 8) return;
            // split interior node `par` (mergeTree.ts:2476-2489)
            u32 q = alloc_in();
            if (q == NONE) return;
            u32 moved = NONE;
            if (L < 4) moved = in_child[par * 8 + 4 + L];
            sync();
            if (L < 4) {
                in_child[q * 8 + L] = moved;
                if (lvl_child == 0) set_bpar_lane(moved, q);
                else if (moved < in_cap) in_par[moved] = q;
            }
            if (L == 0) {
                in_cnt[par] = 4;
                in_cnt[q] = 4;
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
        sync();
        if (mv) store(blk, L + 1, t);
        if (L == 0) store(blk, j, rec);
        const u32 nc = cnt + 1;
        if (nc < 8) {
            if (L == 0) {
                uint4 o = ord[k];
                o.w = nc;
                if (fresh) {
                    o.y += obs_len(rec.len, rec.meta);
                    i32 hi = seq_hi(rec.seq, rec.rseq, rec.meta);
                    if (hi > (i32)o.z) o.z = (u32)hi;
                }
                ord[k] = o;
            }
            sync();
            return blk;
        }
        if (st.n_lb + 1 > ord_cap) {
            fail_cap();
            return NONE;
        }
        u32 nb = alloc_lb();
        if (nb == NONE) return NONE;
        Seg m;
        if (L < 4) m = load(blk, 4 + L);
        sync();
        if (L < 4) store(nb, L, m);
        ord_shift_right(k + 1, 1);
        if (L == 0) {
            ord[k].w = 4;
            ord[k + 1] = make_uint4(nb, 0, 0, 4);
        }
        st.n_lb++;
        if (st.n_lb > st.max_lb) st.max_lb = st.n_lb;
        sync();
        refresh(k, 2);
        insert_after(blk, nb, 0);
        return j < 4 ? blk : nb;
    }

    // ---------------------------------------------------------------- LRU heap (collections.ts:213-265)
    MTE_DEV void heap_push(u32 sid, i32 maxSeq) {
        MTE_PROF(PF_HEAP);
        if (st.heapSize + 1 >= heap_cap) {
            fail_cap();
            return;
        }
        st.heapSize++;
        if (L == 0) {
            u32 k = st.heapSize;
            uint2 b = make_uint2(sid, (u32)maxSeq);
            while (k > 1) {  // sift up: parents with a strictly larger key move down
                uint2 a = heap[k >> 1];
                if (!((i32)a.y - (i32)b.y > 0)) break;
                heap[k] = a;
                k >>= 1;
            }
            heap[k] = b;
        }
        sync();
    }
    MTE_DEV uint2 heap_pop() {
        MTE_PROF(PF_HEAP);
        uint2 x = make_uint2(0, 0);
        if (L == 0) {
            x = heap[1];
            u32 n = st.heapSize;
            uint2 last = heap[n];
            n--;
            u32 k = 1;
            while ((k << 1) <= n) {  // sift down: the smaller child (left on ties) moves up
                u32 j = k << 1;
                uint2 hj = heap[j];
                if (j < n) {
                    uint2 hj1 = heap[j + 1];
                    if ((i32)hj.y - (i32)hj1.y > 0) {
                        j++;
                        hj = hj1;
                    }
                }
                if ((i32)last.y - (i32)hj.y <= 0) break;
                heap[k] = hj;
                k = j;
            }
            if (n >= 1) heap[k] = last;
        }
        x.x = wave_read(x.x, 0);
        x.y = wave_read(x.y, 0);
        st.heapSize--;
        sync();
        return x;
    }
    // addToLRUSet (mergeTree.ts:1273-1283) for a segment whose parent is `blk`.
    MTE_DEV void add_lru(u32 blk, u32 sid, i32 seq) {
        MTE_PROF(PF_LRU);
        if (!collab || blk == NONE) return;
        u32 sc = bscour(blk);
        if (sc != SC_TRUE && seq > st.curSeq) {
            sync();
            set_bscour(blk, SC_TRUE);
            sync();
            heap_push(sid, seq);
        }
    }

    // ---------------------------------------------------------------- property maps (HBM, lane 0)
    MTE_DEV bool val_match(u32 a, u32 b) const {  // matchProperties on one key (properties.ts:72-80)
        if (a == b) return true;
        if (p.val_flags[b] & 2u) {
            u32 j = p.val_objidx[b];
            return j != NONE && ((p.val_objmatch[a] >> j) & 1ull);
        }
        return false;
    }
    MTE_DEV bool match_props(u32 a, u32 b) const {  // properties.ts:62-93
        if (a == b) return true;
        if (a == 0 || b == 0) return false;
        if (a >= cfg.map_cap || b >= cfg.map_cap) return false;
        const u32* ma = maps + (u64)a * MAP_WORDS;
        const u32* mb = maps + (u64)b * MAP_WORDS;
        u32 na = ma[0], nb = mb[0];
        if (na != nb) return false;
        for (u32 i = 0; i < na; i++) {
            u32 k = ma[1 + 2 * i], v = ma[2 + 2 * i];
            bool found = false;
            for (u32 q = 0; q < nb; q++) {
                if (mb[1 + 2 * q] == k) {
                    if (!val_match(v, mb[2 + 2 * q])) return false;
                    found = true;
                    break;
                }
            }
            if (!found) return false;
        }
        return true;
    }
    // SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111) on an immutable map:
    // returns a fresh map id. Executed by lane 0; result broadcast.
    MTE_DEV u32 build_map(u32 old, u32 propset, bool rewrite) {
        MTE_PROF(PF_MAP);
        u32 id = NONE;
        i32 err = 0;
        if (st.mapNext >= cfg.map_cap) err = MTE_DOC_CAPACITY;
        if (L == 0 && !err) {
            u32 kv[2 * MTE_MAX_PROPS];
            u32 n = 0;
            if (old && old < cfg.map_cap) {
                const u32* mo = maps + (u64)old * MAP_WORDS;
                n = mo[0] > MTE_MAX_PROPS ? MTE_MAX_PROPS : mo[0];
                for (u32 i = 0; i < 2 * n; i++) kv[i] = mo[1 + i];
            }
            const mte_propset ps = p.propsets[propset];
            if (rewrite) {  // delete keys whose new value is falsy / absent (:65-78)
                u32 w = 0;
                for (u32 i = 0; i < n; i++) {
                    u32 k = kv[2 * i];
                    bool keep = false;
                    for (u32 q = 0; q < ps.count; q++)
                        if (p.prop_keys[ps.first + q] == k) keep = !(p.val_flags[p.prop_vals[ps.first + q]] & 1u);
                    if (keep) {
                        kv[2 * w] = k;
                        kv[2 * w + 1] = kv[2 * i + 1];
                        w++;
                    }
                }
                n = w;
            }
            for (u32 q = 0; q < ps.count && !err; q++) {
                u32 k = p.prop_keys[ps.first + q], v = p.prop_vals[ps.first + q];
                u32 at = NONE;
                for (u32 i = 0; i < n; i++)
                    if (kv[2 * i] == k) at = i;
                if (v == 0) {  // null deletes (:98-100)
                    if (at != NONE) {
                        for (u32 i = at; i + 1 < n; i++) {
                            kv[2 * i] = kv[2 * i + 2];
                            kv[2 * i + 1] = kv[2 * i + 3];
                        }
                        n--;
                    }
                } else if (at != NONE) {
                    kv[2 * at + 1] = v;
                } else if (n < MTE_MAX_PROPS) {
                    kv[2 * n] = k;
                    kv[2 * n + 1] = v;
                    n++;
                } else {
                    err = MTE_DOC_UNSUPPORTED;
                }
            }
            if (!err) {
                id = st.mapNext;
                u32* m = maps + (u64)id * MAP_WORDS;
                m[0] = n;
                for (u32 i = 0; i < 2 * n; i++) m[1 + i] = kv[i];
            }
        }
        err = wave_read(err, 0);
        id = wave_read(id, 0);
        if (err) {
            fail(err, st.curSeq);
            return 0;
        }
        st.mapNext++;
        return id;
    }

    // ---------------------------------------------------------------- text arena (HBM)
    MTE_DEV u16* text_ptr(u32 off) const {
        return (off & ARENA_BIT) ? arena0 + (u64)st.arenaSel * cfg.arena_cap + (off & ~ARENA_BIT) : payload + off;
    }
    MTE_DEV bool text_ok(u32 off, u32 n) const {
        u64 end = (u64)(off & ~ARENA_BIT) + n;
        return (off & ARENA_BIT) ? end <= cfg.arena_cap : end <= cfg.payload_len;
    }
    // TextSegment.canAppend's `!text.endsWith("\n")` (textSegment.ts:63-69): only documents whose
    // payload holds a newline read text here.
    MTE_DEV bool ends_nl(u32 off, u32 n) const {
        if (!has_nl || n == 0 || !text_ok(off, n)) return false;
        return text_ptr(off)[n - 1] == (u16)u'\n';
    }
    MTE_DEV void copy_text(u32 dst_off, u32 src_off, u32 n) {
        MTE_PROF(PF_TEXT);
        if (!text_ok(dst_off, n) || !text_ok(src_off, n)) {
            fail(MTE_DOC_CAPACITY, st.curSeq);
            return;
        }
        u16* d = text_ptr(dst_off);
        const u16* s = text_ptr(src_off);
        for (u32 i = L; i < n; i += 64) d[i] = s[i];
        st.adirty = 1;
    }
    // Semispace compaction of the merge arena (all live arena-resident segment texts).
    MTE_DEV void arena_gc() {
        fence_arena();
        const u32 other = st.arenaSel ^ 1u;
        u16* dst = arena0 + (u64)other * cfg.arena_cap;
        u32 top = 0;
        for (u32 k = 0; k < st.n_lb; k++) {
            uint4 o = ord[k];
            const u32 cnt = o.w > 8 ? 8u : o.w;
            for (u32 s = 0; s < cnt; s++) {
                uint4 v = vis[o.x * 8 + s];
                uint4 a = aux[o.x * 8 + s];
                if ((v.w & F_MARKER) || !(a.y & ARENA_BIT)) continue;
                const u32 len = v.x;
                const u32 cap = a.z < len ? len : a.z;
                if (!text_ok(a.y, len) || top + cap > cfg.arena_cap) {
                    fail(MTE_DOC_CAPACITY, st.curSeq);
                    return;
                }
                const u16* src = text_ptr(a.y);
                for (u32 i = L; i < len; i += 64) dst[top + i] = src[i];
                sync();
                if (L == 0) aux[o.x * 8 + s] = make_uint4(a.x, top | ARENA_BIT, cap, a.w);
                sync();
                top += cap;
            }
        }
        wave_sync();
        st.arenaSel = other;
        st.arenaTop = top;
        st.nGc++;
    }
    MTE_DEV bool arena_reserve(u32 need) {
        if (st.arenaTop + need <= cfg.arena_cap) return true;
        arena_gc();
        if (st.arenaTop + need <= cfg.arena_cap) return true;
        fail(MTE_DOC_CAPACITY, st.curSeq);
        return false;
    }

    // ---------------------------------------------------------------- zamboni (mergeTree.ts:1289-1478)
    // One scourNode decision pass over the slots of a leaf block (held one per lane in `me`).
    // dry == true: no side effects, returns the arena units the real pass will allocate.
    // dry == false: performs merges (text appends) and records the kept list in scratch.
    MTE_DEV u32 scour_pass(bool dry, const Seg& me, u32 cnt, u32& nkeep) {
        u32* sc_keep = scratch;
        u32* sc_len = scratch + 8;
        u32* sc_off = scratch + 16;
        u32* sc_cap = scratch + 24;
        u32 need = 0;
        nkeep = 0;
        i32 prev = -1;  // index into the kept list of the current merge target
        u32 pLen = 0, pOff = 0, pCap = 0, pProps = 0;
        bool pText = false, pNL = false;
        for (u32 s = 0; s < cnt; s++) {
            const u32 len = wave_read(me.len, s);
            const i32 seq = wave_read(me.seq, s);
            const i32 rseq = wave_read(me.rseq, s);
            const u32 meta = wave_read(me.meta, s);
            const u32 props = wave_read(me.props, s);
            const u32 toff = wave_read(me.toff, s);
            const u32 tcap = wave_read(me.tcap, s);
            const bool marker = (meta & F_MARKER) != 0;
            bool keep = false;
            if (meta & F_REMOVED) {  // tombstone: dropped once removed at or below the MSN (:1296-1319)
                if (rseq > st.minSeq) keep = true;
                prev = -1;
            } else if (seq <= st.minSeq) {
                bool ok = prev >= 0 && pText && !pNL && !marker &&
                          (pLen <= (u32)GRANULARITY || len <= (u32)GRANULARITY) && match_props(pProps, props);
                if (ok) {  // TextSegment.append (textSegment.ts:74-85)
                    if ((pOff & ARENA_BIT) && pLen + len <= pCap) {
                        if (!dry) copy_text(pOff + pLen, toff, len);
                    } else if (pOff + pLen == toff) {
                        if (pOff & ARENA_BIT) pCap = toff + tcap - pOff;
                    } else {
                        u32 ncap = 2 * (pLen + len);
                        if (ncap < 32) ncap = 32;
                        need += ncap;
                        const u32 dst = st.arenaTop | ARENA_BIT;
                        if (!dry) {
                            st.arenaTop += ncap;
                            copy_text(dst, pOff, pLen);
                            copy_text(dst + pLen, toff, len);
                        }
                        pOff = dst;
                        pCap = ncap;
                    }
                    pLen += len;
                    pNL = ends_nl(toff, len);
                    if (!dry && L == 0) {
                        sc_len[prev] = pLen;
                        sc_off[prev] = pOff;
                        sc_cap[prev] = pCap;
                    }
                } else {
                    keep = true;
                    prev = (i32)nkeep;
                    pLen = len;
                    pOff = toff;
                    pCap = tcap;
                    pProps = props;
                    pText = !marker;
                    pNL = !marker && ends_nl(toff, len);
                }
            } else {
                keep = true;
                prev = -1;
            }
            if (keep) {
                if (!dry && L == 0) {
                    sc_keep[nkeep] = s;
                    sc_len[nkeep] = len;
                    sc_off[nkeep] = toff;
                    sc_cap[nkeep] = tcap;
                }
                nkeep++;
            }
        }
        return need;
    }

    // scourNode on leaf block `blk` (doc-order index k, child count cnt), compacting the kept
    // slots in place; returns the new child count. A dry decision pass first (no side effects,
    // sizes the arena need), then the real pass: ONE call site of scour_pass.
    MTE_DEV u32 scour(u32 k, u32 blk, u32 cnt) {
        MTE_PROF(PF_SCOUR);
        if (cnt > 8) cnt = 8;
        Seg me;
        if (L < cnt) me = load(blk, L);
        fence_arena();
        u32 nkeep = 0;
        for (u32 pass = 0; pass < 2; pass++) {
            const bool dry = pass == 0;
            const u32 need = scour_pass(dry, me, cnt, nkeep);
            if (st.status) return cnt;
            if (dry) {
                if (nkeep == cnt) return cnt;  // nothing dropped or merged => nothing changes
                if (need) {
                    if (!arena_reserve(need)) return cnt;
                    if (L < cnt) me = load(blk, L);  // a GC may have moved arena texts
                }
            }
        }
        sync();
        const u32 src = L < nkeep ? scratch[L] : 0u;
        Seg out = shfl_seg(me, src);
        if (L < nkeep) {
            out.len = scratch[8 + L];
            out.toff = scratch[16 + L];
            out.tcap = scratch[24 + L];
        }
        sync();
        if (L < nkeep) store(blk, L, out);
        const u32 ol = L < nkeep ? obs_len(out.len, out.meta) : 0u;
        const i32 om = L < nkeep ? seq_hi(out.seq, out.rseq, out.meta) : 0;
        const u32 tl = wave_read(group8_scan(ol), 7);
        const i32 tm = wave_read(group8_max(om), 7);
        if (L == 0) ord[k] = make_uint4(blk, tl, (u32)tm, nkeep);
        sync();
        return nkeep;
    }

    // pack (mergeTree.ts:1368-1420), second half: the m children of `par` (doc-order run k0..k0+m,
    // already re-scoured; lane i < m holds child i's id in `kids` and its count in `cnts`) are
    // redistributed into max(1, min(7, T/4)) fresh blocks.
    MTE_DEV void pack_leaves(u32 par, u32 m, u32 kids, u32 k0, u32 cnts) {
        MTE_PROF(PF_PACK);
        const u32 T = wave_sum(L < m ? cnts : 0u);
        u32 kk = T / 4;
        if (kk > 7) kk = 7;
        if (kk < 1) kk = 1;
        const u32 base = T / kk, extra = T % kk;
        if (st.n_lb + kk > ord_cap + m) {
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
        for (u32 i = 0; i < m; i++) free_lb(wave_read(kids, i));
        u32 nb = NONE;
        for (u32 j = 0; j < kk; j++) {
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
        if (L < T) store(dstBlk, dq, rec);
        if (L < kk) {
            bmeta[nb] = (par & BM_PAR) | (SC_UNDEF << 30);
            in_child[par * 8 + L] = nb;
        }
        if (L == 0) in_cnt[par] = kk;
        sync();
        // splice ord: the run of the parent's old children becomes the kk new blocks
        if (kk > m) {
            ord_shift_right(k0 + m, kk - m);
            st.n_lb += kk - m;
            if (st.n_lb > st.max_lb) st.max_lb = st.n_lb;
        } else if (kk < m) {
            ord_shift_left(k0 + m, m - kk);
            st.n_lb -= m - kk;
        }
        if (L < kk) ord[k0 + L] = make_uint4(nb, 0, 0, base + (L < extra ? 1u : 0u));
        sync();
        refresh(k0, kk);
        if (kk < 4 && par < in_cap && in_par[par] != NONE) pack_internal(par, 1);
    }

    // pack on an interior level: `node` (level lvl) underflowed; redistribute the grandchildren of
    // its parent over max(1, min(7, T/4)) fresh interior nodes.
    MTE_DEV void pack_internal(u32 node, u32 lvl) {
        for (u32 guard = 0;; guard++) {
            if (guard > 32) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            const u32 par = in_par[node];
            if (par >= in_cap || in_cnt[par] > 8) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                return;
            }
            const u32 m = in_cnt[par];
            const u32 kids = L < m ? in_child[par * 8 + L] : NONE;
            const u32 cnts = (L < m && kids < in_cap) ? in_cnt[kids] : 0u;
            if (wave_ballot(L < m && (kids >= in_cap || cnts > 8))) {
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
            if (L < T) gc = in_child[srcN * 8 + q];
            sync();
            for (u32 i = 0; i < m; i++) free_in(wave_read(kids, i));
            u32 nb = NONE;
            for (u32 j = 0; j < kk; j++) {
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
                in_child[dstN * 8 + dq] = gc;
                if (lvl == 1) set_bpar_lane(gc, dstN);
                else if (gc < in_cap) in_par[gc] = dstN;
            }
            if (L < kk) {
                in_cnt[nb] = base + (L < extra ? 1u : 0u);
                in_par[nb] = par;
                in_child[par * 8 + L] = nb;
            }
            if (L == 0) in_cnt[par] = kk;
            sync();
            if (kk < 4 && in_par[par] != NONE) {
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
            if (st.heapSize == 0) break;
            const i32 top = (i32)heap[1].y;
            if (top > st.minSeq) break;
            uint2 e = heap_pop();
            u32 k, blk, cnt;
            if (!find_seg(e.x, k, blk, cnt)) continue;  // segment no longer linked
            if (bscour(blk) == SC_FALSE) continue;
            bool packing = false;
            u32 par = NONE, m = 0, kids = NONE, k0 = 0, cnts = 0, idx = 0;
            for (;;) {
                const u32 nc = scour(k, blk, cnt);
                if (st.status) return;
                if (!packing) {
                    set_bscour(blk, SC_FALSE);
                    sync();
                    if (!(nc < cnt && nc < 4 && st.height > 1)) break;
                    par = bpar(blk);
                    if (par == NONE || par >= in_cap || in_cnt[par] > 8 || in_cnt[par] == 0) {
                        fail(MTE_DOC_CAPACITY, st.curSeq);
                        return;
                    }
                    m = in_cnt[par];
                    kids = L < m ? in_child[par * 8 + L] : NONE;
                    k0 = ord_find(wave_read(kids, 0));
                    if (k0 == NONE || k0 + m > st.n_lb ||
                        wave_ballot(L < m && ord[k0 + (L < m ? L : 0)].x != kids)) {
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
                const uint4 o = ord[k0 + idx];
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
    MTE_DEV bool edit(u32 type, i32 p1, i32 p2, i32 R, u32 C, i32 seq, Seg rec, u32 propset, bool rewrite) {
        const bool ins = type == MTE_OP_INSERT || type == MTE_OP_INSERT_MARKER;
        const u32 nphase = ins ? 2u : 3u;
        for (u32 ph = 0; ph < nphase; ph++) {
            if (!ins && ph == 2) {
                range_op(type == MTE_OP_REMOVE, p1, p2, R, C, seq, propset, rewrite);
                return st.status == 0;
            }
            const bool place = ins && ph == 1;
            const Found f = resolve(ph == 1 && !ins ? p2 : p1, R, C);
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
                // ensureIntervalBoundary: split slot f.slot at f.r (BaseSegment.splitAt, :524-568)
                Seg left = load(f.blk, (u32)f.slot);
                const u32 sid = new_sid();
                if (sid == NONE) return false;
                task = left;
                const u32 r = (u32)f.r;
                task.len = left.len - r;
                task.toff = left.toff + r;
                task.tcap = (left.toff & ARENA_BIT) ? left.tcap - r : 0u;
                task.sid = sid;
                left.len = r;
                left.tcap = (left.toff & ARENA_BIT) ? r : 0u;
                if (left.meta & F_OVL) {  // the right piece copies removedClientOverlap
                    fence_ovl();
                    if (L == 0 && left.sid < cfg.seg_cap && sid < cfg.seg_cap) ovl[sid] = ovl[left.sid];
                    st.gdirty = 1;
                }
                sync();
                if (L == 0) store(f.blk, (u32)f.slot, left);
                sync();
                j = (u32)f.slot + 1;
            }
            const u32 b = insert_slot(f.k, f.blk, f.cnt, j, task, place);
            if (st.status) return false;
            if (place && collab && seq > st.minSeq) add_lru(b, rec.sid, seq);
        }
        return st.status == 0;
    }

    // markRangeRemoved / annotateRange mark pass (nodeMap, mergeTree.ts:2903-2965): positions are
    // those of the (R, C) view before the op; blocks overlapping [p1, p2) are processed in order.
    MTE_DEV void range_op(bool remove, i32 p1, i32 p2, i32 R, u32 C, i32 seq, u32 propset, bool rewrite) {
        MTE_PROF(PF_RANGE);
        fence_ovl();
        i32 cum = 0;
        u32 memoOld = NONE, memoNew = 0;
        for (u32 base = 0; base < st.n_lb && cum < p2; base += 64) {
            const u32 k = base + L;
            const bool valid = k < st.n_lb;
            uint4 o = valid ? ord[k] : make_uint4(0, 0, 0, 0);
            const u32 v = valid ? blen(o, R, C) : 0u;
            const u32 incl = wave_scan_incl(v);
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
                const u32 idx = blk * 8 + (s & 7);
                uint4 q = make_uint4(0, 0, 0, 0);
                u32 sv = 0;
                if (s < cnt && s < 8) {
                    q = vis[idx];
                    sv = vislen(q, idx, R, C);
                }
                const u32 si = group8_scan(sv);
                const i32 ex = cbj + (i32)(si - sv);
                const bool mark = s < cnt && s < 8 && sv > 0 && ex < p2 && ex + (i32)sv > p1;
                const u64 mm = wave_ballot(mark);
                if (!mm) continue;
                const u32 sid = mark ? aux[idx].w : NONE;
                if (remove) {
                    u32 fresh = 0;
                    if (mark) {
                        if (q.w & F_REMOVED) {  // addOverlappingClient (:2544-2552)
                            if (sid < cfg.seg_cap) {
                                u64 old = (q.w & F_OVL) ? ovl[sid] : 0ull;
                                ovl[sid] = old | (1ull << C);
                            }
                            q.w |= F_OVL;
                            vis[idx].w = q.w;
                        } else {
                            q.w = (q.w & ~0xff00u) | (C << 8) | F_REMOVED;
                            vis[idx] = make_uint4(q.x, q.y, (u32)seq, q.w);
                            fresh = q.x;
                        }
                    }
                    if (wave_ballot(mark && (q.w & F_OVL) && !fresh)) st.gdirty = 1;
                    const u32 gone = wave_read(group8_scan(fresh), 7);
                    if (L == 0) {
                        uint4 ob = ord[kj];
                        ob.y -= gone;
                        if (gone && seq > (i32)ob.z) ob.z = (u32)seq;
                        ord[kj] = ob;
                    }
                } else {
                    const u32 props = mark ? aux[idx].x : 0u;
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
                        if (same) aux[idx].x = nid;
                        pending &= ~wave_ballot(same);
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

    // Client.applyMsg for one op record (client.ts:805-836): the edit, zamboni, then
    // updateSeqNumbers / setMinSeq (client.ts:829-836, mergeTree.ts:1718-1736) and zamboni again
    // when the MSN advanced. One zamboni call site.
    MTE_DEV void apply(const mte_op& op) {
        MTE_PROF(PF_APPLY);
#ifdef MTE_PROFILE
        prof[PF_OPS]++;
#endif
        if (op.client >= MTE_MAX_CLIENTS) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        const u32 C = collab ? (u32)op.client : 0u;
        const i32 seq = collab ? op.seq : 0;
        const i32 R = collab ? op.ref_seq : 0;
        if (collab && op.type != MTE_OP_NOOP && !(st.curSeq < op.seq)) {
            fail(MTE_DOC_SEQ_ORDER, op.seq);
            return;
        }
        bool edited = false;
        if (op.type <= MTE_OP_INSERT_MARKER) {
            Seg rec;
            const bool mk = op.type == MTE_OP_INSERT_MARKER;
            const bool ins = op.type == MTE_OP_INSERT || mk;
            rec.len = mk ? 1u : op.b;
            rec.seq = seq;
            rec.rseq = 0;
            rec.meta = (C & 0xff) | (mk ? F_MARKER : 0u);
            rec.props = (ins && op.props) ? build_map(0, op.props, false) : 0u;
            if (st.status) return;
            rec.toff = mk ? op.b : (u32)op.a;
            rec.tcap = 0;
            rec.sid = 0;
            edited = edit(op.type, op.pos1, op.a, R, C, seq, rec, op.props, (op.flags & MTE_F_REWRITE) != 0);
            st.opsApplied++;
            if (st.status) return;
        }
        for (u32 z = 0; z < 2; z++) {
            bool run = edited;
            if (z == 1) {
                run = false;
                if (collab && (op.flags & MTE_F_END_OF_MSG)) {
                    st.msgs++;
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
            if (run) zamboni();
            if (st.status) return;
        }
    }

    // ---------------------------------------------------------------- driver
    MTE_DEV void init() {
        u32 r = alloc_lb();
        st.root = r;
        st.height = 1;
        if (r == NONE) return;
        if (L == 0) ord[0] = make_uint4(r, 0, 0, 0);
        st.n_lb = 1;
        st.max_lb = 1;
        sync();
    }

    // LDS mode: give every leaf block this wave holds back to the CU's pool (also after an
    // abandoned replay, whose blocks need not all be linked).
    MTE_DEV void release() {
        if (!LDSM) return;
        for (u32 base = 0; base < blk_cap; base += 64) {
            const u32 b = base + L;
            if (b < blk_cap && owner[b] == (unsigned char)wave) {
                owner[b] = 0xFF;
                atomicAnd(&bitmap[b >> 5], ~(1u << (b & 31)));
            }
        }
        st.n_lb = 0;
        sync();
    }

    // Results + the final segments in doc order (walkAllSegments, mergeTree.ts:2969-2983).
    MTE_DEV void finish() {
#ifdef MTE_PROFILE
        if (L == 0 && p.prof)
            for (u32 i = 0; i < PROF_SLOTS; i++) p.prof[(u64)doc * PROF_SLOTS + i] = prof[i];
#endif
        u32 nseg = 0;
        for (u32 base = 0; base < st.n_lb; base += 64) {
            u32 k = base + L;
            nseg += wave_sum(k < st.n_lb ? ord[k].w : 0u);
        }
        u32 off = 0;
        if (st.status == 0) {
            if (L == 0) off = atomicAdd(&p.counters[1], nseg);
            off = wave_read(off, 0);
            if ((u64)off + nseg > p.out_cap) {
                fail(MTE_DOC_CAPACITY, st.curSeq);
                nseg = 0;
            }
        } else {
            nseg = 0;
        }
        if (nseg) {
            fence_ovl();
            u32 run = off;
            for (u32 base = 0; base < st.n_lb; base += 64) {
                const u32 k = base + L;
                uint4 o = k < st.n_lb ? ord[k] : make_uint4(0, 0, 0, 0);
                const u32 c = o.w > 8 ? 8u : o.w;
                const u32 incl = wave_scan_incl(c);
                u32 at = run + incl - c;
                for (u32 s = 0; s < c; s++) {
                    uint4 v = vis[o.x * 8 + s], a = aux[o.x * 8 + s];
                    p.out_vis[at + s] = v;
                    p.out_aux[at + s] = a;
                    p.out_ovl[at + s] = ((v.w & F_OVL) && a.w < cfg.seg_cap) ? ovl[a.w] : 0ull;
                }
                run += wave_read(incl, 63);
            }
        }
        if (L == 0) {
            DocRes& o = p.res[doc];
            o.status = st.status;
            o.failing_seq = st.failingSeq;
            o.ops = st.opsApplied;
            o.msgs = st.msgs;
            o.min_seq = st.minSeq;
            o.cur_seq = st.curSeq;
            o.height = st.height;
            o.n_lb = st.n_lb;
            o.arena_sel = st.arenaSel;
            o.arena_top = st.arenaTop;
            o.map_next = st.mapNext;
            o.seg_next = st.segNext;
            o.heap_size = st.heapSize;
            o.n_gc = st.nGc;
            o.out_off = off;
            o.n_segs = nseg;
            o.max_lb = st.max_lb;
            o.mode = LDSM ? 0u : 1u;
        }
    }

    MTE_DEV void mark_spilled() {
        if (L == 0) {
            DocRes& o = p.res[doc];
            o.status = DOC_SPILL;
            o.failing_seq = st.curSeq;
            o.n_segs = 0;
            o.max_lb = st.max_lb;
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

    // Replay the doc's op log. Returns false if the LDS plan ran out of room (spill).
    MTE_DEV bool replay() {
#ifdef MTE_PROFILE
        ProfScope _total(prof[PF_TOTAL]);
#endif
        init();
        const u64 b = cfg.op_begin, e = cfg.op_end;
        if (LDSM) {
            // op records are staged RING_OPS at a time through LDS; the next batch is prefetched
            // into registers one batch ahead (lane l holds 16 B of record l/2 of the batch).
            const uint4* src = (const uint4*)(p.ops);
            uint4* dst = (uint4*)ring;
            uint4 nxt = make_uint4(0, 0, 0, 0);
            u64 g = b * 2 + L;
            if (b + (L >> 1) < e) nxt = src[g];
            for (u64 i = b; i < e && !st.status; i++) {
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
                    op = read_op(ring + r);
                }
                apply(op);
            }
        } else {
            for (u64 i = b; i < e && !st.status; i++) {
                mte_op op = p.ops[i];
                apply(op);
            }
        }
        return st.status != DOC_SPILL;
    }

    // Synthetic workload generator: simulated writers draw valid ops from their own
    // view (getLength(refSeq, client)); each op is recorded into the doc's op/payload slots and
    // applied immediately, so the recorded log is exactly what a replay will see.
    // Returns false if the LDS plan ran out of room (the host regenerates the doc HBM-resident;
    // the generator is deterministic per (doc, seed)).
    MTE_DEV bool generate() {
        init();
        Rng rng;
        u64 sx = 0xF1D0C0DEull ^ (u64)doc ^ (p.gen_seed * 0x9E3779B97F4A7C15ull);
        rng.seed(sx);
        const u32 nc = p.gen_nclients;
        i32 ref[MTE_MAX_CLIENTS];
        u32 sid_of[MTE_MAX_CLIENTS];
        for (u32 c = 0; c < nc; c++) {
            ref[c] = 0;
            sid_of[c] = 0;
        }
        u32 nextShort = 1;
        u32 pay = 0;
        i32 lastC = -1, lastR = 0, lastPos = 0;
        u32* firstSeen = p.gen_first_seen + (u64)doc * MTE_MAX_CLIENTS;
        const u64 nops = cfg.op_end - cfg.op_begin;
        for (u64 step = 0; step < nops && !st.status; step++) {
            const i32 seq = (i32)step + 1;
            const i32 cur = seq - 1;
            const u32 c = rng.below(nc);
            if (rng.below(4) == 0) ref[c] = cur;
            else {
                i32 nr = ref[c] + (i32)rng.below(5);
                ref[c] = nr < cur ? nr : cur;
            }
            if (p.gen_kind == 5 && ref[c] < cur - 64) ref[c] = cur - 64;
            bool forced = false;
            if (p.gen_kind == 3 && lastC >= 0 && (u32)lastC != c && rng.below(100) < 15 && lastR >= ref[c]) {
                ref[c] = lastR;  // replay a recent other-client op's refSeq and position
                forced = true;
            }
            if (sid_of[c] == 0) {
                sid_of[c] = nextShort++;
                if (L == 0) firstSeen[sid_of[c]] = c;
            }
            const u32 C = sid_of[c];
            const i32 R = ref[c];
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
                const i32 pos = forced ? (lastPos < len ? lastPos : len) : (i32)rng.below((u32)len + 1);
                const u32 n = 1 + rng.below(8);
                op.pos1 = pos;
                op.a = (i32)pay;
                op.b = n;
                for (u32 i = 0; i < n; i++) {
                    const u16 ch = (u16)(u'a' + rng.below(26));
                    if (L == 0) payload[pay + i] = ch;
                }
                pay += n;
                st.adirty = 1;  // later cross-lane text copies read these chars
                if (p.gen_kind == 3 && rng.below(4) == 0) op.props = 1 + rng.below(p.gen_n_propsets);
            } else {
                const i32 a = forced ? (lastPos < len ? lastPos : len - 1) : (i32)rng.below((u32)len);
                const i32 n = 1 + (i32)rng.below(16);
                op.pos1 = a;
                op.a = a + n < len ? a + n : len;
                if (type == MTE_OP_ANNOTATE) op.props = 1 + rng.below(p.gen_n_propsets);
            }
            i32 msn = ref[0];
            for (u32 q = 1; q < nc; q++) msn = ref[q] < msn ? ref[q] : msn;
            op.msn = msn;
            lastC = (i32)c;
            lastR = R;
            lastPos = op.pos1;
            if (L == 0) p.ops[cfg.op_begin + step] = op;
            apply(op);
        }
        wave_sync();  // op records and payload visible before the replay kernel
        return st.status != DOC_SPILL;
    }
};

}  // namespace mte
