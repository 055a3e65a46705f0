// engine_core.hpp — the per-document replay engine executed by ONE wavefront (64 lanes).
//
// Restates the observer replay path of @fluidframework/merge-tree 0.31.0 (paths below are relative
// to packages/dds/merge-tree/src) in an MI355X-first shape:
//   * the B-tree is kept exactly (8-slot blocks, 8->4+4 splits, root growth, zamboni scour/pack),
//     because segment boundaries and SnapshotV1 bytes depend on it;
//   * leaf blocks are 8-slot SoA records in HBM; a per-doc array `lbo` lists leaf blocks in document
//     order, so position resolution is a wavefront scan: lane = (block, slot), 8 blocks per step,
//     visibility predicate per lane (mergeTree.ts:1673-1696), DPP prefix sum, ballot to find the
//     first leaf block whose cumulative end >= pos (blocks win ties, mergeTree.ts:2274-2276) and the
//     first qualifying slot inside it (breakTie, mergeTree.ts:2248-2277);
//   * PartialSequenceLengths (partialLengths.ts) is not needed: the scan evaluates the predicate;
//   * serial pieces (heap, tree maintenance) run on lane 0 with results broadcast.
// Requires the wave primitives (lane_id, wave_sync, wave_ballot, wave_shfl, wave_read,
// wave_scan_incl, wave_sum, atomic_add_u32) and MTE_DEV from the including translation unit.
#pragma once
#include <stdint.h>

#include "engine_types.hpp"

namespace mte {

struct Found {
    bool ok;
    u32 k;      // lbo index of the leaf block
    u32 blk;    // leaf block id
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

struct Engine {
    const Params& p;
    const DocCfg& cfg;
    u32 doc;
    u32 L;  // lane
    // uniform replay state (identical in every lane)
    u32 root, height, n_lb;
    i32 minSeq, curSeq;
    u32 heapSize, segNext, arenaTop, arenaSel, mapNext, lbFree, inFree;
    i32 status, failingSeq;
    u32 opsApplied, msgs, nGc;
    bool collab;
    // doc-relative bases
    u16* payload;
    u16* arena0;
    u32* segParent;
    uint2* heap;
    u32* lbo;
    u32* maps;

    MTE_DEV Engine(const Params& p_, u32 doc_) : p(p_), cfg(p_.docs[doc_]), doc(doc_) {
        L = lane_id();
        payload = p.payload + cfg.payload_off;
        arena0 = p.arena + cfg.arena_off;
        segParent = p.seg_parent + cfg.seg_off;
        heap = p.heap + cfg.heap_off;
        lbo = p.lbo + cfg.lbo_off;
        maps = p.maps + cfg.map_off * MAP_WORDS;
        collab = cfg.collab != 0;
        height = 1;
        n_lb = 0;
        minSeq = curSeq = 0;
        heapSize = segNext = arenaTop = arenaSel = 0;
        mapNext = 1;  // map id 0 == undefined
        lbFree = inFree = NONE;
        status = 0;
        failingSeq = -1;
        opsApplied = msgs = nGc = 0;
    }

    // ---------------------------------------------------------------- errors
    MTE_DEV void fail(i32 code, i32 seq) {
        if (status == 0) {
            status = code;
            failingSeq = seq;
        }
    }

    // ---------------------------------------------------------------- slot access
    // Guards: a corrupted id never reaches memory; it becomes a per-doc status instead of a fault.
    MTE_DEV bool bad_blk(u32 blk) const { return blk >= p.nlb_cap; }
    MTE_DEV bool bad_in(u32 n) const { return n >= p.nin_cap; }
    MTE_DEV u32 lbcnt(u32 blk) const {
        if (blk == NONE || bad_blk(blk)) return 0u;
        u32 c = p.lb_cnt[blk];
        return c > 8 ? 0u : c;
    }
    MTE_DEV void set_seg_parent(u32 sid, u32 blk) const {
        if (sid < cfg.seg_cap) segParent[sid] = blk;
    }

    MTE_DEV SegRec load_slot(u32 blk, u32 s) const {
        SegRec r;
        if (bad_blk(blk) || s >= 8) {
            r.v = Slot{0, 0, 0, 0};
            r.ovl = 0;
            r.props = 0;
            r.toff = 0;
            r.tcap = 0;
            r.sid = 0;
            return r;
        }
        u32 i = blk * 8 + s;
        uint4 v = p.lb_vis[i];
        r.v.len = v.x;
        r.v.seq = (i32)v.y;
        r.v.rseq = (i32)v.z;
        r.v.meta = v.w;
        r.ovl = p.lb_ovl[i];
        r.props = p.lb_props[i];
        uint2 t = p.lb_txt[i];
        r.toff = t.x;
        r.tcap = t.y;
        r.sid = p.lb_sid[i];
        return r;
    }
    MTE_DEV void store_slot(u32 blk, u32 s, const SegRec& r) const {
        if (bad_blk(blk) || s >= 8) return;
        u32 i = blk * 8 + s;
        p.lb_vis[i] = make_uint4(r.v.len, (u32)r.v.seq, (u32)r.v.rseq, r.v.meta);
        p.lb_ovl[i] = r.ovl;
        p.lb_props[i] = r.props;
        p.lb_txt[i] = make_uint2(r.toff, r.tcap);
        p.lb_sid[i] = r.sid;
    }
    MTE_DEV SegRec shfl_rec(const SegRec& r, u32 src) const {
        SegRec o;
        o.v.len = wave_shfl(r.v.len, src);
        o.v.seq = wave_shfl(r.v.seq, src);
        o.v.rseq = wave_shfl(r.v.rseq, src);
        o.v.meta = wave_shfl(r.v.meta, src);
        o.ovl = wave_shfl(r.ovl, src);
        o.props = wave_shfl(r.props, src);
        o.toff = wave_shfl(r.toff, src);
        o.tcap = wave_shfl(r.tcap, src);
        o.sid = wave_shfl(r.sid, src);
        return o;
    }

    MTE_DEV static u32 client_of(u32 meta) { return meta & 0xff; }
    MTE_DEV static u32 rclient_of(u32 meta) { return (meta >> 8) & 0xff; }

    // Visible length of a slot for (refSeq R, client C): nodeLength for a leaf (mergeTree.ts:1659-1699).
    // C == 0 is the observer / local client: localNetLength (mergeTree.ts:1161-1172).
    MTE_DEV u32 vislen(const Slot& s, u32 idx, i32 R, u32 C) const {
        bool removed = (s.meta & F_REMOVED) != 0;
        if (C == 0) return removed ? 0u : s.len;
        if (!(client_of(s.meta) == C || s.seq <= R)) return 0u;
        if (removed) {
            if (rclient_of(s.meta) == C || s.rseq <= R) return 0u;
            if ((p.lb_ovl[idx] >> C) & 1ull) return 0u;
        }
        return s.len;
    }
    // breakTie for a zero-visible leaf at pos 0: skip tombstones already seen at R (mergeTree.ts:2257-2261)
    MTE_DEV static bool tie_ok(const Slot& s, i32 R) {
        return !((s.meta & F_REMOVED) && s.rseq != 0 && s.rseq <= R);
    }

    // ---------------------------------------------------------------- position resolution
    MTE_DEV Found resolve(i32 pos, i32 R, u32 C, u32 k0, i32 cum0) const {
        Found f;
        f.ok = false;
        f.k = 0;
        f.blk = NONE;
        f.slot = -1;
        f.r = 0;
        f.cum = 0;
        i32 cum = cum0;
        const u32 s = L & 7;
        for (u32 base = k0; base < n_lb; base += 8) {
            u32 bk = base + (L >> 3);
            u32 blk = bk < n_lb ? lbo[bk] : NONE;
            u32 cnt = lbcnt(blk);
            u32 v = 0;
            bool tie = false;
            if (s < cnt) {
                uint4 q = p.lb_vis[blk * 8 + s];
                Slot sl{q.x, (i32)q.y, (i32)q.z, q.w};
                v = vislen(sl, blk * 8 + s, R, C);
                tie = (C == 0) ? true : tie_ok(sl, R);
            }
            u32 incl = wave_scan_incl(v);
            i32 ex = cum + (i32)(incl - v);
            bool endLane = (s == 7) && (bk < n_lb) && (cum + (i32)incl >= pos);
            u64 m = wave_ballot(endLane);
            if (m) {
                u32 j = (u32)__builtin_ctzll(m) >> 3;
                u32 first = j * 8;
                i32 r = pos - ex;
                bool cand = ((L >> 3) == j) && (s < cnt) && (r < (i32)v || (r == 0 && v == 0 && tie));
                u64 m2 = wave_ballot(cand);
                f.ok = true;
                f.k = base + j;
                f.blk = wave_read(blk, first);
                f.cum = wave_read(ex, first);
                if (m2) {
                    u32 l2 = (u32)__builtin_ctzll(m2);
                    f.slot = (i32)(l2 - first);
                    f.r = wave_read(r, l2);
                }
                return f;
            }
            cum += (i32)wave_read(incl, 63);
        }
        return f;
    }

    MTE_DEV i32 get_length(i32 R, u32 C) const {  // MergeTree.getLength (mergeTree.ts:1577-1579)
        i32 cum = 0;
        const u32 s = L & 7;
        for (u32 base = 0; base < n_lb; base += 8) {
            u32 bk = base + (L >> 3);
            u32 blk = bk < n_lb ? lbo[bk] : NONE;
            u32 cnt = lbcnt(blk);
            u32 v = 0;
            if (s < cnt) {
                uint4 q = p.lb_vis[blk * 8 + s];
                Slot sl{q.x, (i32)q.y, (i32)q.z, q.w};
                v = vislen(sl, blk * 8 + s, R, C);
            }
            cum += (i32)wave_sum(v);
        }
        return cum;
    }

    // ---------------------------------------------------------------- allocation
    MTE_DEV u32 alloc_lb() {
        u32 id = NONE;
        if (L == 0) {
            if (lbFree != NONE) {
                id = lbFree;
            } else {
                id = atomic_add_u32(&p.counters[0], 1u);
                if (id >= p.nlb_cap) id = NONE;
            }
        }
        id = wave_read(id, 0);
        if (id == NONE) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return NONE;
        }
        if (id == lbFree) {
            u32 nx = p.lb_par[id];
            lbFree = nx;
        }
        wave_sync();
        if (L == 0) {
            p.lb_cnt[id] = 0;
            p.lb_par[id] = NONE;
            p.lb_scour[id] = SC_UNDEF;
        }
        wave_sync();
        return id;
    }
    MTE_DEV void free_lb(u32 id) {
        if (L == 0) p.lb_par[id] = lbFree;
        lbFree = id;
        wave_sync();
    }
    MTE_DEV u32 alloc_in() {
        u32 id = NONE;
        if (L == 0) {
            if (inFree != NONE) {
                id = inFree;
            } else {
                id = atomic_add_u32(&p.counters[1], 1u);
                if (id >= p.nin_cap) id = NONE;
            }
        }
        id = wave_read(id, 0);
        if (id == NONE) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return NONE;
        }
        if (id == inFree) inFree = p.in_par[id];
        wave_sync();
        if (L == 0) {
            p.in_cnt[id] = 0;
            p.in_par[id] = NONE;
        }
        wave_sync();
        return id;
    }
    MTE_DEV void free_in(u32 id) {
        if (L == 0) p.in_par[id] = inFree;
        inFree = id;
        wave_sync();
    }
    MTE_DEV u32 new_sid() {
        if (segNext >= cfg.seg_cap) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return NONE;
        }
        return segNext++;
    }

    // ---------------------------------------------------------------- lbo maintenance
    MTE_DEV void lbo_shift_right(u32 from, u32 d) {  // lbo[from..n_lb) -> lbo[from+d..)
        for (i32 end = (i32)n_lb; end > (i32)from; end -= 64) {
            i32 start = end - 64 < (i32)from ? (i32)from : end - 64;
            i32 idx = start + (i32)L;
            u32 v = 0;
            if (idx < end) v = lbo[idx];
            wave_sync();
            if (idx < end) lbo[idx + d] = v;
            wave_sync();
        }
    }
    MTE_DEV void lbo_shift_left(u32 from, u32 d) {  // lbo[from..n_lb) -> lbo[from-d..)
        for (u32 start = from; start < n_lb; start += 64) {
            u32 idx = start + L;
            u32 v = 0;
            if (idx < n_lb) v = lbo[idx];
            wave_sync();
            if (idx < n_lb) lbo[idx - d] = v;
            wave_sync();
        }
    }
    MTE_DEV u32 lbo_find(u32 blk) const {
        for (u32 base = 0; base < n_lb; base += 64) {
            u32 idx = base + L;
            u64 m = wave_ballot(idx < n_lb && lbo[idx] == blk);
            if (m) return base + (u32)__builtin_ctzll(m);
        }
        return NONE;
    }

    // ---------------------------------------------------------------- tree structure
    // Insert `nn` after `child` in `parent` (a node at level `lvl` >= 1); splits and root growth
    // follow insertingWalk/split/updateRoot (mergeTree.ts:2446-2489, 1876-1887).
    MTE_DEV void set_parent(u32 node, u32 lvl_of_node, u32 par) {
        if (L == 0) {
            if (lvl_of_node == 0) p.lb_par[node] = par;
            else p.in_par[node] = par;
        }
    }
    MTE_DEV void insert_after(u32 child, u32 nn, u32 lvl_child) {
        for (u32 guard = 0;; guard++) {
            if (guard > 32) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return;
            }
            u32 par = lvl_child == 0 ? p.lb_par[child] : p.in_par[child];
            if (par != NONE && bad_in(par)) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return;
            }
            if (par == NONE) {  // child is the root: updateRoot
                u32 r = alloc_in();
                if (r == NONE) return;
                if (L == 0) {
                    p.in_child[r * 8 + 0] = child;
                    p.in_child[r * 8 + 1] = nn;
                    p.in_cnt[r] = 2;
                    p.in_par[r] = NONE;
                }
                set_parent(child, lvl_child, r);
                set_parent(nn, lvl_child, r);
                wave_sync();
                root = r;
                height++;
                return;
            }
            u32 cnt = p.in_cnt[par];
            u32 c = (L < cnt) ? p.in_child[par * 8 + L] : NONE;
            u64 m = wave_ballot(L < cnt && c == child);
            u32 idx = (u32)__builtin_ctzll(m);
            wave_sync();
            if (L > idx && L < cnt) p.in_child[par * 8 + L + 1] = c;
            if (L == 0) {
                p.in_child[par * 8 + idx + 1] = nn;
                p.in_cnt[par] = cnt + 1;
            }
            set_parent(nn, lvl_child, par);
            wave_sync();
            if (cnt + 1 < 8) return;
            // split internal node `par` (mergeTree.ts:2476-2489)
            u32 q = alloc_in();
            if (q == NONE) return;
            u32 moved = NONE;
            if (L < 4) moved = p.in_child[par * 8 + 4 + L];
            wave_sync();
            if (L < 4) {
                p.in_child[q * 8 + L] = moved;
                if (lvl_child == 0) p.lb_par[moved] = q;
                else p.in_par[moved] = q;
            }
            if (L == 0) {
                p.in_cnt[par] = 4;
                p.in_cnt[q] = 4;
            }
            wave_sync();
            child = par;
            nn = q;
            lvl_child++;
        }
    }

    // Insert `rec` at slot j of leaf block `blk` (lbo index k); split 8 -> 4+4 on overflow.
    MTE_DEV void insert_slot(u32 k, u32 blk, u32 j, const SegRec& rec) {
        u32 cnt = p.lb_cnt[blk];
        bool mv = L >= j && L < cnt;
        SegRec t;
        if (mv) t = load_slot(blk, L);
        wave_sync();
        if (mv) store_slot(blk, L + 1, t);
        if (L == 0) {
            store_slot(blk, j, rec);
            p.lb_cnt[blk] = cnt + 1;
            set_seg_parent(rec.sid, blk);
        }
        wave_sync();
        if (cnt + 1 < 8) return;
        u32 nb = alloc_lb();
        if (nb == NONE) return;
        if (n_lb + 1 > cfg.lbo_cap) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return;
        }
        SegRec m;
        if (L < 4) m = load_slot(blk, 4 + L);
        wave_sync();
        if (L < 4) {
            store_slot(nb, L, m);
            set_seg_parent(m.sid, nb);
        }
        if (L == 0) {
            p.lb_cnt[blk] = 4;
            p.lb_cnt[nb] = 4;
        }
        wave_sync();
        lbo_shift_right(k + 1, 1);
        if (L == 0) lbo[k + 1] = nb;
        n_lb++;
        wave_sync();
        insert_after(blk, nb, 0);
    }

    // ensureIntervalBoundary split of slot i at r (BaseSegment.splitAt, mergeTree.ts:524-568).
    MTE_DEV void split_slot(const Found& f) {
        SegRec rec = load_slot(f.blk, (u32)f.slot);
        u32 sid = new_sid();
        if (sid == NONE) return;
        SegRec right = rec;
        u32 r = (u32)f.r;
        right.v.len = rec.v.len - r;
        right.toff = rec.toff + r;
        right.tcap = (rec.toff & ARENA_BIT) ? rec.tcap - r : 0u;
        right.sid = sid;
        rec.v.len = r;
        rec.tcap = (rec.toff & ARENA_BIT) ? r : 0u;
        wave_sync();
        if (L == 0) store_slot(f.blk, (u32)f.slot, rec);
        wave_sync();
        insert_slot(f.k, f.blk, (u32)f.slot + 1, right);
    }

    MTE_DEV void ensure_boundary(i32 pos, i32 R, u32 C) {  // mergeTree.ts:2241-2245
        Found f = resolve(pos, R, C, 0, 0);
        if (f.ok && f.slot >= 0 && f.r > 0) split_slot(f);
    }

    // ---------------------------------------------------------------- LRU heap (collections.ts:213-265)
    MTE_DEV void heap_push(u32 sid, i32 maxSeq) {
        if (heapSize + 1 >= cfg.heap_cap) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return;
        }
        heapSize++;
        if (L == 0) {
            u32 k = heapSize;
            heap[k] = make_uint2(sid, (u32)maxSeq);
            while (k > 1) {
                uint2 a = heap[k >> 1], b = heap[k];
                if (!((i32)a.y - (i32)b.y > 0)) break;
                heap[k >> 1] = b;
                heap[k] = a;
                k >>= 1;
            }
        }
        wave_sync();
    }
    MTE_DEV uint2 heap_pop() {
        uint2 x = make_uint2(0, 0);
        if (L == 0) {
            x = heap[1];
            u32 n = heapSize;
            heap[1] = heap[n];
            n--;
            u32 k = 1;
            while ((k << 1) <= n) {
                u32 j = k << 1;
                uint2 hj = heap[j];
                if (j < n) {
                    uint2 hj1 = heap[j + 1];
                    if ((i32)hj.y - (i32)hj1.y > 0) {
                        j++;
                        hj = hj1;
                    }
                }
                uint2 hk = heap[k];
                if ((i32)hk.y - (i32)hj.y <= 0) break;
                heap[k] = hj;
                heap[j] = hk;
                k = j;
            }
        }
        x.x = wave_read(x.x, 0);
        x.y = wave_read(x.y, 0);
        heapSize--;
        wave_sync();
        return x;
    }
    // addToLRUSet (mergeTree.ts:1273-1283) for a segment whose parent is `blk`.
    MTE_DEV void add_lru(u32 blk, u32 sid, i32 seq) {
        if (!collab) return;
        u32 sc = p.lb_scour[blk];
        if (sc != SC_TRUE && seq > curSeq) {
            wave_sync();
            if (L == 0) p.lb_scour[blk] = SC_TRUE;
            wave_sync();
            heap_push(sid, seq);
        }
    }

    // ---------------------------------------------------------------- property maps
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
        u32 id = NONE;
        i32 err = 0;
        if (mapNext >= cfg.map_cap) err = MTE_DOC_CAPACITY;
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
                id = mapNext;
                u32* m = maps + (u64)id * MAP_WORDS;
                m[0] = n;
                for (u32 i = 0; i < 2 * n; i++) m[1 + i] = kv[i];
            }
        }
        err = wave_read(err, 0);
        id = wave_read(id, 0);
        wave_sync();
        if (err) {
            fail(err, curSeq);
            return 0;
        }
        mapNext++;
        return id;
    }

    // ---------------------------------------------------------------- text arena
    MTE_DEV u16* text_ptr(u32 off) const {
        return (off & ARENA_BIT) ? arena0 + (u64)arenaSel * cfg.arena_cap + (off & ~ARENA_BIT) : payload + off;
    }
    MTE_DEV bool text_ok(u32 off, u32 n) const {
        u64 end = (u64)(off & ~ARENA_BIT) + n;
        return (off & ARENA_BIT) ? end <= cfg.arena_cap : end <= cfg.payload_len;
    }
    MTE_DEV u16 last_char(u32 off, u32 n) const {
        return (n > 0 && text_ok(off, n)) ? text_ptr(off)[n - 1] : (u16)0;
    }
    MTE_DEV void copy_text(u32 dst_off, u32 src_off, u32 n) {
        if (!text_ok(dst_off, n) || !text_ok(src_off, n)) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return;
        }
        u16* d = text_ptr(dst_off);
        const u16* s = text_ptr(src_off);
        for (u32 i = L; i < n; i += 64) d[i] = s[i];
    }
    // Semispace compaction of the merge arena (all live arena-resident segment texts).
    MTE_DEV void arena_gc() {
        u32 other = arenaSel ^ 1u;
        u16* dst = arena0 + (u64)other * cfg.arena_cap;
        u32 top = 0;
        for (u32 k = 0; k < n_lb; k++) {
            u32 blk = lbo[k];
            u32 cnt = lbcnt(blk);
            for (u32 s = 0; s < cnt; s++) {
                uint2 t = p.lb_txt[blk * 8 + s];
                u32 meta = p.lb_vis[blk * 8 + s].w;
                if ((meta & F_MARKER) || !(t.x & ARENA_BIT)) continue;
                u32 len = p.lb_vis[blk * 8 + s].x;
                u32 cap = t.y < len ? len : t.y;
                if (!text_ok(t.x, len) || top + cap > cfg.arena_cap) {
                    fail(MTE_DOC_CAPACITY, curSeq);
                    return;
                }
                const u16* src = text_ptr(t.x);
                for (u32 i = L; i < len; i += 64) dst[top + i] = src[i];
                wave_sync();
                if (L == 0) p.lb_txt[blk * 8 + s] = make_uint2(top | ARENA_BIT, cap);
                top += cap;
            }
        }
        wave_sync();
        arenaSel = other;
        arenaTop = top;
        nGc++;
    }
    MTE_DEV bool arena_reserve(u32 need) {
        if (arenaTop + need <= cfg.arena_cap) return true;
        arena_gc();
        if (arenaTop + need <= cfg.arena_cap) return true;
        fail(MTE_DOC_CAPACITY, curSeq);
        return false;
    }

    // ---------------------------------------------------------------- zamboni (mergeTree.ts:1289-1478)
    // One scourNode decision pass over the slots of a leaf block (held one per lane in `me`).
    // dry == true: no side effects, returns the arena units the real pass will allocate.
    // dry == false: performs merges (text appends) and records the kept list in LDS.
    MTE_DEV u32 scour_pass(bool dry, const SegRec& me, u32 cnt, u32& nkeep, u32* sc_keep, u32* sc_len,
                           u32* sc_off, u32* sc_cap) {
        u32 need = 0;
        nkeep = 0;
        i32 prev = -1;  // index into the kept list of the current merge target
        u32 pLen = 0, pOff = 0, pCap = 0, pProps = 0;
        bool pText = false, pNL = false;
        for (u32 s = 0; s < cnt; s++) {
            u32 len = wave_shfl(me.v.len, s);
            i32 seq = wave_shfl(me.v.seq, s);
            i32 rseq = wave_shfl(me.v.rseq, s);
            u32 meta = wave_shfl(me.v.meta, s);
            u32 props = wave_shfl(me.props, s);
            u32 toff = wave_shfl(me.toff, s);
            u32 tcap = wave_shfl(me.tcap, s);
            u32 sid = wave_shfl(me.sid, s);
            bool marker = (meta & F_MARKER) != 0;
            bool keep = false;
            if (meta & F_REMOVED) {  // tombstone: dropped once removed at or below the MSN (:1296-1319)
                if (rseq > minSeq) keep = true;
                else if (!dry && L == 0) set_seg_parent(sid, NONE);
                prev = -1;
            } else if (seq <= minSeq) {
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
                        u32 dst = arenaTop | ARENA_BIT;
                        if (!dry) {
                            arenaTop += ncap;
                            copy_text(dst, pOff, pLen);
                            copy_text(dst + pLen, toff, len);
                        }
                        pOff = dst;
                        pCap = ncap;
                    }
                    pLen += len;
                    if (!dry) {
                        pNL = last_char(toff, len) == u'\n';
                        wave_sync();
                        if (L == 0) {
                            set_seg_parent(sid, NONE);
                            sc_len[prev] = pLen;
                            sc_off[prev] = pOff;
                            sc_cap[prev] = pCap;
                        }
                    } else {
                        pNL = last_char(toff, len) == u'\n';
                    }
                } else {
                    keep = true;
                    prev = (i32)nkeep;
                    pLen = len;
                    pOff = toff;
                    pCap = tcap;
                    pProps = props;
                    pText = !marker;
                    pNL = !marker && last_char(toff, len) == u'\n';
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

    // scourNode on leaf block `blk`, compacting the kept slots in place; returns the new child count.
    MTE_DEV u32 scour(u32 blk, u32* sc_keep /*LDS[8]*/, u32* sc_len, u32* sc_off, u32* sc_cap) {
        u32 cnt = lbcnt(blk);
        SegRec me;
        if (L < cnt) me = load_slot(blk, L);
        u32 nkeep = 0;
        u32 need = scour_pass(true, me, cnt, nkeep, sc_keep, sc_len, sc_off, sc_cap);
        if (nkeep == cnt) return cnt;  // nothing dropped or merged => nothing changes
        if (need) {
            if (!arena_reserve(need)) return cnt;
            if (L < cnt) me = load_slot(blk, L);  // a GC may have moved arena texts
        }
        scour_pass(false, me, cnt, nkeep, sc_keep, sc_len, sc_off, sc_cap);
        if (status) return cnt;
        wave_sync();
        u32 src = L < nkeep ? sc_keep[L] : 0u;
        SegRec out = shfl_rec(me, src);
        if (L < nkeep) {
            out.v.len = sc_len[L];
            out.toff = sc_off[L];
            out.tcap = sc_cap[L];
        }
        wave_sync();
        if (L < nkeep) store_slot(blk, L, out);
        if (L == 0) p.lb_cnt[blk] = nkeep;
        wave_sync();
        return nkeep;
    }

    // pack (mergeTree.ts:1368-1420). `blk` underflowed; its parent's children are re-scoured and
    // redistributed into max(1, min(7, T/4)) fresh blocks.
    MTE_DEV void pack_leaf(u32 blk, u32* lds) {
        u32 par = p.lb_par[blk];
        if (bad_in(par) || p.in_cnt[par] > 8) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return;
        }
        u32 m = p.in_cnt[par];
        u32 kids = L < m ? p.in_child[par * 8 + L] : NONE;
        u32 cnts = 0;
        for (u32 i = 0; i < m; i++) {
            u32 c = wave_read(kids, i);
            u32 n = scour(c, lds, lds + 8, lds + 16, lds + 24);
            if (L == i) cnts = n;
            if (status) return;
        }
        wave_sync();
        u32 T = wave_sum(L < m ? cnts : 0u);
        u32 k = T / 4;
        if (k > 7) k = 7;
        if (k < 1) k = 1;
        u32 base = T / k, extra = T % k;
        u32 nb = NONE;
        for (u32 j = 0; j < k; j++) {
            u32 id = alloc_lb();
            if (id == NONE) return;
            if (L == j) nb = id;
        }
        // lane t < T moves hold[t]
        u32 sib = 0, q = L;
        for (u32 i = 0; i < m; i++) {
            u32 n = wave_read(cnts, i);
            if (q >= n && sib == i) {
                q -= n;
                sib = i + 1;
            }
        }
        u32 dj, dq;
        u32 big = extra * (base + 1);
        if (L < big) {
            dj = L / (base + 1);
            dq = L % (base + 1);
        } else {
            dj = extra + (L - big) / (base ? base : 1);
            dq = (L - big) % (base ? base : 1);
        }
        u32 srcBlk = wave_shfl(kids, sib < m ? sib : 0u);
        u32 dstBlk = wave_shfl(nb, dj < k ? dj : 0u);
        SegRec rec;
        if (L < T) rec = load_slot(srcBlk, q);
        wave_sync();
        if (L < T) {
            store_slot(dstBlk, dq, rec);
            set_seg_parent(rec.sid, dstBlk);
        }
        if (L < k) {
            u32 c = base + (L < extra ? 1u : 0u);
            p.lb_cnt[nb] = c;
            p.lb_par[nb] = par;
            p.in_child[par * 8 + L] = nb;
        }
        if (L == 0) p.in_cnt[par] = k;
        wave_sync();
        // splice lbo: the run of the parent's old children becomes the k new blocks
        u32 k0 = lbo_find(wave_read(kids, 0));
        if (k0 == NONE || k0 + m > n_lb) {
            fail(MTE_DOC_CAPACITY, curSeq);
            return;
        }
        if (k > m) {
            if (n_lb + (k - m) > cfg.lbo_cap) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return;
            }
            lbo_shift_right(k0 + m, k - m);
            n_lb += k - m;
        } else if (k < m) {
            lbo_shift_left(k0 + m, m - k);
            n_lb -= m - k;
        }
        if (L < k) lbo[k0 + L] = nb;
        wave_sync();
        for (u32 i = 0; i < m; i++) free_lb(wave_read(kids, i));
        if (k < 4 && p.in_par[par] != NONE) pack_internal(par, 1);
    }

    // pack on an interior level: `node` (level lvl) underflowed; redistribute the grandchildren of
    // its parent over max(1, min(7, T/4)) fresh interior nodes.
    MTE_DEV void pack_internal(u32 node, u32 lvl) {
        for (u32 guard = 0;; guard++) {
            if (guard > 32) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return;
            }
            u32 par = p.in_par[node];
            if (bad_in(par) || p.in_cnt[par] > 8) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return;
            }
            u32 m = p.in_cnt[par];
            u32 kids = L < m ? p.in_child[par * 8 + L] : NONE;
            u32 cnts = (L < m && !bad_in(kids)) ? p.in_cnt[kids] : 0u;
            if (wave_ballot(L < m && (bad_in(kids) || cnts > 8))) {
                fail(MTE_DOC_CAPACITY, curSeq);
                return;
            }
            u32 T = wave_sum(cnts);
            u32 k = T / 4;
            if (k > 7) k = 7;
            if (k < 1) k = 1;
            u32 base = T / k, extra = T % k;
            u32 nb = NONE;
            for (u32 j = 0; j < k; j++) {
                u32 id = alloc_in();
                if (id == NONE) return;
                if (L == j) nb = id;
            }
            u32 sib = 0, q = L;
            for (u32 i = 0; i < m; i++) {
                u32 n = wave_read(cnts, i);
                if (q >= n && sib == i) {
                    q -= n;
                    sib = i + 1;
                }
            }
            u32 big = extra * (base + 1), dj, dq;
            if (L < big) {
                dj = L / (base + 1);
                dq = L % (base + 1);
            } else {
                dj = extra + (L - big) / (base ? base : 1);
                dq = (L - big) % (base ? base : 1);
            }
            u32 srcN = wave_shfl(kids, sib < m ? sib : 0u);
            u32 dstN = wave_shfl(nb, dj < k ? dj : 0u);
            u32 gc = NONE;
            if (L < T) gc = p.in_child[srcN * 8 + q];
            wave_sync();
            if (L < T) {
                p.in_child[dstN * 8 + dq] = gc;
                if (lvl == 1) p.lb_par[gc] = dstN;
                else p.in_par[gc] = dstN;
            }
            if (L < k) {
                p.in_cnt[nb] = base + (L < extra ? 1u : 0u);
                p.in_par[nb] = par;
                p.in_child[par * 8 + L] = nb;
            }
            if (L == 0) p.in_cnt[par] = k;
            wave_sync();
            for (u32 i = 0; i < m; i++) free_in(wave_read(kids, i));
            if (k < 4 && p.in_par[par] != NONE) {
                node = par;
                lvl++;
                continue;
            }
            return;
        }
    }

    MTE_DEV void zamboni(u32* lds) {  // zamboniSegments (mergeTree.ts:1422-1478)
        if (!collab) return;
        for (int i = 0; i < 2 && !status; i++) {
            if (heapSize == 0) break;
            i32 top = (i32)heap[1].y;
            if (top > minSeq) break;
            uint2 e = heap_pop();
            u32 par = e.x < cfg.seg_cap ? segParent[e.x] : NONE;
            if (par == NONE || bad_blk(par)) continue;
            if (p.lb_scour[par] == SC_FALSE) continue;
            u32 old = p.lb_cnt[par];
            u32 nc = scour(par, lds, lds + 8, lds + 16, lds + 24);
            if (L == 0) p.lb_scour[par] = SC_FALSE;
            wave_sync();
            if (nc < old && nc < 4 && height > 1) pack_leaf(par, lds);
        }
    }

    // ---------------------------------------------------------------- ops
    // insertSegments (mergeTree.ts:1968-1998) for one new segment.
    MTE_DEV void insert_op(i32 pos, i32 R, u32 C, i32 seq, SegRec rec, u32* lds) {
        Found f = resolve(pos, R, C, 0, 0);
        if (!f.ok) {
            fail(MTE_DOC_INSERT_FAILED, seq);
            return;
        }
        if (f.slot >= 0 && f.r > 0) {
            split_slot(f);
            if (status) return;
            f = resolve(pos, R, C, f.k, f.cum);
            if (!f.ok) {
                fail(MTE_DOC_INSERT_FAILED, seq);
                return;
            }
        }
        if (rec.v.len == 0) return;  // blockInsert skips empty segments (:2196)
        rec.sid = new_sid();
        if (rec.sid == NONE) return;
        u32 cnt = p.lb_cnt[f.blk];
        u32 j = f.slot >= 0 ? (u32)f.slot : cnt;
        insert_slot(f.k, f.blk, j, rec);
        if (status) return;
        if (collab && seq > minSeq && rec.sid < cfg.seg_cap) add_lru(segParent[rec.sid], rec.sid, seq);
        zamboni(lds);
    }

    // markRangeRemoved / annotateRange mark pass (nodeMap, mergeTree.ts:2903-2965).
    MTE_DEV void range_op(bool remove, i32 p1, i32 p2, i32 R, u32 C, i32 seq, u32 propset, bool rewrite) {
        i32 cum = 0;
        const u32 s = L & 7;
        u32 memoOld = NONE, memoNew = 0;
        for (u32 base = 0; base < n_lb && cum < p2; base += 8) {
            u32 bk = base + (L >> 3);
            u32 blk = bk < n_lb ? lbo[bk] : NONE;
            u32 cnt = lbcnt(blk);
            u32 v = 0;
            Slot sl{0, 0, 0, 0};
            if (s < cnt) {
                uint4 q = p.lb_vis[blk * 8 + s];
                sl = Slot{q.x, (i32)q.y, (i32)q.z, q.w};
                v = vislen(sl, blk * 8 + s, R, C);
            }
            u32 incl = wave_scan_incl(v);
            i32 ex = cum + (i32)(incl - v);
            bool mark = v > 0 && ex < p2 && ex + (i32)v > p1;
            u64 mm = wave_ballot(mark);
            cum += (i32)wave_read(incl, 63);
            if (!mm) continue;
            u32 idx = blk * 8 + s;
            if (remove) {
                if (mark) {
                    if (sl.meta & F_REMOVED) {
                        p.lb_ovl[idx] |= (1ull << C);  // addOverlappingClient (:2544-2552)
                    } else {
                        sl.meta = (sl.meta & ~0xff00u) | (C << 8) | F_REMOVED;
                        sl.rseq = seq;
                        p.lb_vis[idx] = make_uint4(sl.len, (u32)sl.seq, (u32)sl.rseq, sl.meta);
                    }
                }
            } else {
                u32 props = mark ? p.lb_props[idx] : 0u;
                u64 pending = mm;
                while (pending) {
                    u32 leader = (u32)__builtin_ctzll(pending);
                    u32 old = wave_read(props, leader);
                    u32 nid;
                    if (old == memoOld) {
                        nid = memoNew;
                    } else {
                        nid = build_map(old, propset, rewrite);
                        if (status) return;
                        memoOld = old;
                        memoNew = nid;
                    }
                    bool same = mark && props == old && ((pending >> L) & 1ull);
                    if (same) p.lb_props[idx] = nid;
                    pending &= ~wave_ballot(same);
                }
            }
            wave_sync();
            // addToLRUSet in document order: per leaf block, only the first marked slot can enqueue
            if (collab) {
                u32 sid = mark ? p.lb_sid[idx] : 0u;
                for (u32 j = 0; j < 8; j++) {
                    u32 bm = (u32)((mm >> (8 * j)) & 0xffull);
                    if (!bm) continue;
                    u32 lead = 8 * j + (u32)__builtin_ctz(bm);
                    add_lru(wave_read(blk, lead), wave_read(sid, lead), seq);
                    if (status) return;
                }
            }
        }
    }

    MTE_DEV void remove_op(i32 p1, i32 p2, i32 R, u32 C, i32 seq, u32* lds) {  // mergeTree.ts:2607-2719
        ensure_boundary(p1, R, C);
        if (status) return;
        ensure_boundary(p2, R, C);
        if (status) return;
        range_op(true, p1, p2, R, C, seq, 0, false);
        if (status) return;
        zamboni(lds);
    }

    MTE_DEV void annotate_op(i32 p1, i32 p2, i32 R, u32 C, i32 seq, u32 propset, bool rewrite, u32* lds) {
        ensure_boundary(p1, R, C);  // mergeTree.ts:2565-2605
        if (status) return;
        ensure_boundary(p2, R, C);
        if (status) return;
        range_op(false, p1, p2, R, C, seq, propset, rewrite);
        if (status) return;
        zamboni(lds);
    }

    // Client.applyMsg for one op record (client.ts:805-836).
    MTE_DEV void apply(const mte_op& op, u32* lds) {
        if (op.client >= MTE_MAX_CLIENTS) {
            fail(MTE_DOC_UNSUPPORTED, op.seq);
            return;
        }
        u32 C = collab ? (u32)op.client : 0u;
        i32 seq = collab ? op.seq : 0;
        i32 R = collab ? op.ref_seq : 0;
        if (collab && op.type != MTE_OP_NOOP && !(curSeq < op.seq)) {
            fail(MTE_DOC_SEQ_ORDER, op.seq);
            return;
        }
        switch (op.type) {
            case MTE_OP_INSERT:
            case MTE_OP_INSERT_MARKER: {
                SegRec rec;
                bool mk = op.type == MTE_OP_INSERT_MARKER;
                rec.v.len = mk ? 1u : op.b;
                rec.v.seq = seq;
                rec.v.rseq = 0;
                rec.v.meta = (C & 0xff) | (mk ? F_MARKER : 0u);
                rec.ovl = 0;
                rec.props = op.props ? build_map(0, op.props, false) : 0u;
                if (status) return;
                rec.toff = mk ? op.b : (u32)op.a;
                rec.tcap = 0;
                rec.sid = 0;
                insert_op(op.pos1, R, C, seq, rec, lds);
                opsApplied++;
                break;
            }
            case MTE_OP_REMOVE:
                remove_op(op.pos1, op.a, R, C, seq, lds);
                opsApplied++;
                break;
            case MTE_OP_ANNOTATE:
                annotate_op(op.pos1, op.a, R, C, seq, op.props, (op.flags & MTE_F_REWRITE) != 0, lds);
                opsApplied++;
                break;
            default:
                break;
        }
        if (status) return;
        if (collab && (op.flags & MTE_F_END_OF_MSG)) {  // updateSeqNumbers / setMinSeq (:829-836, mergeTree.ts:1718-1736)
            msgs++;
            if (op.seq < curSeq || op.msn > op.seq || op.msn < minSeq) {
                fail(MTE_DOC_SEQ_ORDER, op.seq);
                return;
            }
            curSeq = op.seq;
            if (op.msn > minSeq) {
                minSeq = op.msn;
                zamboni(lds);
            }
        }
    }

    // ---------------------------------------------------------------- driver
    MTE_DEV void init() {
        u32 r = alloc_lb();
        root = r;
        height = 1;
        if (r == NONE) return;
        if (L == 0) lbo[0] = r;
        n_lb = 1;
        wave_sync();
    }

    MTE_DEV void finish() {
        if (L == 0) {
            DocRes& o = p.res[doc];
            o.status = status;
            o.failing_seq = failingSeq;
            o.ops = opsApplied;
            o.msgs = msgs;
            o.min_seq = minSeq;
            o.cur_seq = curSeq;
            o.root = root;
            o.height = height;
            o.n_lb = n_lb;
            o.arena_sel = arenaSel;
            o.arena_top = arenaTop;
            o.map_next = mapNext;
            o.seg_next = segNext;
            o.heap_size = heapSize;
            o.n_gc = nGc;
            o.lb_free = lbFree;
        }
    }

    MTE_DEV void replay(u32* lds) {
        init();
        for (u64 i = cfg.op_begin; i < cfg.op_end && !status; i++) {
            mte_op op = p.ops[i];
            apply(op, lds);
        }
        finish();
    }

    // Synthetic workload generator: simulated writers draw valid ops from their own
    // view (getLength(refSeq, client)); each op is recorded into the doc's op/payload slots and
    // applied immediately, so the recorded log is exactly what a replay will see.
    MTE_DEV void generate(u32* lds) {
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
        for (u64 step = 0; step < nops && !status; step++) {
            i32 seq = (i32)step + 1;
            i32 cur = seq - 1;
            u32 c = rng.below(nc);
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
            u32 C = sid_of[c];
            i32 R = ref[c];
            i32 len = get_length(R, C);
            u32 roll = rng.below(100);
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
                i32 pos = forced ? (lastPos < len ? lastPos : len) : (i32)rng.below((u32)len + 1);
                u32 n = 1 + rng.below(8);
                op.pos1 = pos;
                op.a = (i32)pay;
                op.b = n;
                for (u32 i = 0; i < n; i++) {
                    u16 ch = (u16)(u'a' + rng.below(26));
                    if (L == 0) payload[pay + i] = ch;
                }
                pay += n;
                if (p.gen_kind == 3 && rng.below(4) == 0) op.props = 1 + rng.below(p.gen_n_propsets);
            } else {
                i32 a = forced ? (lastPos < len ? lastPos : len - 1) : (i32)rng.below((u32)len);
                i32 n = 1 + (i32)rng.below(16);
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
            wave_sync();
            apply(op, lds);
        }
        finish();
    }
};

}  // namespace mte
