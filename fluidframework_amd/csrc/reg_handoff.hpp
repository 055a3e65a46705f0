// reg_handoff.hpp — hand a document from the register-resident engine (reg_engine.hpp) to the
// LDS-resident solo engine (engine.hpp, Engine<true, true, LVL>: k_solo) or to an HBM-resident one
// (Engine<false, false, LVL> in a wave's HBM slot: k_rows) between two ops.
//
// The register engine keeps leaf blocks in document order and the interior levels as child-count
// vectors; the LDS engine keeps blocks and interior nodes by id with parent pointers and a doc-order
// block list. The handoff assigns ids in document order (leaf block k -> id k; interior nodes level by
// level), writes every slot, block summary, interior node and heap entry, and copies the replay state
// and per-document counters. Taken only when a document outgrows the register plan or reaches an op
// the register engine does not implement (reg_engine.hpp apply()), so it is built for clarity, not speed.
#pragma once
#include "engine.hpp"
#include "reg_engine.hpp"

namespace mte {

// Returns false, writing nothing, when the target's arrays cannot hold the document's state (an HBM
// slot sized for shorter documents): the caller gives the document to the host's re-run then.
template <class E, class R>
MTE_DEV bool reg_handoff(R& r, E& e) {
    using simd::V;
    const u32 L = lane_id();
    const u32 nrows = (r.n_lb + 7) >> 3;
    // interior node ids: level i (1..height-1) nodes get ids base[i] .. base[i] + n[i] - 1
    const u32 H = r.height;
    u32 base[RG_LEVELS + 2], nn[RG_LEVELS + 2];
    u32 tot = 0;
    for (u32 i = 1; i < H; i++) {
        nn[i] = i == H - 1 ? 1u : simd::readlane(simd::scan_incl(r.LV.get(i)), 63);
        base[i] = tot;
        tot += nn[i];
    }
    if (nrows * 8 > e.blk_cap() || r.n_lb > e.ord_cap() || tot > e.in_cap() || r.heapSize >= e.heap_cap()) return false;
    // leaf block summaries and metadata (parent | needsScour << 30)
    u32 node = 0, left = H > 1 ? simd::readlane(r.LV.get(0), 0) : 0u;
    for (u32 k = 0; k < r.n_lb; k++) {
        if (H > 1) {
            while (left == 0 && node + 1 < 64) left = simd::readlane(r.LV.get(0), ++node);
            left--;
        }
        const u32 rr = k >> 3, gb = (k & 7) * 8;
        const auto w = r.ldrow(rr);
        u32 olen = 0, cnt = 0;
        i32 mx = 0;
        for (u32 s = 0; s < 8; s++) {
            const u32 len = simd::readlane(w.len, gb + s);
            if (!len) continue;
            const i32 seq = (i32)simd::readlane(w.seq, gb + s);
            const u32 rseq = simd::readlane(w.rseq, gb + s);
            const bool live = rseq == RSEQ_LIVE;
            cnt++;
            olen += live ? len : 0u;
            const i32 hi = !live && (i32)rseq > seq ? (i32)rseq : seq;
            if (cnt == 1 || hi > mx) mx = hi;
        }
        const u32 par = H > 1 ? base[1] + node : BM_NOPAR;
        if (L == 0) {
            e.ORD()[k] = make_uint4(k, olen, (u32)mx, cnt);
            e.BMETA()[k] = (par & BM_PAR) | (((simd::readlane(w.meta, gb) >> NS_SHIFT) & 3u) << 30);
        }
    }
    // interior nodes: children, counts, parents
    for (u32 i = 1; i < H; i++) {
        const simd::V cntv = r.LV.get(i - 1);
        u32 first = 0, pnode = 0, pleft = i + 1 < H ? simd::readlane(r.LV.get(i), 0) : 0u;
        for (u32 j = 0; j < nn[i]; j++) {
            const u32 c = simd::readlane(cntv, j);
            const u32 id = base[i] + j;
            u32 par = NONE;
            if (i + 1 < H) {
                while (pleft == 0 && pnode + 1 < 64) pleft = simd::readlane(r.LV.get(i), ++pnode);
                pleft--;
                par = base[i + 1] + pnode;
            }
            if (L < c && L < 8) e.INCH()[id * 8 + L] = i == 1 ? first + L : base[i - 1] + first + L;
            if (L == 0) {
                e.INCNT()[id] = c;
                e.INPAR()[id] = par;
            }
            first += c;
        }
    }
    // LRU heap (positions 1..heapSize). The register index must be a compile-time constant: a
    // run-time index here made the compiler keep a heap register set in scratch memory for the whole
    // kernel, so every heap access of the row engine's replay loop was a scratch load.
#pragma unroll
    for (u32 j = 0; j < 8; j++) {
        const u32 q = j * 64 + L;
        const u32 hk = r.HK.get(j).x, hs = r.HS.get(j).x;
        if (q >= 1 && q <= r.heapSize) e.HEAP()[q] = make_uint2(hs - 1u, hk);  // ids 1-based in the rows
    }
    // slots: row rr lane l is block 8*rr + l/8, slot l%8 = the LDS engine's slot index 64*rr + l
    // (for k_solo the same LDS words: each lane reads its slot before it rewrites it); only the
    // encoding of live segments and needsScour differ
    lds_order();
    for (u32 rr = 0; rr < nrows; rr++) {
        const auto w = r.ldrow(rr);
        const uint4 v = make_uint4(w.len.x, w.seq.x, w.rseq.x, w.meta.x), a = make_uint4(w.cap.x, w.toff.x, w.rm.x, w.sid.x);
        const bool live = v.z == RSEQ_LIVE, ov = (v.w & F_OVL) != 0;
        const u32 m2 = (live ? (v.w & ~0xFF00u) : v.w) & ~NS_MASK;
        // aux.z: a live segment's text capacity, a removed one's removedClientOverlap (rm without
        // removedClient) or 0
        u32 ovm = a.z & ~(1u << ((v.w >> 8) & 31u)), m3 = m2;
        if constexpr (R::kWide) {  // removers 32..63: the LDS engine keeps them in its HBM mask by id
            const u32 rc = (v.w >> 8) & 0xFFu, rm2 = w.rm2.x;
            ovm = a.z & ~(rc < 32 ? 1u << rc : 0u);
            const u32 hi = (!live && ov) ? rm2 & ~(rc >= 32 ? 1u << (rc & 31u) : 0u) : 0u;
            if (v.x && hi && a.w - 1u < e.seg_cap) {
                e.ovl[a.w - 1u] = (u64)hi << 32;
                if (e.ovl2) e.ovl2[a.w - 1u] = 0ull;  // (the row engine's writers are below 64)
                m3 |= F_OVLHI;
            }
        }
        lds_order();  // (k_solo: the row's reads before the writes over the same words)
        e.VIS()[64 * rr + L] = make_uint4(v.x, v.y, live ? 0u : v.z, m3);
        u32 props = 0;
        if constexpr (R::kProps) props = v.x ? w.props.x : 0u;
        e.AUX()[64 * rr + L] = make_uint4(props, a.y, live ? a.x : (ov ? ovm : 0u), v.x ? a.w - 1u : 0u);
    }
    // replay state and per-document counters
    St& st = e.st;
    st.root = H > 1 ? base[H - 1] : 0u;
    st.height = H;
    st.n_lb = r.n_lb;
    st.minSeq = r.minSeq;
    st.curSeq = r.curSeq;
    st.heapSize = r.heapSize;
    st.heapTop = r.heapTop;
    st.segNext = r.segNext;
    st.arenaTop = r.arenaTop;
    st.arenaSel = r.arenaSel;
    if constexpr (R::kProps) st.mapNext = r.mapNext;  // the same per-document map table
    else st.mapNext = 1;
    st.lbFree = NONE;
    st.lbBump = r.n_lb;
    st.inFree = NONE;
    st.inBump = tot;
    st.inUsed = tot;
    st.credit = 0;
    st.status = 0;
    st.adirty = 1;  // merge-arena text written by other lanes: fence before the next read
    st.gdirty = R::kProps ? 1 : 0;  // map records written lane-parallel by the register engine
    if (L == 0) {
        u32* S = e.STATS();
        S[ST_OPS] = r.ops_n();
        S[ST_MSGS] = r.msgs_n();
        S[ST_GC] = r.n_gc;
        S[ST_MAXLB] = r.max_lb;
        S[ST_FAILSEQ] = NONE;
        S[ST_APPEND] = 0;
        S[ST_CU] = 0;
        S[E::ST_CUOP] = 0;
    }
    wave_sync();  // LDS state and the arena text the register engine wrote, before the LDS engine reads
    return true;
}

}  // namespace mte
