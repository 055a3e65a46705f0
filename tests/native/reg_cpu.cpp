// TEST INFRASTRUCTURE ONLY: the register-resident replay engine (fluidframework_amd/csrc/reg_engine.hpp)
// built for the CPU with the emulated wave backend (wave_simd.hpp MTE_CPU), so the CPU suite can check
// the engine's logic against the oracle without a GPU (tests/test_reg_engine_cpu.py). The product
// runs the device build only (k_solo); nothing in fluidframework_amd/ loads this library.
#define MTE_CPU 1
#include <string.h>

#include <vector>

#include "../../fluidframework_amd/csrc/reg_engine.hpp"

using namespace mte;


// Replays one document's op records. Outputs are the engine's own final rows (LDS-engine format:
// vis = len, seq, removedSeq, meta; aux = props, text offset, text capacity / overlap, segment id),
// the gathered text, and the DocRes record. Returns the op index the replay stopped at (n_ops when
// done or failed; earlier when the document would hand over to the LDS engine).
// Property tables of a PROPS replay (the host's interned propsets, Params::propsets & co.).
struct PropTables {
    const mte_propset* propsets;
    uint32_t n_propsets;
    const uint32_t* prop_keys;
    const uint32_t* prop_vals;
    const uint32_t* val_flags;
    uint32_t n_vals;
    uint32_t map_words, map_cap;
    uint32_t* out_maps;  // per output row, map_words words
};

template <bool PAGED, bool PROPS, bool WIDE = false>
static uint64_t replay_impl(const mte_op* ops, uint64_t n_ops, const uint16_t* payload, uint32_t payload_len,
                            uint32_t seg_cap, uint32_t arena_cap, uint32_t* out_vis, uint32_t* out_aux,
                            uint64_t* out_ovl, uint32_t out_cap, uint16_t* out_text, uint64_t out_text_cap,
                            DocRes* res, uint32_t pool_rows, const PropTables* pt = nullptr, uint64_t cut = 0,
                            uint64_t* ck_resumed = nullptr) {
    std::vector<uint16_t> pay(payload, payload + payload_len + 1);
    std::vector<uint16_t> arena((size_t)arena_cap * 2 + 1, 0);
    DocCfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.op_begin = 0;
    cfg.op_end = n_ops;
    cfg.payload_len = payload_len;
    cfg.arena_cap = arena_cap;
    cfg.seg_cap = seg_cap;
    cfg.collab = 1;
    uint32_t counters[16] = {0};
    Params p;
    memset(&p, 0, sizeof p);
    p.ops = (mte_op*)ops;
    p.payload = pay.data();
    p.docs = &cfg;
    p.n_docs = 1;
    p.res = res;
    p.arena = arena.data();
    p.out_vis = (uint4*)out_vis;
    p.out_aux = (uint4*)out_aux;
    p.out_ovl = out_ovl;
    p.out_cap = out_cap;
    p.out_text = out_text;
    p.out_text_cap = out_text_cap;
    p.counters = counters;
    std::vector<uint32_t> maps, objidx;
    std::vector<uint64_t> objmatch;
    if (PROPS) {
        cfg.map_cap = pt->map_cap;
        maps.assign((size_t)pt->map_cap * pt->map_words, 0);
        objidx.assign(pt->n_vals, NONE);
        objmatch.assign(pt->n_vals, 0);
        p.maps = maps.data();
        p.map_words = pt->map_words;
        p.propsets = pt->propsets;
        p.n_propsets = pt->n_propsets;
        p.prop_keys = pt->prop_keys;
        p.prop_vals = pt->prop_vals;
        p.val_flags = pt->val_flags;
        p.val_objidx = objidx.data();
        p.val_objmatch = objmatch.data();
        p.n_vals = pt->n_vals;
        p.out_maps = pt->out_maps;
    }
    // (the paged engine's pool is its own row arrays here, rows taken in a scattered order)
    typedef RegEngine<(int)RG_ROWS, PAGED, PROPS, WIDE> E;
    auto make = [&]() {
        E* x = new E(p, 0);
        if (PAGED) {
            x->release_rows();
            x->pool_rows = pool_rows < RG_ROWS ? pool_rows : RG_ROWS;
            x->init();
        }
        return x;
    };
    E* ep = make();
    uint64_t at0 = 0;
    std::vector<uint32_t> ck;
    if (cut && cut < n_ops) {
        // incremental replay (option retain): ops [0, cut) in a first "pass" that checkpoints, then a
        // fresh engine -- a fresh arena and map table -- continues from the checkpoint
        cfg.op_end = cut;
        cfg.ck_cap = E::ck_words(arena_cap, cfg.map_cap, PROPS ? pt->map_words : 0);
        ck.assign(cfg.ck_cap, 0);
        p.ck_out = ck.data();
        const uint64_t a1 = ep->status ? 0 : ep->replay(0, cut);
        if (ep->status == 0 && a1 == cut) ep->ckpt_save(a1);
        delete ep;
        p.ck_out = nullptr;
        std::fill(arena.begin(), arena.end(), (uint16_t)0);
        std::fill(maps.begin(), maps.end(), 0u);
        cfg.op_end = n_ops;
        cfg.ck_at = cut;
        p.ck_in = ck.data();
        ep = make();
        at0 = ep->ckpt_resume(0);
        if (ck_resumed) *ck_resumed = at0;
    }
    E& e = *ep;
    const uint64_t at = e.status ? 0 : e.replay(at0, n_ops);
    if (e.status == REG_HANDOFF) {
        memset(res, 0, sizeof *res);
        res->status = REG_HANDOFF;
        res->n_lb = e.n_lb;
        res->heap_size = e.heapSize;
        res->height = e.height;
        delete ep;
        return at;
    }
    e.finish();
    delete ep;
    return at;
}

extern "C" {

uint64_t regcpu_replay(const mte_op* ops, uint64_t n_ops, const uint16_t* payload, uint32_t payload_len,
                       uint32_t seg_cap, uint32_t arena_cap, uint32_t* out_vis, uint32_t* out_aux,
                       uint64_t* out_ovl, uint32_t out_cap, uint16_t* out_text, uint64_t out_text_cap,
                       DocRes* res) {
    return replay_impl<false, false>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                     out_cap, out_text, out_text_cap, res, 0);
}

// The PAGED engine (k_rows): logical rows mapped to pool rows taken in a scattered order from a pool
// of pool_rows rows; a document the pool cannot hold stops with REG_HANDOFF (k_rows spills it).
uint64_t regcpu_replay_paged(const mte_op* ops, uint64_t n_ops, const uint16_t* payload, uint32_t payload_len,
                             uint32_t seg_cap, uint32_t arena_cap, uint32_t* out_vis, uint32_t* out_aux,
                             uint64_t* out_ovl, uint32_t out_cap, uint16_t* out_text, uint64_t out_text_cap,
                             DocRes* res, uint32_t pool_rows) {
    return replay_impl<true, false>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                    out_cap, out_text, out_text_cap, res, pool_rows);
}

// The PROPS engine (k_rows of property-carrying batches), paged when pool_rows > 0: property maps in
// a table of map_cap records of map_words words; each final row's map copied to out_maps.
uint64_t regcpu_replay_props(const mte_op* ops, uint64_t n_ops, const uint16_t* payload, uint32_t payload_len,
                             uint32_t seg_cap, uint32_t arena_cap, uint32_t* out_vis, uint32_t* out_aux,
                             uint64_t* out_ovl, uint32_t out_cap, uint16_t* out_text, uint64_t out_text_cap,
                             DocRes* res, uint32_t pool_rows, const uint32_t* propsets, uint32_t n_propsets,
                             const uint32_t* prop_keys, const uint32_t* prop_vals, const uint32_t* val_flags,
                             uint32_t n_vals, uint32_t map_words, uint32_t map_cap, uint32_t* out_maps, uint32_t wide) {
    PropTables t{(const mte_propset*)propsets, n_propsets, prop_keys, prop_vals, val_flags, n_vals, map_words, map_cap, out_maps};
    if (wide && pool_rows)  // k_rows' WIDE instantiation (batches with writers 32..63), paged
        return replay_impl<true, true, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux,
                                             out_ovl, out_cap, out_text, out_text_cap, res, pool_rows, &t);
    if (wide)  // k_solo's FULL instantiation: clients up to 63
        return replay_impl<false, true, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux,
                                              out_ovl, out_cap, out_text, out_text_cap, res, 0, &t);
    if (pool_rows)
        return replay_impl<true, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                       out_cap, out_text, out_text_cap, res, pool_rows, &t);
    return replay_impl<false, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                    out_cap, out_text, out_text_cap, res, 0, &t);
}

// Incremental replay: ops [0, cut) checkpointed (reg_engine.hpp ckpt_save), the rest continued on a
// fresh engine from the checkpoint (ckpt_resume; *resumed = the op it went on from, 0 = it started
// over). kind: 0 lean, 1 paged, 2 PROPS (3 PROPS paged, +4 WIDE) with the tables of regcpu_replay_props.
uint64_t regcpu_replay_split(const mte_op* ops, uint64_t n_ops, const uint16_t* payload, uint32_t payload_len,
                             uint32_t seg_cap, uint32_t arena_cap, uint32_t* out_vis, uint32_t* out_aux,
                             uint64_t* out_ovl, uint32_t out_cap, uint16_t* out_text, uint64_t out_text_cap,
                             DocRes* res, uint32_t pool_rows, uint32_t kind, uint64_t cut, uint64_t* resumed,
                             const uint32_t* propsets, uint32_t n_propsets, const uint32_t* prop_keys,
                             const uint32_t* prop_vals, const uint32_t* val_flags, uint32_t n_vals, uint32_t map_words,
                             uint32_t map_cap, uint32_t* out_maps) {
    PropTables t{(const mte_propset*)propsets, n_propsets, prop_keys, prop_vals, val_flags, n_vals, map_words, map_cap, out_maps};
    switch (kind) {
        case 0:
            return replay_impl<false, false>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                             out_cap, out_text, out_text_cap, res, 0, nullptr, cut, resumed);
        case 1:
            return replay_impl<true, false>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                            out_cap, out_text, out_text_cap, res, pool_rows, nullptr, cut, resumed);
        case 2:
            return replay_impl<false, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                            out_cap, out_text, out_text_cap, res, 0, &t, cut, resumed);
        case 3:
            return replay_impl<true, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux, out_ovl,
                                           out_cap, out_text, out_text_cap, res, pool_rows, &t, cut, resumed);
        case 6:
            return replay_impl<false, true, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux,
                                                  out_ovl, out_cap, out_text, out_text_cap, res, 0, &t, cut, resumed);
        default:
            return replay_impl<true, true, true>(ops, n_ops, payload, payload_len, seg_cap, arena_cap, out_vis, out_aux,
                                                 out_ovl, out_cap, out_text, out_text_cap, res, pool_rows, &t, cut, resumed);
    }
}

uint32_t regcpu_docres_size(void) { return (uint32_t)sizeof(DocRes); }

// The engine's LRU heap alone: ops[i] > 0 pushes (segment id i + 1, key ops[i]), ops[i] == 0 pops.
// Writes the popped segment ids in order; returns how many (the heap's own sift rules, both the
// lane-parallel and the serial pop, against tests/test_reg_engine_cpu.py's restatement).
uint32_t regcpu_heap(const int32_t* ops, uint32_t n, uint32_t* popped) {
    DocCfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.seg_cap = 1;
    cfg.arena_cap = 1;
    Params p;
    memset(&p, 0, sizeof p);
    p.docs = &cfg;
    p.n_docs = 1;
    uint16_t pay[2] = {0, 0};
    p.payload = pay;
    p.arena = pay;
    RegEngine<>* e = new RegEngine<>(p, 0);
    uint32_t np = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (ops[i] > 0) {
            e->heap_push(i + 1, ops[i]);
        } else if (e->heapSize) {
            popped[np++] = e->heap_pop();
        }
    }
    delete e;
    return np;
}

#ifdef MTE_CPU_STATS
// the event statistics of every replay since the last call (tools/rg_stats.py), then cleared
uint32_t regcpu_stats(uint64_t* out, uint32_t n) {
    const uint32_t m = n < (uint32_t)RS_N + 2 ? n : (uint32_t)RS_N + 2;
    for (uint32_t i = 0; i < m; i++) out[i] = g_rg_stats[i];
    memset(g_rg_stats, 0, sizeof g_rg_stats);
    return (uint32_t)RS_N;
}
#endif
}
