// mte_host.cpp — host side of the MI355X merge-tree replay engine: the C ABI of include/mte.h.
//
//   * mte_builder_*: ISequencedDocumentMessage JSON logs -> SoA op records + interned property sets
//     (Client.applyMsg input, client.ts:805-836; op shapes ops.ts:29-110).
//   * mte_load / mte_generate: stage batches in HBM, size per-document arenas.
//   * mte_replay: one wavefront per document on the GPU (mte_kernels.hip / engine.hpp): an
//     LDS-resident pass over every document, then an HBM-resident pass for the documents that
//     outgrew the LDS plan.
//   * outputs: text (textSegment.ts:154-172), segment table (walkAllSegments, mergeTree.ts:2969),
//     SnapshotV1 ITree (snapshotV1.ts:85-247), per-doc FNV-1a-64 summary.
// There is no CPU execution path for replay: without a HIP device mte_create fails.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mte.h"
#include "../../include/mte_diag.h"
#include "emit.h"
#include "engine_types.hpp"
#include "gather_plan.hpp"
#include "jsonlite.hpp"
#include "mte_kernels.h"

using namespace mte;

namespace {

struct HostBatch {
    std::vector<uint64_t> doc_op_offsets{0};
    std::vector<mte_op> ops;
    std::vector<uint64_t> doc_payload_offsets{0};
    std::vector<uint16_t> payload;
    std::vector<mte_propset> propsets{mte_propset{0, 0}};
    std::vector<uint32_t> prop_keys, prop_vals;
    std::vector<uint64_t> key_offsets{0};
    std::string key_text;
    std::vector<uint64_t> val_offsets{0};
    std::string val_text;
    std::vector<uint32_t> doc_client_offsets{0};
    std::vector<uint64_t> client_name_offsets{0};
    std::string client_names;
    // legacy catch-up messages (include/mte.h mte_batch.msg_*)
    std::vector<uint64_t> doc_msg_offsets{0};
    std::vector<uint64_t> msg_first_op;
    std::vector<uint64_t> msg_text_offsets{0};
    std::string msg_text;

    uint32_t n_docs() const { return (uint32_t)doc_op_offsets.size() - 1; }
    void view(mte_batch* b) const {
        b->n_docs = n_docs();
        b->doc_op_offsets = doc_op_offsets.data();
        b->ops = ops.data();
        b->doc_payload_offsets = doc_payload_offsets.data();
        b->payload = payload.data();
        b->n_propsets = (uint32_t)propsets.size();
        b->propsets = propsets.data();
        b->prop_keys = prop_keys.data();
        b->prop_vals = prop_vals.data();
        b->n_keys = (uint32_t)key_offsets.size() - 1;
        b->key_offsets = key_offsets.data();
        b->key_text = key_text.data();
        b->n_vals = (uint32_t)val_offsets.size() - 1;
        b->val_offsets = val_offsets.data();
        b->val_text = val_text.data();
        b->doc_client_offsets = doc_client_offsets.data();
        b->client_name_offsets = client_name_offsets.data();
        b->client_names = client_names.data();
        const bool msgs = doc_msg_offsets.size() == (size_t)n_docs() + 1;  // generated batches keep none
        b->doc_msg_offsets = msgs ? doc_msg_offsets.data() : nullptr;
        b->msg_first_op = msgs ? msg_first_op.data() : nullptr;
        b->msg_text_offsets = msgs ? msg_text_offsets.data() : nullptr;
        b->msg_text = msgs ? msg_text.data() : nullptr;
    }
    // with_ops = false: everything but the op records and the payload (mte_load uploads those straight
    // from the caller's buffers; ensure_host_ops reads them back if a host walker ever needs them)
    void copy_from(const mte_batch* b, bool with_ops = true) {
        const uint32_t n = b->n_docs;
        doc_op_offsets.assign(b->doc_op_offsets, b->doc_op_offsets + n + 1);
        doc_payload_offsets.assign(b->doc_payload_offsets, b->doc_payload_offsets + n + 1);
        if (with_ops) {
            ops.assign(b->ops, b->ops + doc_op_offsets[n]);
            payload.assign(b->payload, b->payload + doc_payload_offsets[n]);
        } else {
            std::vector<mte_op>().swap(ops);
            std::vector<uint16_t>().swap(payload);
        }
        propsets.assign(b->propsets, b->propsets + b->n_propsets);
        size_t nkv = 0;
        for (auto& ps : propsets) nkv = std::max<size_t>(nkv, (size_t)ps.first + ps.count);
        prop_keys.assign(b->prop_keys, b->prop_keys + nkv);
        prop_vals.assign(b->prop_vals, b->prop_vals + nkv);
        key_offsets.assign(b->key_offsets, b->key_offsets + b->n_keys + 1);
        key_text.assign(b->key_text, b->key_offsets[b->n_keys]);
        val_offsets.assign(b->val_offsets, b->val_offsets + b->n_vals + 1);
        val_text.assign(b->val_text, b->val_offsets[b->n_vals]);
        doc_client_offsets.assign(b->doc_client_offsets, b->doc_client_offsets + n + 1);
        uint32_t nn = doc_client_offsets[n];
        client_name_offsets.assign(b->client_name_offsets, b->client_name_offsets + nn + 1);
        client_names.assign(b->client_names, b->client_name_offsets[nn]);
        if (b->doc_msg_offsets && b->msg_first_op && b->msg_text_offsets && b->msg_text) {
            doc_msg_offsets.assign(b->doc_msg_offsets, b->doc_msg_offsets + n + 1);
            const uint64_t nm = doc_msg_offsets[n];
            msg_first_op.assign(b->msg_first_op, b->msg_first_op + nm);
            msg_text_offsets.assign(b->msg_text_offsets, b->msg_text_offsets + nm + 1);
            msg_text.assign(b->msg_text, b->msg_text_offsets[nm]);
        } else {
            doc_msg_offsets.assign(n + 1, 0);
            msg_first_op.clear();
            msg_text_offsets.assign(1, 0);
            msg_text.clear();
        }
    }
    std::string message(uint64_t i) const {
        return msg_text.substr(msg_text_offsets[i], msg_text_offsets[i + 1] - msg_text_offsets[i]);
    }
    std::string key(uint32_t k) const { return key_text.substr(key_offsets[k], key_offsets[k + 1] - key_offsets[k]); }
    std::string val(uint32_t v) const { return val_text.substr(val_offsets[v], val_offsets[v + 1] - val_offsets[v]); }
    std::string client(uint32_t doc, uint32_t shortId) const {
        uint32_t i = doc_client_offsets[doc] + shortId;
        if (i >= doc_client_offsets[doc + 1]) return std::string();
        return client_names.substr(client_name_offsets[i], client_name_offsets[i + 1] - client_name_offsets[i]);
    }
};

// Interning tables shared by the builder and the generator.
struct Interner {
    HostBatch* hb;
    std::unordered_map<std::string, uint32_t> keys, vals;
    std::map<std::vector<uint32_t>, uint32_t> sets;
    explicit Interner(HostBatch* h) : hb(h) {
        if (hb->val_offsets.size() == 1) {  // value id 0 == JSON null (a delete in annotate)
            hb->val_text = "null";
            hb->val_offsets.push_back(4);
        }
        vals["null"] = 0;
    }
    uint32_t key(const std::u16string& k) {
        std::string q;
        json::quote(q, k);
        auto it = keys.find(q);
        if (it != keys.end()) return it->second;
        uint32_t id = (uint32_t)hb->key_offsets.size() - 1;
        hb->key_text += q;
        hb->key_offsets.push_back(hb->key_text.size());
        keys[q] = id;
        return id;
    }
    uint32_t val(const std::string& canonical) {
        auto it = vals.find(canonical);
        if (it != vals.end()) return it->second;
        uint32_t id = (uint32_t)hb->val_offsets.size() - 1;
        hb->val_text += canonical;
        hb->val_offsets.push_back(hb->val_text.size());
        vals[canonical] = id;
        return id;
    }
    // A props object in Object.keys order (properties are applied key by key in that order,
    // segmentPropertiesManager.ts:81-106).
    uint32_t propset(const json::Value& obj) {
        std::vector<uint32_t> kv;
        for (size_t i : json::key_order(obj)) {
            kv.push_back(key(obj.members[i].first));
            kv.push_back(val(json::stringify(obj.members[i].second)));
        }
        return intern_kv(kv);
    }
    uint32_t intern_kv(const std::vector<uint32_t>& kv) {
        auto it = sets.find(kv);
        if (it != sets.end()) return it->second;
        uint32_t id = (uint32_t)hb->propsets.size();
        mte_propset ps{(uint32_t)hb->prop_keys.size(), (uint32_t)(kv.size() / 2)};
        for (size_t i = 0; i < kv.size(); i += 2) {
            hb->prop_keys.push_back(kv[i]);
            hb->prop_vals.push_back(kv[i + 1]);
        }
        hb->propsets.push_back(ps);
        sets[kv] = id;
        return id;
    }
};

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t count) {
        release();
        n = count;
        if (count == 0) count = 1;
        return hipMalloc((void**)&p, count * sizeof(T));
    }
    // keep a buffer that is large enough: a later mte_load of a batch no larger than the last one
    // allocates nothing (hipFree + hipMalloc of the multi-GB tables took 2.7-3.0 s on some loads,
    // profiles/pcie_r03m_c4.json)
    hipError_t fit(size_t count) { return (p && n >= count) ? hipSuccess : alloc(count); }
};

}  // namespace

struct DocBuild;
struct mte_builder {
    HostBatch hb;
    std::unique_ptr<Interner> in;
    std::string err;
    std::vector<std::string> paths;  // per document: channel full path (container logs), else ""
    uint32_t n_cells = 0;            // SharedMatrix cell ops so far (MTE_OP_CELL's cell index)
    // open documents (mte_builder_open_doc): logs still growing, after every committed document;
    // mte_builder_batch commits copies of them into `view`
    std::vector<std::unique_ptr<DocBuild>> open;
    HostBatch view;
    mte_builder() { in.reset(new Interner(&hb)); }
    ~mte_builder();
};

struct mte_engine {
    int device = 0;
    uint32_t chunk = 10000;
    hipStream_t stream = nullptr, stream2 = nullptr;  // stream2: the HBM-resident waves (k_hbmq)
    hipStream_t stream3 = nullptr;                    // stream3: the solo workgroups (k_solo)
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
    hipEvent_t ev_s0 = nullptr, ev_s1 = nullptr;  // timing of the solo workgroups (critical path)
    hipEvent_t ev_gate = nullptr;                 // after k_solo_gate: the second bulk stream starts here
    // pinned staging for uploads from the caller's (pageable) buffers: two chunks, each refilled by
    // host threads while the DMA engine copies the other one (upload_staged)
    void* stage[2] = {nullptr, nullptr};
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    std::string err;
    HostBatch hb;
    bool generated = false;    // ops/payload live on the device; host copy filled on demand
    bool host_ops_valid = false;
    uint32_t gen_kind = 0;
    // derived per-value data (matchProperties, rewrite truthiness)
    std::vector<uint32_t> val_flags, val_objidx;
    std::vector<uint64_t> val_objmatch;
    std::vector<uint8_t> key_is_index;
    std::vector<uint32_t> key_index;
    // layout
    std::vector<DocCfg> cfg;
    std::vector<uint32_t> order;
    std::vector<DocRes> res;
    Params P{};
    bool replayed = false;
    bool downloaded = false;
    double last_kernel_ms = 0, last_h2d_ms = 0;
    // device buffers
    DevBuf<mte_op> d_ops;
    DevBuf<uint16_t> d_payload, d_arena, d_out_text;
    DevBuf<mte_propset> d_propsets;
    DevBuf<uint32_t> d_out_maps, d_prop_keys, d_prop_vals, d_val_flags, d_val_objidx, d_order, d_list, d_maps, d_counters,
        d_first_seen;
    DevBuf<uint64_t> d_val_objmatch, d_ovl, d_out_ovl, d_prof, d_solo_clk;
    DevBuf<uint64_t> d_ovl2, d_out_ovl2;  // removedClientOverlap of clients 64..127 (wide windows only)
    DevBuf<uint32_t> d_solo_started;  // k_solo_gate's counter
    DevBuf<uint32_t> d_rows_retry;    // k_rows' restart queue (Params::rows_retry)
    DevBuf<uint32_t> d_rows_cont;     // k_rows' continuation records (Params::rows_cont), one per slot
    bool solo_gate = true;            // option "solo_gate"
    uint64_t last_solo_cycles = 0, last_solo_ref = 0;  // critical wave: s_memtime / s_memrealtime deltas
    double last_cell_pass_ms = 0;                       // a SharedMatrix batch's first (positions) pass
    int64_t last_solo_start_delay = 0;                  // critical wave's start - the bulk's (100 MHz ticks)
    // property maps of the documents the host re-ran (their worst-case table), by document
    DevBuf<uint32_t> d_maps_rr;
    std::vector<uint64_t> map_rr_off;  // UINT64_MAX = the document's maps are in d_maps
    std::vector<uint32_t> map_rr_cap;
    DevBuf<DocCfg> d_cfg;
    DevBuf<DocRes> d_res;
    DevBuf<uint4> d_out_vis, d_out_aux;
    DevBuf<uint32_t> d_out_esc;  // per output row: the emission word (engine_types.hpp ESC_*)
    DevBuf<unsigned char> d_hbm, d_spill, d_solo_spill;
    DevBuf<uint32_t> d_slot_bits;
    std::vector<uint64_t> n_ops_doc;
    // options (mte_set_option)
    bool force_hbm = false;           // no LDS-resident waves: every document HBM-resident
    uint32_t pool_limit = 0;
    uint32_t reg_solo = 1;               // option "reg_solo": k_solo's register-resident engine (lean batches)
    uint32_t reg_lb_limit = 0;           // option "reg_lb_limit": test knob, leaf blocks the register plan holds
    uint32_t map_words = MAP_WORDS;      // property-map record width of the loaded batch (Params::map_words)
#ifndef MTE_HBMQ_PER_CU
#define MTE_HBMQ_PER_CU 8
#endif
    uint32_t hbm_waves_per_cu = MTE_HBMQ_PER_CU;  // HBM-resident waves (slots) per CU beside the LDS workgroup
    bool hbm_waves_set = false;          // ... set by mte_set_option (else wave_plan may drop them)
    uint64_t slot_budget = 48ull << 30;  // HBM for per-wave slots
    uint64_t slot_ops_cap = 65536;       // slots are sized for documents of at most this many ops
    uint32_t slot_blk_limit = 0;         // test knob: leaf blocks per slot (0 = from slot_ops_cap)
    // critical-path documents replayed by k_solo (a whole CU's LDS for one wave each)
    bool lean_ok = false;                // batch_is_lean: the replay may run the FULL = false kernels
    bool ext_needed = false;             // catch-up records or permutation runs: the EXT kernels (level 2)
    bool ext_perm = false;               // the loaded batch has permutation runs (always EXT)
    // SharedMatrix cell ops (MTE_OP_CELL): two passes (engine_types.hpp Params::cell_mode); per doc
    // with cell records, the records' (cell index, seq, value id) for the cells blob
    struct CellRec {
        uint32_t cell;
        int32_t seq;
        uint32_t val;
    };
    std::unordered_map<uint32_t, std::vector<CellRec>> cell_recs;
    // a SharedMatrix loaded from a summary (MTE_F_MX_* records of its rows document): the loaded
    // cells (row handle, col handle, value id), tiles (key hi, depth, low-key prefix) and root extent
    struct MxInit {
        std::vector<std::array<uint32_t, 3>> cells, tiles;
        uint32_t root_len = 1;
    };
    std::unordered_map<uint32_t, MxInit> mx_init;
    uint64_t n_cells = 0;                // cell indices 0 .. n_cells - 1
    DevBuf<uint32_t> d_cell_pos, d_cell_h, d_htab, d_htab0;  // HandleTables, and their state at document start
    bool ext_cu = false;                 // ... MTE_F_CATCHUP ops: EXT only when a legacy summary is emitted
    bool lean_base = false;              // batch_is_lean, before the catch-up records decide
    uint32_t rows_pool_lim = 0;          // option rows_pool: k_rows pool rows per CU (test knob, 0 = all)
    bool props_rows_ok = false;          // k_rows may take the batch: no '\n', relative positions, summary loads or local documents
    std::vector<uint8_t> doc_not_rows;   // per document: the row engines cannot replay it (hands over at op 0)
    int rows_mixed = 1;                  // option "rows_mixed": a batch with a few such documents still runs its
                                         // bulk on k_rows (4 waves), those continuing HBM-resident from op 0:
                                         // 1 on retained passes, 2 always, 0 never
    bool rows_wide = false;              // ... on its WIDE row engine: a document has writers 32..63
    bool lean_opt = true;                // option "lean" (0 = always the FULL kernels)
    bool last_lean = false;
    uint32_t solo_max = 16;              // at most this many (0 = off)
    uint64_t solo_min_ops = 20000;       // ... each at least this long
    uint32_t solo_div = 6;               // ... and at least 1/solo_div of the longest document
    uint64_t doc_id_base = 0;            // global id of a loaded batch's document 0 (summary records)
    // per-wave slot plan (layout_and_alloc)
    uint32_t n_slots = 0;
    // last run
    double last_lds_ms = 0, last_hbm_ms = 0;
    uint32_t last_spilled = 0, last_continued = 0, last_hbm_docs = 0, last_hbm_waves = 0, last_lds_groups = 0;
    uint32_t last_solo = 0;
    double last_solo_ms = 0;
    double last_alloc_ms = 0;  // mte_load: device layout and allocation (inside h2d_ms)
    double stage_copy_ms = 0, stage_wait_ms = 0;  // mte_load: host memcpy into / DMA waits on the stage
    double last_solo_lead_ms = 0, last_solo_tail_ms = 0;  // pass start -> solo start, solo end -> pass end
    uint32_t n_groups = 256;
    // SnapshotV1 emission on the device (emit.hip): property / name tables, scratch, and two output
    // pools -- round 0 (every document but the solo ones) runs while the critical path is still
    // replaying, round 1 (solo and host-re-run documents) after it
    int32_t rows_bulk = -1;   // option "rows_bulk": lean replays run the bulk on k_rows, 4, 8 or 12 waves per
                              // CU; -1 (auto: 4 for long documents, 12 without solo documents), 0: never
    bool xcd_align = true;    // option "xcd_align": bulk grids leave solo CUs free in every XCD (bulk_cus)
    uint32_t last_rows = 0;   // waves per CU of the last pass's k_rows (0: k_lds / k_hbmq)
    bool last_mixed = false;  // the last pass ran a mixed batch on k_rows (rows_mixed)
    bool emit_opt = true;     // option "emit"
    bool legacy = false;      // snapshot_format 1 (mte_config / option "snapshot_format"): SnapshotLegacy
    bool emitted_legacy = false;  // format of the last emission
    DevBuf<uint4> d_cu;       // catch-up delta records (Params::cu_rec)
    bool emit_tables = false; // tables uploaded for the current batch
    DevBuf<char> d_key_text, d_val_text, d_names;
    DevBuf<uint64_t> d_key_off, d_val_off, d_name_off, d_name_base, d_emit_size, d_out_off, d_blob_base;
    DevBuf<unsigned char> d_key_is_index;
    DevBuf<uint32_t> d_key_index, d_n_ent, d_nblobs, d_emit_list[2];
    DevBuf<uint4> d_ent;
    DevBuf<uint16_t> d_tscr;
    struct EmitPool {
        DevBuf<char> out;
        DevBuf<uint64_t> blob_off;
        uint64_t used = 0, blobs = 0;
        std::vector<char> h;
        std::vector<uint64_t> h_blob_off;
    } pool[2];
    std::vector<uint64_t> h_emit_size, h_out_off, h_blob_base;
    std::vector<uint32_t> h_nblobs;
    std::vector<uint8_t> emit_pool_of;  // per document: its pool, 255 = not emitted (failed / emission off)
    bool emit_downloaded = false;
    double last_emit_ms = 0;
    // incremental replay (option "retain"; reg_engine.hpp ckpt_save / ckpt_resume): the row engines
    // leave every finished document's state in a checkpoint region; a pass over a batch whose logs
    // extend the last pass's (ck_match) continues each such document from its checkpoint
    bool retain = false;
    DevBuf<uint32_t> d_ck[2];
    int ck_cur = -1;  // the buffer with the last pass's checkpoints (-1: none)
    struct CkDoc {
        uint64_t n_ops = 0, n_pay = 0, off = 0, h_ops = 0, h_pay = 0;
    };
    std::vector<CkDoc> ck_prev;        // per document of the last pass: what its checkpoint covers, and where
    std::vector<CkDoc> ck_load;        // per document of the loaded batch: its whole log's hashes
    std::vector<uint64_t> ck_match;    // per document of the loaded batch: op records it shares with ck_prev
    HostBatch ck_tabs;                 // the last pass's property tables (ids must keep their meaning)
    uint64_t ck_tabs_n = 0;            // their key / value / propset counts, 0 = none kept
    uint32_t ck_map_words = 0;
    uint32_t last_resumed_docs = 0, last_resumed_ops = 0, last_ck_offered = 0;
    // downloaded final state
    std::vector<uint32_t> h_maps;
    std::vector<uint4> h_out_vis, h_out_aux;
    std::vector<uint64_t> h_out_ovl, h_out_ovl2;
    std::vector<uint16_t> h_out_text;
};

static int set_err(mte_engine* e, int code, const std::string& m) {
    if (e) e->err = m;
    return code;
}
#define HIP_TRY(e, x)                                                                     \
    do {                                                                                  \
        hipError_t _r = (x);                                                              \
        if (_r != hipSuccess) return set_err(e, MTE_E_HIP, std::string(#x ": ") + hipGetErrorString(_r)); \
    } while (0)

// ------------------------------------------------------------------------------------------------
// Value / key metadata for the device: JS falsiness (rewrite), object-typed values and the
// matchProperties relation against object-typed values (properties.ts:62-93).
static int derive_value_tables(mte_engine* e) {
    const HostBatch& hb = e->hb;
    uint32_t nv = (uint32_t)hb.val_offsets.size() - 1;
    std::vector<json::Value> vals(nv);
    for (uint32_t v = 0; v < nv; v++) {
        std::string t = hb.val(v);
        try {
            vals[v] = json::parse(t.data(), t.size());
        } catch (std::exception& ex) {
            return set_err(e, MTE_E_PARSE, ex.what());
        }
    }
    e->val_flags.assign(nv, 0);
    e->val_objidx.assign(nv, NONE);
    e->val_objmatch.assign(nv, 0);
    std::vector<uint32_t> objs;
    for (uint32_t v = 0; v < nv; v++) {
        if (!json::truthy(&vals[v])) e->val_flags[v] |= 1u;
        if (json::is_object_typed(&vals[v]) && v != 0) {
            e->val_flags[v] |= 2u;
            if (objs.size() < 64) {
                e->val_objidx[v] = (uint32_t)objs.size();
                objs.push_back(v);
            }
        }
    }
    for (uint32_t v = 0; v < nv; v++)
        for (size_t j = 0; j < objs.size(); j++)
            if (json::match_properties(&vals[v], &vals[objs[j]])) e->val_objmatch[v] |= 1ull << j;
    uint32_t nk = (uint32_t)hb.key_offsets.size() - 1;
    e->key_is_index.assign(nk, 0);
    e->key_index.assign(nk, 0);
    for (uint32_t k = 0; k < nk; k++) {
        std::string t = hb.key(k);
        json::Value kv = json::parse(t.data(), t.size());
        uint32_t idx;
        if (json::array_index(kv.str, &idx)) {
            e->key_is_index[k] = 1;
            e->key_index[k] = idx;
        }
    }
    return MTE_OK;
}

template <class F>
static void run_pool(unsigned n, F&& work);

// Host -> device copy of a large caller buffer through two pinned chunks: host threads copy chunk i+1
// out of the (pageable) source while the DMA engine moves chunk i. A pageable hipMemcpyAsync stages
// through the runtime's own buffers and ran at 3.6 GB/s on the first C4-sized load
// (profiles/pcie_r02l_c4.json); this path does not depend on what the runtime has pinned before.
static constexpr size_t STAGE_BYTES = 64ull << 20;
static int upload_staged(mte_engine* e, void* dst, const void* src, size_t bytes) {
    if (bytes < (4ull << 20)) {  // small: the runtime's path is fine
        HIP_TRY(e, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream));
        return MTE_OK;
    }
    for (int i = 0; i < 2; i++) {
        if (!e->stage[i]) HIP_TRY(e, hipHostMalloc(&e->stage[i], STAGE_BYTES, hipHostMallocDefault));
        if (!e->ev_stage[i]) HIP_TRY(e, hipEventCreateWithFlags(&e->ev_stage[i], hipEventDisableTiming));
    }
    const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    int k = 0;
    for (size_t off = 0; off < bytes; off += STAGE_BYTES, k ^= 1) {
        const size_t n = std::min(STAGE_BYTES, bytes - off);
        auto t0 = std::chrono::steady_clock::now();
        HIP_TRY(e, hipEventSynchronize(e->ev_stage[k]));  // the DMA out of this chunk is done
        auto t1 = std::chrono::steady_clock::now();
        char* stg = (char*)e->stage[k];
        const char* from = (const char*)src + off;
        const size_t piece = (n + nt - 1) / nt;
        std::atomic<unsigned> next{0};
        run_pool(nt, [&]() {
            for (unsigned t; (t = next.fetch_add(1)) < nt;) {
                const size_t a = (size_t)t * piece;
                if (a < n) memcpy(stg + a, from + a, std::min(piece, n - a));
            }
        });
        auto t2 = std::chrono::steady_clock::now();
        e->stage_wait_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
        e->stage_copy_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
        HIP_TRY(e, hipMemcpyAsync((char*)dst + off, stg, n, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(e, hipEventRecord(e->ev_stage[k], e->stream));
    }
    return MTE_OK;
}

template <class T>
static int upload(mte_engine* e, DevBuf<T>& d, const T* h, size_t n) {
    HIP_TRY(e, d.fit(n));
    if (n) return upload_staged(e, d.p, h, n * sizeof(T));
    return MTE_OK;
}
template <class T>
static int upload(mte_engine* e, DevBuf<T>& d, const std::vector<T>& h) {
    return upload(e, d, h.data(), h.size());
}

static int alloc_slots(mte_engine* e);

// Per-document arena sizing (see DESIGN.md "HBM layout").
static int layout_and_alloc(mte_engine* e, const std::vector<uint64_t>& n_ops, const std::vector<uint64_t>& pay_len,
                            const std::vector<uint64_t>& n_prop_ins, const std::vector<uint64_t>& n_ann,
                            const std::vector<uint8_t>& collab, const std::vector<uint8_t>& has_nl,
                            uint64_t arena_limit = 0, const uint64_t* op_offsets = nullptr,
                            const uint64_t* payload_offsets = nullptr, const uint32_t* doc_ids = nullptr) {
    const uint32_t nd = (uint32_t)n_ops.size();
    e->cfg.assign(nd, DocCfg{});
    e->n_ops_doc = n_ops;
    uint64_t op = 0, pay = 0, ar = 0, seg = 0, seg2 = 0, mp = 0, out = 0;
    bool any_props = false;
    for (uint32_t d = 0; d < nd; d++) {
        DocCfg& c = e->cfg[d];
        uint64_t n = n_ops[d];
        // a loaded batch's documents need not start at op / payload 0 (mte_batch offsets are absolute)
        c.op_begin = op_offsets ? op_offsets[d] : op;
        c.op_end = c.op_begin + n;
        op += n;
        c.payload_off = payload_offsets ? payload_offsets[d] : pay;
        c.payload_len = (uint32_t)pay_len[d];
        pay += pay_len[d];
        // merge arena semispace: live arena text <= 2x live text, a scour needs <= 4x a block's text
        uint64_t acap = 6 * pay_len[d] + 4096;
        if (arena_limit) acap = std::min<uint64_t>(acap, arena_limit);
        c.arena_cap = (uint32_t)std::min<uint64_t>(acap, 0x7FFFFFF0ull / 2);
        c.arena_off = ar;
        ar += 2ull * c.arena_cap;
        c.seg_cap = (uint32_t)std::min<uint64_t>(3 * n + 8, 0xFFFFFFF0ull);
        c.ovl_off = seg;
        seg += c.seg_cap;
        // a window of more than 64 clients (a loaded batch's names; the generator's stay below 64):
        // removedClientOverlap of clients 64..127 in a second per-segment word
        const auto& dco = e->hb.doc_client_offsets;
        c.ovl2_off = OVL2_NONE;
        if (dco.size() > d + 1 && dco[d + 1] - dco[d] > 64) {
            c.ovl2_off = seg2;
            seg2 += c.seg_cap;
        }
        c.map_cap = (uint32_t)(n_prop_ins[d] + 4 * n_ann[d] + 16);
        c.map_off = mp;
        mp += c.map_cap;
        any_props |= n_prop_ins[d] + n_ann[d] > 0;
        c.collab = collab[d];
        c.has_nl = has_nl[d];
        c.prio = 0;
        c.gid = doc_ids ? doc_ids[d] : (uint32_t)(e->doc_id_base + d);
        out += std::min<uint64_t>(3 * n + 8, 4096);
    }
    out += 1u << 20;
    // critical-path documents (Zipf heads): at least 8x the mean op count
    if (nd > 1) {
        const double mean = (double)op / nd;
        for (uint32_t d = 0; d < nd; d++)
            if ((double)n_ops[d] >= 8.0 * mean) e->cfg[d].prio = 1;
    }
    HIP_TRY(e, e->d_arena.fit(ar));
    HIP_TRY(e, e->d_ovl.fit(seg));
    if (seg2) HIP_TRY(e, e->d_ovl2.fit(seg2));
    HIP_TRY(e, e->d_maps.fit(mp * e->map_words));
    HIP_TRY(e, e->d_out_vis.fit(out));
    HIP_TRY(e, e->d_out_esc.fit(out));
    HIP_TRY(e, e->d_out_aux.fit(out));
    HIP_TRY(e, e->d_out_ovl.fit(out));
    if (seg2) HIP_TRY(e, e->d_out_ovl2.fit(out));
    if (any_props) HIP_TRY(e, e->d_out_maps.fit(out * e->map_words));  // some document can carry props
    HIP_TRY(e, e->d_counters.fit(16));
    HIP_TRY(e, e->d_rows_retry.fit(nd));
    HIP_TRY(e, e->d_res.fit(nd));
    HIP_TRY(e, e->d_prof.fit((size_t)nd * PROF_SLOTS));
    HIP_TRY(e, hipMemsetAsync(e->d_prof.p, 0, (size_t)nd * PROF_SLOTS * 8, e->stream));
    HIP_TRY(e, e->d_solo_clk.fit(4 * SOLO_CLK_SLOTS + 1));  // 4 u64 per solo workgroup + the bulk's start
    HIP_TRY(e, e->d_solo_started.fit(1));
    // LPT order: longest documents start first
    e->order.resize(nd);
    for (uint32_t d = 0; d < nd; d++) e->order[d] = d;
    std::stable_sort(e->order.begin(), e->order.end(), [&](uint32_t a, uint32_t b) { return n_ops[a] > n_ops[b]; });
    int rc;
    if ((rc = upload(e, e->d_cfg, e->cfg))) return rc;
    if ((rc = upload(e, e->d_order, e->order))) return rc;
    Params& P = e->P;
    P = Params{};
    P.n_docs = nd;
    P.docs = e->d_cfg.p;
    P.doc_list = e->d_order.p;
    P.n_list = nd;
    P.res = e->d_res.p;
    P.arena = e->d_arena.p;
    P.ovl = e->d_ovl.p;
    P.ovl2 = seg2 ? e->d_ovl2.p : nullptr;
    P.out_ovl2 = seg2 ? e->d_out_ovl2.p : nullptr;
    P.maps = e->d_maps.p;
    P.map_words = e->map_words;
    P.out_vis = e->d_out_vis.p;
    P.out_aux = e->d_out_aux.p;
    P.out_ovl = e->d_out_ovl.p;
    P.out_cap = out;
    P.out_maps = any_props ? e->d_out_maps.p : nullptr;
    P.counters = e->d_counters.p;
    P.prof = e->d_prof.p;
    P.solo_clk = e->d_solo_clk.p;
    P.solo_started = e->d_solo_started.p;
    P.rows_retry = e->d_rows_retry.p;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->device) != hipSuccess || cus <= 0) cus = 256;
    e->n_groups = (uint32_t)cus;
    // per-wave HBM slots, each sized for the longest document up to slot_ops_cap ops (hbm_caps);
    // a longer document that outgrows its slot is re-run by the host with worst-case capacities
    uint64_t nmax = 0;
    for (uint32_t d = 0; d < nd; d++) nmax = std::max<uint64_t>(nmax, n_ops[d]);
    hbm_caps(std::min<uint64_t>(nmax, e->slot_ops_cap), P.slot_blk, P.slot_ord, P.slot_in, P.slot_heap);
    if (e->slot_blk_limit) {  // test knob: slots that overflow (documents re-run by the host)
        P.slot_blk = std::min(P.slot_blk, e->slot_blk_limit);
        P.slot_ord = std::min(P.slot_ord, e->slot_blk_limit);
    }
    P.slot_bytes = (HbmLayout::of(P.slot_blk, P.slot_ord, P.slot_in, P.slot_heap).bytes + 255) & ~255ull;
    return alloc_slots(e);
}

// Wave plan of a replay: G LDS workgroups (LDS_WAVES waves each, one per CU) plus up to H
// HBM-resident waves at a time (k_hbmq, one document per wave, H slots), or HBM-resident waves
// alone when the LDS plan is off or the slots for its waves do not fit the budget. Every LDS wave
// owns a slot for a document that outgrows the plan.
// CUs left to the bulk beside n_solo solo workgroups. Workgroups are handed to the 8 XCDs in turn,
// so a grid that is not a multiple of 8 fills some XCDs' CUs completely: a solo workgroup dispatched
// to such an XCD waits for a bulk workgroup to finish -- a whole bulk pass, ~1.1 s, on every other
// C4 step (the critical wave's own cycles and clock were the same in slow and fast steps, BENCH_r03
// and profiles/r04_c4_steps.json). Leaving ceil(n_solo / 8) CUs free in EVERY XCD keeps each one's
// share of the bulk at most its CUs minus its solo workgroups, whatever XCD the first one lands on.
static uint32_t bulk_cus(const mte_engine* e, uint32_t n_solo) {
    constexpr uint32_t XCDS = 8;  // MI355X (gfx950)
    const uint32_t keep = !e->xcd_align ? n_solo : n_solo ? XCDS * ((n_solo + XCDS - 1) / XCDS) : 0u;
    return e->n_groups > keep ? e->n_groups - keep : 1u;
}

static void wave_plan(const mte_engine* e, uint32_t nd, uint32_t& groups, uint32_t& hbm_waves,
                      uint32_t* lds_active = nullptr, uint32_t n_solo = 0) {
    const uint32_t cus = bulk_cus(e, n_solo);  // k_solo holds n_solo CUs
    nd -= std::min(nd, n_solo);
    const uint64_t max_slots = std::max<uint64_t>(1, e->slot_budget / std::max<uint64_t>(e->P.slot_bytes, 1));
    // fewer documents than LDS waves: every CU still gets a workgroup, with fewer active waves
    // (each with its own SIMD and a larger share of the CU's block pool)
    groups = std::min<uint32_t>(cus, nd);
    if (e->force_hbm || (uint64_t)groups * LDS_WAVES > max_slots) groups = 0;
    if (lds_active) *lds_active = groups ? std::min<uint32_t>(LDS_WAVES, (nd + groups - 1) / groups) : 0;
    // 16 = 4 SIMDs x 4 waves at <= 128 VGPRs (k_hbmq's bound): more can never be resident at once
    uint32_t per_cu = groups ? std::min<uint32_t>(e->hbm_waves_per_cu, 16) : 16;
    // A batch bounded by its critical-path documents: the HBM-resident waves' memory traffic slows
    // the solo waves (C4: steps of 4.0-4.77 s with them, 4.00-4.08 s without, profiles/r03hw_*.json),
    // so the bulk runs LDS-resident only when it still finishes inside the longest document's replay
    // (estimates: >= 120 M ops/s for the LDS-only bulk -- C2 163 M, C3 187 M, tools/sweep.py hw 0 --
    // and ~4 us/op on the critical path).
    if (groups && n_solo && !e->hbm_waves_set && !e->order.empty()) {
        uint64_t nmax = 0, bulk = 0;
        for (uint32_t k = 0; k < (uint32_t)e->order.size(); k++) {
            const uint64_t n = e->n_ops_doc[e->order[k]];
            if (k < n_solo) nmax = std::max(nmax, n);
            else bulk += n;
        }
        if ((double)nmax * 4.0e-6 > 1.1 * (double)bulk / 120.0e6) per_cu = 0;
    }
    uint64_t h = (uint64_t)per_cu * cus;
    h = std::min<uint64_t>(h, max_slots - (uint64_t)groups * LDS_WAVES);
    if (nd > (uint64_t)groups * LDS_WAVES) h = std::min<uint64_t>(h, nd - (uint64_t)groups * LDS_WAVES);
    else h = 0;
    if (groups == 0 && h == 0 && nd) h = 1;
    hbm_waves = (uint32_t)h;
}

// Output text pool: a document's final text never exceeds the text its log inserted, so the
// payload's size bounds the whole batch (Engine::finish gathers into it).
static int alloc_out_text(mte_engine* e) {
    const uint64_t pay = e->hb.doc_payload_offsets.empty() ? 0 : e->hb.doc_payload_offsets.back();
    const uint64_t n = std::max<uint64_t>(1, std::min<uint64_t>(pay, 0xFFFFFFFFull));
    if (n > e->d_out_text.n || !e->d_out_text.p) HIP_TRY(e, e->d_out_text.alloc(n));
    e->P.out_text = e->d_out_text.p;
    e->P.out_text_cap = n;
    return MTE_OK;
}

// Critical-path documents for k_solo: the leading documents of the LPT order that are far longer
// than the batch mean (or the only document) and within 1/solo_div of the longest one.
static uint32_t solo_count(const mte_engine* e) {
    const uint32_t nd = (uint32_t)e->order.size();
    if (!nd || !e->solo_max || e->force_hbm) return 0;
    uint64_t total = 0, nmax = 0;
    for (uint64_t n : e->n_ops_doc) {
        total += n;
        nmax = std::max(nmax, n);
    }
    const double mean = (double)total / nd;
    const uint32_t cap = std::min<uint32_t>(e->solo_max, std::max<uint32_t>(1, e->n_groups / 8));
    uint32_t k = 0;
    while (k < nd && k < cap) {
        const uint64_t n = e->n_ops_doc[e->order[k]];
        if (n < e->solo_min_ops || n * e->solo_div < nmax || (nd > 1 && (double)n < 8.0 * mean)) break;
        if (e->cell_recs.count(e->order[k])) break;  // cell ops run in the LDS / HBM engines only
        k++;
    }
    return k;
}

static int alloc_slots(mte_engine* e) {
    uint32_t g, h;
    const uint32_t ns = solo_count(e);
    wave_plan(e, e->P.n_docs, g, h, nullptr, ns);
    const uint32_t n = g * LDS_WAVES + h;
    const size_t bytes = (size_t)n * e->P.slot_bytes;
    if (bytes > e->d_spill.n || !e->d_spill.p) HIP_TRY(e, e->d_spill.alloc(bytes));
    const size_t words = (n + 31) / 32 + 1;  // (k_rows may claim any of the n slots: rows_continue)
    if (words > e->d_slot_bits.n || !e->d_slot_bits.p) HIP_TRY(e, e->d_slot_bits.alloc(words));
    HIP_TRY(e, e->d_rows_cont.fit((size_t)std::max<uint32_t>(n, 1) * ROWS_CONT_WORDS));
    // (k_rows dumps a document's state into its slot before k_rows_cont converts it in place)
    e->P.rows_cont = e->P.slot_bytes >= ROWS_DUMP_BYTES ? e->d_rows_cont.p : nullptr;
    e->n_slots = n;
    e->P.spill = e->d_spill.p;
    e->P.slot_bits = e->d_slot_bits.p;
    // solo documents continue in slots of their own, sized for the longest of them
    e->P.n_solo = ns;
    if (ns) {
        uint64_t nmax = 0;
        for (uint32_t k = 0; k < ns; k++) nmax = std::max(nmax, e->n_ops_doc[e->order[k]]);
        hbm_caps(nmax, e->P.solo_blk, e->P.solo_ord, e->P.solo_in, e->P.solo_heap);
        e->P.solo_slot_bytes =
            (HbmLayout::of(e->P.solo_blk, e->P.solo_ord, e->P.solo_in, e->P.solo_heap).bytes + 255) & ~255ull;
        const size_t sb = (size_t)ns * e->P.solo_slot_bytes;
        if (sb > e->d_solo_spill.n || !e->d_solo_spill.p) HIP_TRY(e, e->d_solo_spill.alloc(sb));
        e->P.solo_spill = e->d_solo_spill.p;
    }
    return MTE_OK;
}

static int upload_props(mte_engine* e) {
    int rc;
    if ((rc = derive_value_tables(e))) return rc;
    if ((rc = upload(e, e->d_propsets, e->hb.propsets))) return rc;
    if ((rc = upload(e, e->d_prop_keys, e->hb.prop_keys))) return rc;
    if ((rc = upload(e, e->d_prop_vals, e->hb.prop_vals))) return rc;
    if ((rc = upload(e, e->d_val_flags, e->val_flags))) return rc;
    if ((rc = upload(e, e->d_val_objidx, e->val_objidx))) return rc;
    if ((rc = upload(e, e->d_val_objmatch, e->val_objmatch))) return rc;
    e->P.propsets = e->d_propsets.p;
    e->P.prop_keys = e->d_prop_keys.p;
    e->P.prop_vals = e->d_prop_vals.p;
    e->P.val_flags = e->d_val_flags.p;
    e->P.val_objidx = e->d_val_objidx.p;
    e->P.val_objmatch = e->d_val_objmatch.p;
    e->P.n_propsets = (uint32_t)e->hb.propsets.size();
    e->P.n_vals = (uint32_t)e->val_flags.size();
    return MTE_OK;
}

// ------------------------------------------------------------------------------------------------
extern "C" {

int mte_abi_version(void) { return MTE_ABI_VERSION; }

const char* mte_build_info(void) {
    static std::string s = std::string("mte gfx950 hip ") + std::to_string(HIP_VERSION_MAJOR) + "." +
                           std::to_string(HIP_VERSION_MINOR);
    return s.c_str();
}

int mte_create(const mte_config* cfg, mte_engine** out) {
    if (!out) return MTE_E_ARG;
    *out = nullptr;
    std::unique_ptr<mte_engine> e(new mte_engine());
    if (cfg) {
        e->device = cfg->device;
        if (cfg->chunk_size) e->chunk = cfg->chunk_size;
        e->legacy = cfg->snapshot_format == 1;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= e->device) {
        // No CPU fallback: the replay path runs on the GPU only.
        static thread_local std::string why;
        why = "mte: no HIP device available (MI355X/gfx950 required)";
        return MTE_E_HIP;
    }
    HIP_TRY(e.get(), hipSetDevice(e->device));
    HIP_TRY(e.get(), hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    HIP_TRY(e.get(), hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking));
    HIP_TRY(e.get(), hipStreamCreateWithFlags(&e->stream3, hipStreamNonBlocking));
    HIP_TRY(e.get(), hipEventCreateWithFlags(&e->ev3, hipEventDisableTiming));
    HIP_TRY(e.get(), hipEventCreate(&e->ev_s0));
    HIP_TRY(e.get(), hipEventCreate(&e->ev_s1));
    HIP_TRY(e.get(), hipEventCreateWithFlags(&e->ev2, hipEventDisableTiming));
    HIP_TRY(e.get(), hipEventCreateWithFlags(&e->ev_gate, hipEventDisableTiming));
    HIP_TRY(e.get(), hipEventCreate(&e->ev0));
    HIP_TRY(e.get(), hipEventCreate(&e->ev1));
    *out = e.release();
    return MTE_OK;
}

void mte_destroy(mte_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (int i = 0; i < 2; i++) {
        if (e->stage[i]) (void)hipHostFree(e->stage[i]);
        if (e->ev_stage[i]) (void)hipEventDestroy(e->ev_stage[i]);
    }
    if (e->ev_gate) (void)hipEventDestroy(e->ev_gate);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->ev2) (void)hipEventDestroy(e->ev2);
    if (e->ev3) (void)hipEventDestroy(e->ev3);
    if (e->ev_s0) (void)hipEventDestroy(e->ev_s0);
    if (e->ev_s1) (void)hipEventDestroy(e->ev_s1);
    if (e->stream3) (void)hipStreamDestroy(e->stream3);
    if (e->stream2) (void)hipStreamDestroy(e->stream2);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

const char* mte_last_error(const mte_engine* e) { return e ? e->err.c_str() : "null engine"; }

static void count_doc_ops(const mte_op* ops, const uint64_t* off, uint32_t d, uint64_t& pi, uint64_t& an,
                          bool* rel = nullptr) {
    pi = an = 0;
    for (uint64_t i = off[d]; i < off[d + 1]; i++) {
        const mte_op& o = ops[i];
        if (rel && o.type == MTE_OP_RELPOS) *rel = true;  // FULL kernels only
        if ((o.type == MTE_OP_INSERT || o.type == MTE_OP_INSERT_MARKER || o.type == MTE_OP_LOAD_SEG ||
             o.type == MTE_OP_LOAD_APPEND) && o.props)
            pi++;
        if (o.type == MTE_OP_ANNOTATE) an++;
    }
}

// Runs `work` on up to n threads, the caller being one of them. `work` pulls from a shared queue, so a
// thread that cannot be created (std::system_error under RLIMIT_NPROC or a cgroup pids limit) only
// leaves its share to the others: the caller alone still finishes, and no exception crosses the C ABI.
extern "C++" {
template <class F>
static void run_pool(unsigned n, F&& work) {
    std::vector<std::thread> ts;
    try {
        for (unsigned i = 1; i < n; i++) ts.emplace_back(work);
    } catch (...) {
    }
    work();
    for (auto& t : ts) t.join();
}
}

// SharedMatrix cell records (include/mte.h MTE_OP_CELL): each vector document with some gets a
// HandleTable region (1 + 2 * (records + 2) words) and the batch two words per cell index for each
// pass's results; the records' cell / seq / value are kept for the cells blob (mte_snapshot_matrix).
static int load_cells(mte_engine* e, const mte_batch* b, const std::vector<uint32_t>& n_cell) {
    e->cell_recs.clear();
    e->mx_init.clear();
    e->n_cells = 0;
    uint64_t words = 0;
    std::vector<uint32_t> init;  // every region's state at document start (Params::htab0)
    bool any = false;
    for (uint32_t d = 0; d < b->n_docs; d++) {
        DocCfg& c = e->cfg[d];
        c.ht_cap = 0;
        c.ht_off = 0;
        // a loaded HandleTable (MX_HANDLE records) and cells (MX_CELL / MX_TILE)
        std::vector<uint32_t> h0;
        for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++) {
            const mte_op& o = b->ops[i];
            if (o.type != MTE_OP_NOOP || !(o.flags & MTE_F_MX_MASK)) continue;
            const uint32_t f = o.flags & MTE_F_MX_MASK;
            if (f == MTE_F_MX_HANDLE) {
                if (o.pos1 < 0 || o.pos1 > (1 << 26)) return set_err(e, MTE_E_RANGE, "loaded handle table too long");
                if (h0.size() <= (size_t)o.pos1) h0.resize((size_t)o.pos1 + 1, 0);
                h0[(size_t)o.pos1] = (uint32_t)o.a;
            } else if (f == MTE_F_MX_CELL) {
                e->mx_init[d].cells.push_back({(uint32_t)o.pos1, (uint32_t)o.a, o.props < b->n_vals ? o.props : 0u});
            } else if (o.b == 4) {
                e->mx_init[d].root_len = (uint32_t)o.pos1 + 1;
            } else {
                e->mx_init[d].tiles.push_back({(uint32_t)o.pos1, o.b, (uint32_t)o.a});
            }
        }
        if (!n_cell[d] && h0.empty()) continue;
        if (n_cell[d]) {
            std::vector<mte_engine::CellRec>& v = e->cell_recs[d];
            for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++) {
                const mte_op& o = b->ops[i];
                if (o.type != MTE_OP_CELL) continue;
                if (o.b >= (1u << 28)) return set_err(e, MTE_E_RANGE, "cell index beyond 2^28");
                v.push_back({o.b, o.seq, o.props < b->n_vals ? o.props : 0u});
                e->n_cells = std::max<uint64_t>(e->n_cells, (uint64_t)o.b + 1);
            }
        }
        if (h0.empty()) h0.push_back(1);  // new HandleTable(): [1]
        // every set allocates at most one handle per vector
        c.ht_cap = (uint32_t)h0.size() + n_cell[d] + 2;
        c.ht_off = words;
        words += 1 + 2 * (uint64_t)c.ht_cap;
        init.push_back((uint32_t)h0.size());
        init.insert(init.end(), h0.begin(), h0.end());
        init.resize(words, 0u);  // the rest of the handles, and no handle freed yet
        any = true;
    }
    e->P.cell_pos = e->P.cell_h = e->P.htab = nullptr;
    e->P.htab0 = nullptr;
    if (!any) return MTE_OK;
    if (e->d_htab.n < words) HIP_TRY(e, e->d_htab.alloc(words));
    if (e->d_htab0.n < words) HIP_TRY(e, e->d_htab0.alloc(words));
    HIP_TRY(e, hipMemcpyAsync(e->d_htab0.p, init.data(), words * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->P.htab = e->d_htab.p;
    e->P.htab0 = e->d_htab0.p;
    if (!e->n_cells) return MTE_OK;
    if (e->d_cell_pos.n < 2 * e->n_cells) HIP_TRY(e, e->d_cell_pos.alloc(2 * e->n_cells));
    if (e->d_cell_h.n < 2 * e->n_cells) HIP_TRY(e, e->d_cell_h.alloc(2 * e->n_cells));
    // a cell index no document carries keeps both positions undefined
    HIP_TRY(e, hipMemsetAsync(e->d_cell_pos.p, 0xFF, 2 * e->n_cells * sizeof(uint32_t), e->stream));
    HIP_TRY(e, hipMemsetAsync(e->d_cell_h.p, 0, 2 * e->n_cells * sizeof(uint32_t), e->stream));
    e->P.cell_pos = e->d_cell_pos.p;
    e->P.cell_h = e->d_cell_h.p;
    return MTE_OK;
}

// ---------------------------------------------------------------- incremental replay (option retain)
static void ck_forget(mte_engine* e) {
    e->ck_cur = -1;
    e->ck_prev.clear();
    e->ck_load.clear();
    e->ck_match.clear();
    e->ck_tabs_n = 0;
}
// word-wise hash of a byte range, continuing from h (a prefix's hash continues to the whole log's)
static uint64_t ck_hash(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, b + i, 8);
        h = (h ^ w) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
    }
    for (; i < n; i++) h = (h ^ b[i]) * 0x100000001B3ull;
    return h;
}
// payload units one at a time: a prefix's hash continued over the rest is the whole run's hash
// whatever the prefix's length (a word-wise hash would regroup the units after an odd cut)
static uint64_t ck_hash_units(uint64_t h, const uint16_t* y, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        h = (h ^ y[i]) * 0x100000001B3ull;
        h ^= h >> 31;
    }
    return h;
}
// an op record as the engine reads it: MTE_F_CATCHUP marks the ops of the messages still above
// minSeq at the END of a log (DocBuild::commit), which the row engines never read, so a prefix log
// and its extension differ there and nowhere else
static uint64_t ck_hash_ops(uint64_t h, const mte_op* o, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        mte_op x = o[i];
        x.flags &= ~MTE_F_CATCHUP;
        h = ck_hash(h, &x, sizeof x);
    }
    return h;
}
static uint64_t ck_tabs_count(const HostBatch& t) {
    return (uint64_t)t.propsets.size() + t.prop_keys.size() + t.key_offsets.size() + t.val_offsets.size();
}
// the loaded tables start with the last pass's: every id the checkpointed map records hold means the
// same key / value / property set
static bool ck_tabs_extend(const HostBatch& old, const HostBatch& nw) {
    auto pre = [](const auto& a, const auto& b) { return a.size() <= b.size() && std::equal(a.begin(), a.end(), b.begin()); };
    auto pre_ps = [](const std::vector<mte_propset>& a, const std::vector<mte_propset>& b) {
        if (a.size() > b.size()) return false;
        for (size_t i = 0; i < a.size(); i++)
            if (a[i].first != b[i].first || a[i].count != b[i].count) return false;
        return true;
    };
    return pre_ps(old.propsets, nw.propsets) && pre(old.prop_keys, nw.prop_keys) && pre(old.prop_vals, nw.prop_vals) &&
           pre(old.key_offsets, nw.key_offsets) && pre(old.key_text, nw.key_text) && pre(old.val_offsets, nw.val_offsets) &&
           pre(old.val_text, nw.val_text);
}
// mte_load with retain: which documents of the batch extend the last pass's (ck_match), and the
// hashes of their whole logs for the next one
static void ck_match_batch(mte_engine* e, const mte_batch* b) {
    const uint32_t nd = b->n_docs;
    e->ck_match.assign(nd, 0);
    e->ck_load.assign(nd, mte_engine::CkDoc{});
    const bool same = e->ck_cur >= 0 && e->ck_prev.size() == nd && e->ck_tabs_n &&
                      e->ck_map_words == e->map_words && ck_tabs_extend(e->ck_tabs, e->hb);
    for (uint32_t d = 0; d < nd; d++) {
        const mte_op* o = b->ops + b->doc_op_offsets[d];
        const uint16_t* y = b->payload + b->doc_payload_offsets[d];
        const uint64_t n = b->doc_op_offsets[d + 1] - b->doc_op_offsets[d];
        const uint64_t np = b->doc_payload_offsets[d + 1] - b->doc_payload_offsets[d];
        mte_engine::CkDoc& c = e->ck_load[d];
        c.n_ops = n;
        c.n_pay = np;
        uint64_t ho = 0xCBF29CE484222325ull, hp = 0xCBF29CE484222325ull, k = 0, kp = 0;
        if (same) {
            const mte_engine::CkDoc& q = e->ck_prev[d];
            if (q.n_ops && q.n_ops <= n && q.n_pay <= np) {
                ho = ck_hash_ops(ho, o, q.n_ops);
                hp = ck_hash_units(hp, y, q.n_pay);
                k = q.n_ops;
                kp = q.n_pay;
                if (ho == q.h_ops && hp == q.h_pay) e->ck_match[d] = q.n_ops;
            }
        }
        c.h_ops = ck_hash_ops(ho, o + k, n - k);
        c.h_pay = ck_hash_units(hp, y + kp, np - kp);
    }
}
// run_kernel with retain: this pass's regions, the previous pass's ones to continue from
static int ck_begin(mte_engine* e) {
    const uint32_t nd = (uint32_t)e->cfg.size();
    const int out = e->ck_cur == 0 ? 1 : 0;
    uint64_t tot = 0;
    e->last_ck_offered = 0;
    for (uint32_t d = 0; d < nd; d++) {
        DocCfg& c = e->cfg[d];
        c.ck_out_off = tot;
        c.ck_cap = ck_region_words(c.arena_cap, c.map_cap, e->map_words);
        tot += (c.ck_cap + 63) & ~63ull;
        const bool have = e->ck_cur >= 0 && d < e->ck_match.size() && d < e->ck_prev.size() && e->ck_match[d];
        c.ck_at = have ? e->ck_match[d] : 0;
        c.ck_in_off = have ? e->ck_prev[d].off : 0;
        e->last_ck_offered += have;
    }
    HIP_TRY(e, e->d_ck[out].fit(std::max<uint64_t>(tot, 64)));
    HIP_TRY(e, hipMemsetAsync(e->d_ck[out].p, 0, tot * 4, e->stream));  // every region invalid until saved
    HIP_TRY(e, hipMemcpyAsync(e->d_cfg.p, e->cfg.data(), nd * sizeof(DocCfg), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->P.ck_out = e->d_ck[out].p;
    e->P.ck_in = e->ck_cur >= 0 ? e->d_ck[e->ck_cur].p : nullptr;
    return MTE_OK;
}
// after the pass: its checkpoints are the ones the next pass continues from (the same batch replayed
// again continues every document from its end)
static void ck_end(mte_engine* e, const uint32_t* ctr) {
    const uint32_t nd = (uint32_t)e->cfg.size();
    e->ck_cur = e->ck_cur == 0 ? 1 : 0;
    e->ck_prev.assign(nd, mte_engine::CkDoc{});
    for (uint32_t d = 0; d < nd; d++) {
        mte_engine::CkDoc& q = e->ck_prev[d];
        if (d < e->ck_load.size()) q = e->ck_load[d];
        q.off = e->cfg[d].ck_out_off;
        q.n_ops = e->n_ops_doc[d];
        q.n_pay = e->cfg[d].payload_len;
    }
    e->ck_match.assign(nd, 0);
    for (uint32_t d = 0; d < nd; d++) e->ck_match[d] = e->ck_prev[d].n_ops;
    e->ck_tabs.propsets = e->hb.propsets;
    e->ck_tabs.prop_keys = e->hb.prop_keys;
    e->ck_tabs.prop_vals = e->hb.prop_vals;
    e->ck_tabs.key_offsets = e->hb.key_offsets;
    e->ck_tabs.key_text = e->hb.key_text;
    e->ck_tabs.val_offsets = e->hb.val_offsets;
    e->ck_tabs.val_text = e->hb.val_text;
    e->ck_tabs_n = 1 + ck_tabs_count(e->hb);
    e->ck_map_words = e->map_words;
    e->last_resumed_docs = ctr[12];
    e->last_resumed_ops = ctr[13];
    e->P.ck_out = nullptr;
    e->P.ck_in = nullptr;
}

int mte_load(mte_engine* e, const mte_batch* b) {
    if (!e || !b) return MTE_E_ARG;
    HIP_TRY(e, hipSetDevice(e->device));
    e->hb.copy_from(b, false);
    e->emit_tables = false;
    e->generated = false;
    e->host_ops_valid = false;
    e->replayed = e->downloaded = false;
    e->stage_copy_ms = e->stage_wait_ms = 0;
    const uint32_t nd = b->n_docs;
    std::vector<uint64_t> n_ops(nd), pay(nd), pi(nd), an(nd);
    std::vector<uint8_t> collab(nd), has_nl(nd, 0), not_lean(nd, 0), doc_ext(nd, 0), doc_cu(nd, 0), not_rows(nd, 0),
        wide(nd, 0);
    std::vector<uint32_t> doc_keys(nd, 0);  // distinct property keys of each document's ops
    std::vector<uint32_t> n_cell(nd, 0);    // SharedMatrix cell records (MTE_OP_CELL)
    // one pass over each document's ops and payload, documents spread over host threads (the scan is
    // most of mte_load's host time on large batches)
    auto scan = [&](uint32_t d) {
        for (uint64_t q = b->doc_payload_offsets[d]; q < b->doc_payload_offsets[d + 1]; q++)
            if (b->payload[q] == (uint16_t)'\n') {
                has_nl[d] = 1;
                break;
            }
        n_ops[d] = b->doc_op_offsets[d + 1] - b->doc_op_offsets[d];
        pay[d] = b->doc_payload_offsets[d + 1] - b->doc_payload_offsets[d];
        bool rel = false;
        count_doc_ops(b->ops, b->doc_op_offsets, d, pi[d], an[d], &rel);
        std::vector<uint32_t> keys;
        for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++) {
            if ((b->ops[i].flags & MTE_F_PERM) || b->ops[i].type == MTE_OP_CELL) doc_ext[d] = 1;
            if (b->ops[i].type > MTE_OP_NOOP) not_rows[d] = 1;  // summary loads: the row engine would spill
            if (b->ops[i].type == MTE_OP_CELL) n_cell[d]++;
            if (b->ops[i].flags & MTE_F_CATCHUP) doc_cu[d] = 1;
            const uint32_t ps = b->ops[i].props;
            if (ps && ps < b->n_propsets)
                for (uint32_t q = 0; q < b->propsets[ps].count; q++) keys.push_back(b->prop_keys[b->propsets[ps].first + q]);
        }
        if (keys.size() > 7) {  // only a document that could exceed the narrow record pays the sort
            std::sort(keys.begin(), keys.end());
            doc_keys[d] = (uint32_t)(std::unique(keys.begin(), keys.end()) - keys.begin());
        }
        collab[d] = e->hb.client(d, 0).empty() ? 0 : 1;  // empty observer name => local, non-collab
        // writers 32..63: FULL kernels (the lean LDS engine's removers masks are 32 bits), and the
        // WIDE row engine in k_rows (a second removers word per slot)
        const uint32_t n_names = e->hb.doc_client_offsets[d + 1] - e->hb.doc_client_offsets[d];
        wide[d] = n_names > 32;
        // (clients 64..127: the LDS / HBM engines only, whose overlap masks have a second word)
        not_rows[d] = not_rows[d] || has_nl[d] || rel || n_names > 64;
        not_lean[d] = not_rows[d] || wide[d] || pi[d] || an[d];
        // a local, non-collaborative document is the LDS engine's path (lean or not): RegEngine::replay
        // hands it over at op 0, and k_rows has no LDS plan to hand it to
        not_rows[d] = not_rows[d] || !collab[d];
        // a document with more than MTE_MAX_CLIENTS clients in a window fails alone (MTE_DOC_UNSUPPORTED at its
        // first op from a client beyond the cap), never the batch
    };
    {
        const unsigned nt = std::max(1u, std::min({16u, std::thread::hardware_concurrency(), (nd + 255) / 256}));
        std::atomic<uint32_t> next{0};
        auto work = [&]() {
            for (uint32_t d0; (d0 = next.fetch_add(256)) < nd;)
                for (uint32_t d = d0; d < std::min(nd, d0 + 256); d++) scan(d);
        };
        run_pool(nt, work);
    }
    bool lean = true, ext = false, cu_any = false, rows_ok = true, any_wide = false;
    uint32_t max_keys = 7;
    for (uint32_t d = 0; d < nd; d++) max_keys = std::max(max_keys, std::min<uint32_t>(doc_keys[d], MTE_MAX_PROPS));
    e->map_words = ((1 + 2 * max_keys) + 3) & ~3u;  // 16 for up to 7 keys, 128 for MTE_MAX_PROPS
    for (uint32_t d = 0; d < nd; d++) {
        lean = lean && !not_lean[d];
        rows_ok = rows_ok && !not_rows[d];
        any_wide = any_wide || wide[d];
        ext = ext || doc_ext[d];
        cu_any = cu_any || doc_cu[d];
    }
    auto t0 = std::chrono::steady_clock::now();
    int rc;
    if ((rc = layout_and_alloc(e, n_ops, pay, pi, an, collab, has_nl, 0, b->doc_op_offsets, b->doc_payload_offsets)))
        return rc;
    e->last_alloc_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    // catch-up delta records (legacy summaries): an insert has one range, a remove / annotate at most
    // one per character of its range (every delta segment is visible in the op's view), or at most
    // every segment when a position is relative
    uint64_t cu = 0;
    for (uint32_t d = 0; d < nd && cu_any; d++) {  // (no catch-up record in a batch without catch-up ops)
        DocCfg& c = e->cfg[d];
        uint64_t cap = 0;
        for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++) {
            const mte_op& o = b->ops[i];
            if (!(o.flags & MTE_F_CATCHUP)) continue;
            if (o.type == MTE_OP_INSERT || o.type == MTE_OP_INSERT_MARKER) cap += 1;
            else if (o.flags & MTE_F_REL) cap += c.seg_cap;
            else cap += (uint64_t)std::max<int64_t>(0, (int64_t)o.a - (int64_t)o.pos1);
        }
        c.cu_off = cu;
        c.cu_cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFF0ull);
        cu += c.cu_cap;
    }
    // (the catch-up offsets reach the device with the cell tables' below: the same size, copied into
    // the buffer the kernels' Params::docs already points at -- upload would reallocate it)
    if (cu) HIP_TRY(e, e->d_cu.alloc(2 * cu));
    e->P.cu_rec = cu ? e->d_cu.p : nullptr;
    if ((rc = load_cells(e, b, n_cell))) return rc;
    if (cu || e->n_cells)  // ht_off / ht_cap: the same re-upload as the catch-up offsets above
        HIP_TRY(e, hipMemcpyAsync(e->d_cfg.p, e->cfg.data(), e->cfg.size() * sizeof(DocCfg), hipMemcpyHostToDevice,
                                  e->stream));
    if ((rc = upload(e, e->d_ops, b->ops, b->doc_op_offsets[nd]))) return rc;
    if ((rc = upload(e, e->d_payload, b->payload, b->doc_payload_offsets[nd]))) return rc;
    if ((rc = upload_props(e))) return rc;
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->last_h2d_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    e->P.ops = e->d_ops.p;
    e->P.payload = e->d_payload.p;
    // catch-up delta records are only read by the SnapshotLegacy writer: a batch whose only extension
    // is MTE_F_CATCHUP runs the lean / FULL kernels (which ignore the flag) unless the replay emits
    // the legacy format (run_kernel decides, snapshot_format may change after the load)
    e->lean_base = lean;
    e->props_rows_ok = rows_ok;
    e->doc_not_rows = not_rows;
    e->rows_wide = any_wide;
    e->ext_perm = ext;
    e->ext_cu = cu_any;
    e->lean_ok = lean && !ext;
    e->ext_needed = ext;
    if ((rc = alloc_out_text(e))) return rc;
    if (e->retain) ck_match_batch(e, b);
    else ck_forget(e);
    return MTE_OK;
}

// HBM-resident capacities for a document that outgrew the LDS plan (blocks hold >= 4 segments
// except transiently; segments <= 2 per op + 1 without zamboni).
static void doc_hbm_caps(uint64_t n, DocCfg& c, uint64_t& bytes) {
    hbm_caps(n, c.hb_blk, c.hb_ord, c.hb_in, c.hb_heap);
    bytes = HbmLayout::of(c.hb_blk, c.hb_ord, c.hb_in, c.hb_heap).bytes;
}

extern "C++" {
template <class T>
static hipError_t grow(DevBuf<T>& b, size_t n) {  // grow-only device buffer (contents not kept)
    if (b.p && b.n >= n) return hipSuccess;
    return b.alloc(std::max<size_t>(n, 1));
}
}

// Property texts (interned JSON), key order data and every document's client names (JSON-quoted
// UTF-8, by slot) for the emission kernels; once per loaded / generated batch.
static int emit_tables(mte_engine* e) {
    if (e->emit_tables) return MTE_OK;
    const HostBatch& hb = e->hb;
    const uint32_t nd = e->P.n_docs;
    std::vector<char> names;
    std::vector<uint64_t> off{0}, base;
    for (uint32_t d = 0; d < nd; d++) {
        base.push_back(off.size() - 1);
        const uint32_t nc = hb.doc_client_offsets.size() > d + 1 ? hb.doc_client_offsets[d + 1] - hb.doc_client_offsets[d] : 0;
        for (uint32_t c = 0; c < nc; c++) {
            const std::string n = hb.client(d, c);
            std::u16string u;
            json::decode_utf8(n.data(), n.size(), u);
            std::string q;
            json::quote(q, u);
            names.insert(names.end(), q.begin(), q.end());
            off.push_back(names.size());
        }
    }
    base.push_back(off.size() - 1);
    std::vector<char> kt(hb.key_text.begin(), hb.key_text.end()), vt(hb.val_text.begin(), hb.val_text.end());
    int rc;
    if ((rc = upload(e, e->d_names, names)) || (rc = upload(e, e->d_name_off, off)) || (rc = upload(e, e->d_name_base, base)) ||
        (rc = upload(e, e->d_key_text, kt)) || (rc = upload(e, e->d_key_off, hb.key_offsets)) ||
        (rc = upload(e, e->d_val_text, vt)) || (rc = upload(e, e->d_val_off, hb.val_offsets)) ||
        (rc = upload(e, e->d_key_is_index, e->key_is_index)) || (rc = upload(e, e->d_key_index, e->key_index)))
        return rc;
    HIP_TRY(e, grow(e->d_ent, e->P.out_cap));
    HIP_TRY(e, grow(e->d_tscr, e->P.out_text_cap));
    HIP_TRY(e, grow(e->d_n_ent, nd));
    HIP_TRY(e, grow(e->d_nblobs, nd));
    HIP_TRY(e, grow(e->d_emit_size, nd));
    HIP_TRY(e, grow(e->d_out_off, nd));
    HIP_TRY(e, grow(e->d_blob_base, nd));
    e->h_emit_size.assign(nd, 0);
    e->h_nblobs.assign(nd, 0);
    e->h_out_off.assign(nd, 0);
    e->h_blob_base.assign(nd, 0);
    e->emit_tables = true;
    return MTE_OK;
}

static EmitParams emit_params(mte_engine* e) {
    EmitParams P{};
    P.chunk = e->chunk;
    P.legacy = e->legacy ? 1u : 0u;
    P.res = e->d_res.p;
    P.cfg = e->d_cfg.p;
    P.vis = e->d_out_vis.p;
    P.aux = e->d_out_aux.p;
    P.maps = e->P.out_maps;
    P.map_words = e->map_words;
    P.text = e->d_out_text.p;
    P.esc = e->d_out_esc.p;
    P.key_text = e->d_key_text.p;
    P.key_off = e->d_key_off.p;
    P.key_is_index = e->d_key_is_index.p;
    P.key_index = e->d_key_index.p;
    P.val_text = e->d_val_text.p;
    P.val_off = e->d_val_off.p;
    P.val_flags = e->d_val_flags.p;
    P.val_objidx = e->d_val_objidx.p;
    P.val_objmatch = e->d_val_objmatch.p;
    P.names = e->d_names.p;
    P.name_off = e->d_name_off.p;
    P.name_base = e->d_name_base.p;
    P.ent = e->d_ent.p;
    P.tscr = e->d_tscr.p;
    P.n_ent = e->d_n_ent.p;
    P.size = e->d_emit_size.p;
    P.nblobs = e->d_nblobs.p;
    P.out_off = e->d_out_off.p;
    P.blob_base = e->d_blob_base.p;
    return P;
}

// SnapshotV1 bytes of the listed documents into pool k on stream s: COUNT, lay the documents out,
// WRITE. Returns with s drained (the host needs the sizes between the two kernels).
static int emit_list(mte_engine* e, int k, const std::vector<uint32_t>& list, hipStream_t s) {
    auto& pl = e->pool[k];
    pl.used = pl.blobs = 0;
    if (list.empty()) return MTE_OK;
    const uint32_t nd = e->P.n_docs;
    HIP_TRY(e, grow(e->d_emit_list[k], list.size()));
    HIP_TRY(e, hipMemcpyAsync(e->d_emit_list[k].p, list.data(), list.size() * 4, hipMemcpyHostToDevice, s));
    EmitParams P = emit_params(e);
    P.list = e->d_emit_list[k].p;
    P.n_list = (uint32_t)list.size();
    HIP_TRY(e, launch_emit(P, false, s));
    HIP_TRY(e, hipMemcpyAsync(e->h_emit_size.data(), e->d_emit_size.p, nd * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(e, hipMemcpyAsync(e->h_nblobs.data(), e->d_nblobs.p, nd * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(e, hipStreamSynchronize(s));
    for (uint32_t d : list) {
        if (!e->h_emit_size[d]) continue;
        e->h_out_off[d] = pl.used;
        pl.used += e->h_emit_size[d];
        e->h_blob_base[d] = pl.blobs;
        pl.blobs += e->h_nblobs[d];
        e->emit_pool_of[d] = (uint8_t)k;
    }
    HIP_TRY(e, grow(pl.out, pl.used));
    HIP_TRY(e, grow(pl.blob_off, pl.blobs));
    HIP_TRY(e, hipMemcpyAsync(e->d_out_off.p, e->h_out_off.data(), nd * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(e, hipMemcpyAsync(e->d_blob_base.p, e->h_blob_base.data(), nd * 8, hipMemcpyHostToDevice, s));
    P.out = pl.out.p;
    P.blob_off = pl.blob_off.p;
    HIP_TRY(e, launch_emit(P, true, s));
    HIP_TRY(e, hipStreamSynchronize(s));
    return MTE_OK;
}

static int run_kernel(mte_engine* e, bool gen) {
    HIP_TRY(e, hipSetDevice(e->device));
    // nd: the documents this pass replays (e->order, LPT; a SharedMatrix batch's first pass runs
    // only its cell documents), nall: the batch's documents (results are indexed by document)
    const uint32_t nd = (uint32_t)e->order.size(), nall = e->P.n_docs;
    e->P.pool_limit = e->pool_limit;
    e->P.rows_pool_lim = e->rows_pool_lim;
    e->P.reg_solo = e->reg_solo;
    e->P.reg_lb_limit = e->reg_lb_limit;
    e->P.doc_list = e->d_order.p;
    e->P.n_list = nd;
    int rc;
    if ((rc = alloc_slots(e))) return rc;  // options may have changed the wave plan
    // option retain: checkpoints out, and in from the last pass (not for the generator, whose batch
    // is made in the pass, nor the two passes of a SharedMatrix batch)
    const bool ck = e->retain && !gen && e->P.cell_mode == 0;
    e->P.ck_in = e->P.ck_out = nullptr;
    if (ck && (rc = ck_begin(e))) return rc;
    uint32_t groups, hbm_waves, lds_active;
    const uint32_t n_solo = e->P.n_solo;
    // engine level (engine.hpp): the generator always runs FULL
    if (!gen) {
        e->ext_needed = e->ext_perm || (e->ext_cu && e->legacy);
        e->lean_ok = e->lean_base && !e->ext_needed;
    }
    const int full = gen ? 1 : e->ext_needed ? 2 : (e->lean_ok && e->lean_opt) ? 0 : 1;
    e->last_lean = full == 0;
    wave_plan(e, nd, groups, hbm_waves, &lds_active, n_solo);
    // Lean replays run the bulk on the row engine (k_rows; DOC_SPILL re-runs as below): 4 waves per
    // CU for long documents, each on a SIMD of its own with fixed rows (C5: 1 024 x 10^6 ops, 4.4 s
    // per step against 9.8 s on k_lds / k_hbmq), else 12 (three per SIMD on the shared row pool; C2
    // 98 ms against 110 at 8 and 166 on the sixteen LDS / HBM waves per CU; C3 1.34 s against 1.87 at
    // 8 and 2.15 on k_lds / k_hbmq; a document the pool cannot grow restarts inside the pass), beside
    // the solo documents too (C4: the same critical path, 4 046 vs 4 047 ms, but none of the 4 100
    // documents k_lds continued HBM-resident, whose spill and continuation traffic was 15 GB a pass).
    // Property-carrying batches, and batches with writers 32..63 (FULL only for those: no '\n', no
    // relative positions) take the same route on the PROPS row engine, WIDE for the latter.
    uint32_t rows = 0;
    // (PROPS rows only when properties are what requires FULL: option lean = 0 on a lean batch keeps
    // the FULL LDS kernels, as that diagnostic switch says)
    bool props_rows = full == 1 && !e->lean_ok && e->props_rows_ok;
    // A FULL batch with a few documents the row engines cannot replay (summary loads, relative
    // positions, '\n' in a property-carrying document, local edits, 64+ clients): its bulk still runs
    // on k_rows' fixed rows, and those documents hand over at op 0 (rows_dump) to continue
    // HBM-resident in k_rows_cont on the FULL engine -- instead of the whole bulk leaving k_rows for
    // k_lds / k_hbmq. Only while they are a small share of the bulk and each finds an HBM slot.
    // (a lean batch's only such documents are local ones: '\n', relative positions, summaries and
    // 64+ clients make a batch FULL)
    bool mixed = false;
    if (!gen && full <= 1 && !e->props_rows_ok && e->rows_mixed && e->rows_bulk && !e->force_hbm && nd > n_solo &&
        e->doc_not_rows.size() == nall) {
        uint64_t nr_docs = 0, nr_ops = 0, all_ops = 0;
        for (uint32_t k = n_solo; k < nd; k++) {
            const uint32_t d = e->order[k];
            all_ops += e->n_ops_doc[d];
            if (e->doc_not_rows[d]) {
                nr_docs++;
                nr_ops += e->n_ops_doc[d];
            }
        }
        // Once k_hbmq takes a slot before a document, k_lds / k_hbmq replay such a FULL batch about
        // as fast as k_rows' 4-wave fixed rows (2 048 x 3 000-op logs: 51 vs 58 ms; 512 x 20 000:
        // 228 vs 240 ms, profiles/r06/mixed_route.json), so the rows route is taken where it buys
        // something: a retained pass (its row documents continue from their checkpoints next time)
        // -- option 2 forces it
        mixed = nr_docs <= e->n_slots && nr_docs <= 4096 && nr_ops * 4 <= all_ops && (e->rows_mixed >= 2 || ck);
        if (full == 1) props_rows = mixed;
    }
    if (!gen && ((full == 0 && (e->props_rows_ok || mixed)) || props_rows) && e->rows_bulk && !e->force_hbm && nd > n_solo) {
        uint64_t bulk_ops = 0;
        for (uint32_t k = n_solo; k < nd; k++) bulk_ops += e->n_ops_doc[e->order[k]];
        // (long documents take 4 waves whatever their count: eight of them, ~120 leaf blocks each,
        // would not fit one CU's 79-row pool and spill to HBM re-runs of 10^5+ ops)
        const bool long_docs = bulk_ops >= 200000ull * (nd - n_solo);
        // (writers 32..63: documents grow fast -- minSeq trails far behind, zamboni settles little --
        // so the shared pool at 8 / 12 waves is full most of the time: 4 waves on fixed rows, a
        // document outgrowing them continuing HBM-resident; tools/wide_probe.py, profiles/r05/r05l)
        rows = e->rows_bulk > 0 ? (uint32_t)e->rows_bulk : (long_docs || e->rows_wide) ? 4u : 12u;
        if (mixed) rows = 4;  // (the handoff at op 0 needs the fixed rows' state dump)
    }
    e->last_mixed = rows && mixed;
    if (ck && rows) rows = 4;  // (the checkpointing k_rows runs 4 waves per CU on fixed rows)
    e->last_rows = rows;
    if (rows) groups = hbm_waves = lds_active = 0;
    e->P.slot_hbm0 = groups * LDS_WAVES;
    e->P.lds_active = lds_active;
    e->P.n_prio = 0;
    if (groups)  // critical-path documents lead the LPT order
        while (e->P.n_prio < nd && e->cfg[e->order[e->P.n_prio]].prio) e->P.n_prio++;
    e->P.n_prio = std::max(e->P.n_prio, n_solo);  // k_lds / k_hbmq / k_rows start after the solo documents
    e->P.n_hslots = hbm_waves;
    if (rows) {  // k_rows alone: its waves continue documents HBM-resident in any free slot
        e->P.slot_hbm0 = 0;
        e->P.n_hslots = e->n_slots;
    }
    // the streams of this pass (an A/B with CU-masked streams, hipExtStreamCreateWithCUMask, that kept
    // the solo workgroups' CUs to themselves measured the C4 pass 8 % SLOWER -- 9.07 s vs 8.38 s, the
    // solo workgroups themselves included -- and hung at teardown: not used)
    hipStream_t s_main = e->stream, s_hbmq = e->stream2, s_solo = e->stream3;
    HIP_TRY(e, hipMemsetAsync(e->d_counters.p, 0, 16 * sizeof(uint32_t), s_main));
    if (e->d_rows_retry.p) HIP_TRY(e, hipMemsetAsync(e->d_rows_retry.p, 0, e->d_rows_retry.n * sizeof(uint32_t), s_main));
    HIP_TRY(e, hipMemsetAsync(e->d_slot_bits.p, 0, e->d_slot_bits.n * sizeof(uint32_t), s_main));
    HIP_TRY(e, hipMemsetAsync(e->d_prof.p, 0, e->d_prof.n * sizeof(uint64_t), s_main));  // profiling build
    HIP_TRY(e, hipMemsetAsync(e->d_solo_started.p, 0, sizeof(uint32_t), s_main));  // k_solo_gate's counter
    HIP_TRY(e, hipEventRecord(e->ev0, s_main));
    std::vector<uint32_t> spill;
    e->map_rr_off.clear();  // (set again below for this pass's re-run documents)
    float lds_ms = 0, hbm_ms = 0;
    // pass 1: the solo workgroups first (third stream: each takes a CU), then the LDS workgroups
    // (one per remaining CU, all of its LDS), then the HBM-resident waves on the second stream so
    // they fill every CU's remaining wave slots; k_lds and k_hbmq drain one document queue
    if (n_solo) {
        HIP_TRY(e, hipStreamWaitEvent(s_solo, e->ev0, 0));
        HIP_TRY(e, hipEventRecord(e->ev_s0, s_solo));
        HIP_TRY(e, launch_solo(e->P, gen, full, n_solo, ck, s_solo));
        HIP_TRY(e, hipEventRecord(e->ev_s1, s_solo));
        HIP_TRY(e, hipEventRecord(e->ev3, s_solo));
        // the bulk starts once the solo workgroups hold their CUs (k_solo_gate)
        if (e->solo_gate && (groups || rows || hbm_waves)) HIP_TRY(e, launch_solo_gate(e->d_solo_started.p, n_solo, s_main));
    }
    HIP_TRY(e, hipEventRecord(e->ev_gate, s_main));
    if (groups) HIP_TRY(e, launch_lds(e->P, gen, full, groups, s_main));
    if (rows) {
        const uint32_t cus = bulk_cus(e, n_solo);
        const uint32_t per = rows >= 12 ? 12u : rows >= 8 ? 8u : 4u;
        HIP_TRY(e, launch_rows(e->P, per, std::min<uint32_t>(cus, (nd - n_solo + per - 1) / per), full == 1,
                               full == 1 && e->rows_wide, ck, s_main));
        // documents k_rows handed to HBM slots between two ops continue here (k_rows_cont)
        HIP_TRY(e, launch_rows_cont(e->P, full == 1, full == 1 && e->rows_wide, e->P.n_hslots, s_main));
    }
    // k_hbmq: one workgroup (wave) per document; those that find the queue drained exit at once
    if (hbm_waves && !groups) {
        HIP_TRY(e, launch_hbmq(e->P, gen, full, nd, s_main));
    } else if (hbm_waves) {
        HIP_TRY(e, hipStreamWaitEvent(s_hbmq, e->ev_gate, 0));
        HIP_TRY(e, launch_hbmq(e->P, gen, full, nd, s_hbmq));
        HIP_TRY(e, hipEventRecord(e->ev2, s_hbmq));
        HIP_TRY(e, hipStreamWaitEvent(s_main, e->ev2, 0));
    }
    const bool emit = !gen && e->emit_opt;
    e->emitted_legacy = e->legacy;
    e->emit_downloaded = false;
    e->emit_pool_of.assign(nall, 255);
    e->pool[0].used = e->pool[0].blobs = e->pool[1].used = e->pool[1].blobs = 0;
    int erc;
    if (emit) {
        if ((erc = emit_tables(e))) return erc;
        // round 0: every document but the solo ones, while k_solo still replays the critical path
        // (the documents the host re-runs are still DOC_SPILL here: COUNT skips them)
        std::vector<uint32_t> bulk(e->order.begin() + std::min<uint32_t>(n_solo, nd), e->order.end());
        if ((erc = emit_list(e, 0, bulk, s_main))) return erc;
    }
    if (n_solo) HIP_TRY(e, hipStreamWaitEvent(s_main, e->ev3, 0));
    HIP_TRY(e, hipEventRecord(e->ev1, s_main));
    HIP_TRY(e, hipStreamSynchronize(s_main));
    HIP_TRY(e, hipEventElapsedTime(&lds_ms, e->ev0, e->ev1));
    e->res.resize(nall);
    HIP_TRY(e, hipMemcpy(e->res.data(), e->d_res.p, nall * sizeof(DocRes), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < nd; i++)
        if (e->res[e->order[i]].status == DOC_SPILL) spill.push_back(e->order[i]);
    uint32_t ctr[16];
    HIP_TRY(e, hipMemcpy(ctr, e->d_counters.p, sizeof ctr, hipMemcpyDeviceToHost));
    e->last_continued = ctr[4];
    e->last_hbm_docs = 0;
    for (uint32_t i = 0; i < nd; i++) e->last_hbm_docs += e->res[e->order[i]].mode == 1;
    e->last_hbm_waves = hbm_waves;
    e->last_lds_groups = groups;
    e->last_solo = n_solo;
    e->last_solo_ms = 0;
    if (n_solo) {
        float sm = 0;
        if (hipEventElapsedTime(&sm, e->ev_s0, e->ev_s1) == hipSuccess) e->last_solo_ms = sm;
        if (hipEventElapsedTime(&sm, e->ev0, e->ev_s0) == hipSuccess) e->last_solo_lead_ms = sm;
        if (hipEventElapsedTime(&sm, e->ev_s1, e->ev1) == hipSuccess) e->last_solo_tail_ms = sm;
        uint64_t clk[4] = {0, 0, 0, 0}, bulk0 = 0;  // solo workgroup 0: the batch's longest document
        if (e->d_solo_clk.p) {
            HIP_TRY(e, hipMemcpy(clk, e->d_solo_clk.p, sizeof clk, hipMemcpyDeviceToHost));
            HIP_TRY(e, hipMemcpy(&bulk0, e->d_solo_clk.p + 4 * SOLO_CLK_SLOTS, 8, hipMemcpyDeviceToHost));
        }
        e->last_solo_cycles = clk[2] - clk[0];
        e->last_solo_ref = clk[3] - clk[1];
        // the critical wave's start after the bulk's first wave (100 MHz ticks; negative: before it)
        e->last_solo_start_delay = (groups || rows) && bulk0 ? (int64_t)(clk[1] - bulk0) : 0;
    }
    e->last_spilled = (uint32_t)spill.size();
    if (!spill.empty()) {
        // second pass: the spilled documents, HBM-resident, one wave each, longest first
        uint64_t total = 0;
        for (uint32_t d : spill) {
            uint64_t bytes;
            doc_hbm_caps(e->n_ops_doc[d], e->cfg[d], bytes);
            e->cfg[d].hb_off = total;
            total += (bytes + 255) & ~255ull;
        }
        HIP_TRY(e, e->d_hbm.alloc(total));
        // property maps: the load-time estimate (prop inserts + 4 per annotate) may be short for a
        // re-run document; it gets the worst case, a new map per annotated character, in a table of
        // its own (e->map_rr_off; the first pass's layout stays as it was)
        std::vector<std::pair<uint64_t, uint32_t>> keep_maps;
        uint64_t mtot = 0;
        e->map_rr_off.assign(nall, UINT64_MAX);
        e->map_rr_cap.assign(nall, 0);
        for (uint32_t d : spill) {
            DocCfg& c = e->cfg[d];
            uint64_t cap = 16;
            if (gen) {
                cap += e->n_ops_doc[d] * 17;  // generated annotates span at most 16 characters
            } else {
                std::vector<mte_op> ops(c.op_end - c.op_begin);
                if (!ops.empty())
                    HIP_TRY(e, hipMemcpy(ops.data(), e->d_ops.p + c.op_begin, ops.size() * sizeof(mte_op), hipMemcpyDeviceToHost));
                // a relative-position annotate can touch every segment of the document: bound it by
                // the longest the document can get, its payload plus one unit per marker insert
                uint64_t markers = 0;
                for (const mte_op& o : ops) markers += o.type == MTE_OP_INSERT_MARKER;
                for (const mte_op& o : ops) {
                    if (o.type == MTE_OP_ANNOTATE)
                        cap += (o.flags & MTE_F_REL) ? (uint64_t)c.payload_len + markers + 2
                                                     : (uint64_t)std::max<int64_t>(0, (int64_t)o.a - o.pos1) + 2;
                    else if (o.props)
                        cap += 1;
                }
            }
            keep_maps.emplace_back(c.map_off, c.map_cap);
            c.map_cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFF0ull);
            c.map_off = mtot;
            e->map_rr_off[d] = mtot;
            e->map_rr_cap[d] = c.map_cap;
            mtot += c.map_cap;
        }
        HIP_TRY(e, e->d_maps_rr.alloc(std::max<uint64_t>(mtot, 1) * e->map_words));
        if ((rc = upload(e, e->d_cfg, e->cfg))) return rc;
        if ((rc = upload(e, e->d_list, spill))) return rc;
        e->P.docs = e->d_cfg.p;
        e->P.hbm = e->d_hbm.p;
        e->P.doc_list = e->d_list.p;
        e->P.n_list = (uint32_t)spill.size();
        e->P.maps = e->d_maps_rr.p;
        e->P.map_rerun = 1;
        HIP_TRY(e, hipEventRecord(e->ev0, e->stream));
        HIP_TRY(e, launch_hbm(e->P, gen, full, (uint32_t)spill.size(), e->stream));
        HIP_TRY(e, hipEventRecord(e->ev1, e->stream));
        HIP_TRY(e, hipStreamSynchronize(e->stream));
        HIP_TRY(e, hipEventElapsedTime(&hbm_ms, e->ev0, e->ev1));
        e->P.maps = e->d_maps.p;
        e->P.map_rerun = 0;
        for (size_t q = 0; q < spill.size(); q++) {  // the next pass starts from the load-time layout
            e->cfg[spill[q]].map_off = keep_maps[q].first;
            e->cfg[spill[q]].map_cap = keep_maps[q].second;
        }
        if ((rc = upload(e, e->d_cfg, e->cfg))) return rc;
        e->P.docs = e->d_cfg.p;
        e->P.doc_list = e->d_order.p;
        e->P.n_list = nd;
    }
    e->last_lds_ms = lds_ms;
    e->last_hbm_ms = hbm_ms;
    e->last_kernel_ms = (double)lds_ms + hbm_ms;
    e->last_emit_ms = 0;
    if (emit) {  // round 1: the solo documents and those the host re-ran
        std::vector<uint32_t> rest(e->order.begin(), e->order.begin() + std::min<uint32_t>(n_solo, nd));
        rest.insert(rest.end(), spill.begin(), spill.end());
        HIP_TRY(e, hipEventRecord(e->ev0, e->stream));
        if ((erc = emit_list(e, 1, rest, e->stream))) return erc;
        HIP_TRY(e, hipEventRecord(e->ev1, e->stream));
        HIP_TRY(e, hipEventSynchronize(e->ev1));
        float ms = 0;
        HIP_TRY(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
        e->last_emit_ms = ms;
    }
    e->res.resize(nall);
    HIP_TRY(e, hipMemcpy(e->res.data(), e->d_res.p, nall * sizeof(DocRes), hipMemcpyDeviceToHost));
    if (ck) ck_end(e, ctr);
    else if (!gen) e->last_resumed_docs = e->last_resumed_ops = 0;
    e->replayed = true;
    e->downloaded = false;
    return MTE_OK;
}

int mte_retain(mte_engine* e, int on) { return e ? mte_set_option(e, "retain", on) : MTE_E_ARG; }

int mte_replay(mte_engine* e, mte_stats* out) {
    if (!e) return MTE_E_ARG;
    if (!e->P.ops) return set_err(e, MTE_E_STATE, "mte_replay before mte_load/mte_generate");
    int rc;
    if (e->n_cells && !e->generated) {
        // cell ops: pass 1 evaluates adjustPosition in both vectors of every cell op, pass 2 replays
        // with the handle allocations both gate (a vector's positions do not depend on its handles)
        // Pass 1 runs only the documents that carry cell records (their positions are all it
        // produces), without emission; pass 2 replays the whole batch.
        std::vector<uint32_t> all = e->order, sub;
        for (uint32_t d : all)
            if (e->cell_recs.count(d)) sub.push_back(d);
        const bool emit_was = e->emit_opt;
        e->order = sub;
        e->emit_opt = false;
        e->P.cell_mode = 1;
        rc = upload(e, e->d_order, e->order);
        if (!rc) rc = run_kernel(e, false);
        const double ms1 = e->last_kernel_ms;
        e->order = all;
        e->emit_opt = emit_was;
        if (!rc) rc = upload(e, e->d_order, e->order);
        e->last_cell_pass_ms = ms1;
        e->P.cell_mode = 2;
        if (!rc) rc = run_kernel(e, false);
        e->last_kernel_ms += ms1;
    } else {
        e->P.cell_mode = 0;
        rc = run_kernel(e, false);
    }
    if (rc) return rc;
    if (out) {
        memset(out, 0, sizeof *out);
        out->docs = e->P.n_docs;
        for (auto& r : e->res) {
            out->ops += r.ops;
            out->messages += r.msgs;
            if (r.status) out->failed_docs++;
        }
        out->kernel_ms = e->last_kernel_ms;
        out->h2d_ms = e->last_h2d_ms;
    }
    return MTE_OK;
}

// The generator's property sets: every single-key set and every two-key set over the C3 keys and
// values, in a fixed order.
static uint32_t build_generator_props(mte_engine* e) {
    Interner in(&e->hb);
    const char16_t* keys[4] = {u"bold", u"italic", u"color", u"size"};
    const char* vals[7] = {"true", "false", "\"red\"", "\"blue\"", "10", "12", "null"};
    uint32_t kid[4], vid[7];
    for (int i = 0; i < 4; i++) kid[i] = in.key(keys[i]);
    for (int i = 0; i < 7; i++) vid[i] = in.val(vals[i]);
    uint32_t n = 0;
    for (int k = 0; k < 4; k++)
        for (int v = 0; v < 7; v++) {
            in.intern_kv({kid[k], vid[v]});
            n++;
        }
    for (int k1 = 0; k1 < 4; k1++)
        for (int k2 = k1 + 1; k2 < 4; k2++)
            for (int v1 = 0; v1 < 7; v1++)
                for (int v2 = 0; v2 < 7; v2++) {
                    in.intern_kv({kid[k1], vid[v1], kid[k2], vid[v2]});
                    n++;
                }
    return n;
}

int mte_generate(mte_engine* e, uint32_t kind, uint32_t n_docs, uint32_t n_ops, const uint32_t* ops_per_doc,
                 uint32_t n_clients, uint64_t seed_base) {
    return mte_generate_ids(e, kind, n_docs, n_ops, ops_per_doc, nullptr, n_clients, seed_base);
}

int mte_generate_ids(mte_engine* e, uint32_t kind, uint32_t n_docs, uint32_t n_ops, const uint32_t* ops_per_doc,
                     const uint32_t* doc_ids, uint32_t n_clients, uint64_t seed_base) {
    if (!e || n_docs == 0 || n_clients == 0 || n_clients >= GEN_MAX_CLIENTS) return MTE_E_ARG;
    e->map_words = MAP_WORDS;  // the generator's property sets hold at most four keys
    if (kind != 2 && kind != 3 && kind != 5) return set_err(e, MTE_E_ARG, "generator kind must be 2, 3 or 5");
    HIP_TRY(e, hipSetDevice(e->device));
    ck_forget(e);  // (a new batch: no checkpoint of the last one may be continued)
    e->hb = HostBatch();
    uint32_t nps = build_generator_props(e);
    std::vector<uint64_t> nops(n_docs), pay(n_docs), pi(n_docs), an(n_docs);
    std::vector<uint8_t> collab(n_docs, 1), has_nl(n_docs, 0);
    for (uint32_t d = 0; d < n_docs; d++) {
        uint64_t n = ops_per_doc ? ops_per_doc[d] : n_ops;
        nops[d] = n;
        pay[d] = 8 * n;
        // kind 3 draws 45 % inserts / 20 % annotates (engine.hpp generate_run): property-map capacity
        // from n/2 and n/4 (the layout adds 4 maps per annotate), not n each -- 5n maps per document
        // (3.2 MB) put the 64k-document C3 batch past the 288 GB of HBM
        pi[d] = kind == 3 ? n / 2 + 64 : 0;
        an[d] = kind == 3 ? n / 4 + 64 : 0;
        e->hb.doc_op_offsets.push_back(e->hb.doc_op_offsets.back() + n);
        e->hb.doc_payload_offsets.push_back(e->hb.doc_payload_offsets.back() + 8 * n);
    }
    int rc;
    // generated docs hover around a 2048-char target length: 64K-unit semispaces are ample
    if ((rc = layout_and_alloc(e, nops, pay, pi, an, collab, has_nl, 65536, nullptr, nullptr, doc_ids))) return rc;
    // generated documents carry no SharedMatrix cell ops: drop an earlier load's cell records, so
    // solo_count and the matrix snapshot never see them (load_cells does the same for a cell-free batch)
    e->cell_recs.clear();
    e->n_cells = 0;
    e->P.cell_pos = e->P.cell_h = e->P.htab = nullptr;
    for (uint32_t d = 0; d < n_docs; d++) e->cfg[d].ht_cap = e->cfg[d].ht_off = 0;
    HIP_TRY(e, e->d_ops.alloc(e->hb.doc_op_offsets.back()));
    HIP_TRY(e, e->d_payload.alloc(e->hb.doc_payload_offsets.back()));
    HIP_TRY(e, hipMemsetAsync(e->d_payload.p, 0, e->d_payload.n * sizeof(uint16_t), e->stream));
    HIP_TRY(e, e->d_first_seen.alloc((size_t)n_docs * GEN_MAX_CLIENTS));
    HIP_TRY(e, hipMemsetAsync(e->d_first_seen.p, 0xFF, (size_t)n_docs * GEN_MAX_CLIENTS * 4, e->stream));
    if ((rc = upload_props(e))) return rc;
    e->P.ops = e->d_ops.p;
    e->P.payload = e->d_payload.p;
    if ((rc = alloc_out_text(e))) return rc;
    e->P.gen_first_seen = e->d_first_seen.p;
    e->P.gen_kind = kind;
    e->P.gen_nclients = n_clients;
    e->P.gen_seed = seed_base;
    e->P.gen_n_propsets = nps;
    e->gen_kind = kind;
    e->emit_tables = false;  // names are known after the generator ran
    // kinds 2 and 5 draw no properties and no '\n'; short ids stay below 1 + n_clients
    e->lean_ok = e->lean_base = kind != 3 && n_clients < 32;
    e->props_rows_ok = true;
    e->rows_wide = n_clients >= 32;  // (and then FULL: lean_ok is false)
    e->ext_needed = e->ext_perm = e->ext_cu = false;
    rc = run_kernel(e, true);
    if (rc) return rc;
    // client names: observer + writers in first-appearance (short id) order
    std::vector<uint32_t> fs((size_t)n_docs * GEN_MAX_CLIENTS);
    HIP_TRY(e, hipMemcpy(fs.data(), e->d_first_seen.p, fs.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t d = 0; d < n_docs; d++) {
        std::vector<std::string> names{"__observer__"};
        for (uint32_t s = 1; s < GEN_MAX_CLIENTS; s++) {
            uint32_t w = fs[(size_t)d * GEN_MAX_CLIENTS + s];
            if (w == 0xFFFFFFFFu) break;
            names.push_back("client-" + std::to_string(w));
        }
        for (auto& nm : names) {
            e->hb.client_names += nm;
            e->hb.client_name_offsets.push_back(e->hb.client_names.size());
        }
        e->hb.doc_client_offsets.push_back(e->hb.doc_client_offsets.back() + (uint32_t)names.size());
    }
    e->generated = true;
    e->host_ops_valid = false;
    return MTE_OK;
}

static int ensure_host_ops(mte_engine* e) {
    if (e->host_ops_valid) return MTE_OK;
    // (the device buffers may be larger than the batch: DevBuf::fit keeps earlier allocations)
    e->hb.ops.resize(e->hb.doc_op_offsets.empty() ? 0 : e->hb.doc_op_offsets.back());
    e->hb.payload.resize(e->hb.doc_payload_offsets.empty() ? 0 : e->hb.doc_payload_offsets.back());
    HIP_TRY(e, hipMemcpy(e->hb.ops.data(), e->d_ops.p, e->hb.ops.size() * sizeof(mte_op), hipMemcpyDeviceToHost));
    HIP_TRY(e, hipMemcpy(e->hb.payload.data(), e->d_payload.p, e->hb.payload.size() * 2, hipMemcpyDeviceToHost));
    e->host_ops_valid = true;
    return MTE_OK;
}

int mte_export_batch(mte_engine* e, mte_batch* out) {
    if (!e || !out) return MTE_E_ARG;
    if (!e->P.ops) return set_err(e, MTE_E_STATE, "nothing loaded");
    int rc = ensure_host_ops(e);
    if (rc) return rc;
    e->hb.view(out);
    return MTE_OK;
}

// ------------------------------------------------------------------------------------------------
// Final-state download and the host-side output walkers.
static int ensure_download(mte_engine* e) {
    if (!e->replayed) return set_err(e, MTE_E_STATE, "no replay results yet");
    if (e->downloaded) return MTE_OK;
    int rc;
    HIP_TRY(e, hipSetDevice(e->device));
    uint32_t ctr[8];
    HIP_TRY(e, hipMemcpy(ctr, e->d_counters.p, sizeof ctr, hipMemcpyDeviceToHost));
    const uint64_t rows = std::min<uint64_t>(ctr[1], e->P.out_cap);
    auto dl = [&](auto& h, auto& d, size_t n) -> int {
        h.resize(n);
        if (n) HIP_TRY(e, hipMemcpy(h.data(), d.p, n * sizeof(h[0]), hipMemcpyDeviceToHost));
        return MTE_OK;
    };
    if (e->P.out_maps && (rc = dl(e->h_maps, e->d_out_maps, rows * e->map_words))) return rc;
    if ((rc = dl(e->h_out_vis, e->d_out_vis, rows))) return rc;
    if ((rc = dl(e->h_out_aux, e->d_out_aux, rows))) return rc;
    if ((rc = dl(e->h_out_ovl, e->d_out_ovl, rows))) return rc;
    if (e->P.out_ovl2) {
        if ((rc = dl(e->h_out_ovl2, e->d_out_ovl2, rows))) return rc;
    } else {
        e->h_out_ovl2.clear();
    }
    uint64_t units;
    memcpy(&units, ctr + 6, sizeof units);
    if ((rc = dl(e->h_out_text, e->d_out_text, std::min<uint64_t>(units, e->P.out_text_cap)))) return rc;
    e->downloaded = true;
    return MTE_OK;
}

namespace {
struct SegView {
    uint32_t kind;  // 0 text, 1 marker, 2 permutation run
    uint32_t len;
    int32_t seq, client, rseq, rclient;
    bool removed;
    uint64_t ovl, ovl2;  // removedClientOverlap: clients 0..63, 64..127
    uint32_t props;
    uint32_t reftype;
    const uint16_t* text;
};

struct DocView {
    const mte_engine* e;
    uint32_t d;
    std::vector<SegView> segs;
    void build() {
        const DocCfg& c = e->cfg[d];
        const DocRes& r = e->res[d];
        const uint16_t* txt = e->h_out_text.data() + r.text_off;  // gathered by Engine::finish
        if (r.status || (uint64_t)r.out_off + r.n_segs > e->h_out_vis.size()) return;
        for (uint32_t q = 0; q < r.n_segs; q++) {
            {
                const uint64_t i = (uint64_t)r.out_off + q;
                uint4 v = e->h_out_vis[i];
                uint4 a = e->h_out_aux[i];
                uint2 t = make_uint2(a.y, a.z);
                SegView sv;
                sv.kind = (v.w & F_MARKER) ? 1 : (v.w & F_PERM) ? 2 : 0;
                sv.len = v.x;
                sv.seq = (int32_t)v.y;
                sv.removed = (v.w & F_REMOVED) != 0;
                sv.rseq = (int32_t)v.z;
                sv.client = c.collab ? (int32_t)(v.w & 0xff) : -1;
                sv.rclient = c.collab ? (int32_t)((v.w >> 8) & 0xff) : -1;
                sv.ovl = e->h_out_ovl[i];
                sv.ovl2 = i < e->h_out_ovl2.size() ? e->h_out_ovl2[i] : 0ull;
                sv.props = a.x ? (uint32_t)(i + 1) : 0u;
                // bits 16..31 of a marker's word: its tag; a permutation run's word: its start handle
                sv.reftype = sv.kind == 1 ? (t.x & 0xFFFFu) : sv.kind == 2 ? t.x : 0;
                sv.text = sv.kind ? nullptr : txt + t.x;
                segs.push_back(sv);
            }
        }
    }
    std::string long_id(int32_t shortId) const {
        if (shortId < 0) return "original";
        return e->hb.client(d, (uint32_t)shortId);
    }
    // SegView::props: 1 + the row's index in the output pool (its map was copied there), 0 = none
    const uint32_t* map(uint32_t id) const { return e->h_maps.data() + (uint64_t)(id - 1) * e->map_words; }
    // JSON of a property map in JS key order (integer-like keys ascending first, then insertion order)
    void props_json(std::string& o, uint32_t id) const {
        const uint32_t* m = map(id);
        uint32_t n = m[0];
        std::vector<std::pair<uint32_t, uint32_t>> idx;
        std::vector<uint32_t> rest;
        for (uint32_t i = 0; i < n; i++) {
            uint32_t k = m[1 + 2 * i];
            if (e->key_is_index[k]) idx.emplace_back(e->key_index[k], i);
            else rest.push_back(i);
        }
        std::sort(idx.begin(), idx.end());
        o.push_back('{');
        bool first = true;
        auto emit = [&](uint32_t i) {
            if (!first) o.push_back(',');
            first = false;
            o += e->hb.key(m[1 + 2 * i]);
            o.push_back(':');
            o += e->hb.val(m[2 + 2 * i]);
        };
        for (auto& p : idx) emit(p.second);
        for (uint32_t i : rest) emit(i);
        o.push_back('}');
    }
    bool val_match(uint32_t a, uint32_t b) const {
        if (a == b) return true;
        if (e->val_flags[b] & 2u) {
            uint32_t j = e->val_objidx[b];
            return j != NONE && ((e->val_objmatch[a] >> j) & 1ull);
        }
        return false;
    }
    bool match_props(uint32_t a, uint32_t b) const {
        if (a == b) return true;
        if (!a || !b) return false;
        const uint32_t *ma = map(a), *mb = map(b);
        if (ma[0] != mb[0]) return false;
        for (uint32_t i = 0; i < ma[0]; i++) {
            bool found = false;
            for (uint32_t q = 0; q < mb[0]; q++)
                if (mb[1 + 2 * q] == ma[1 + 2 * i]) {
                    if (!val_match(ma[2 + 2 * i], mb[2 + 2 * q])) return false;
                    found = true;
                }
            if (!found) return false;
        }
        return true;
    }
    void seg_json(std::string& o, const SegView& s, const std::u16string* text) const {
        if (s.kind == 1) {
            o += "{\"marker\":{\"refType\":" + json::number((double)s.reftype) + "}";
            if (s.props) {
                o += ",\"props\":";
                props_json(o, s.props);
            }
            o += "}";
        } else if (s.props) {
            o += "{\"text\":";
            if (text) json::quote(o, *text); else json::quote(o, (const char16_t*)s.text, s.len);
            o += ",\"props\":";
            props_json(o, s.props);
            o += "}";
        } else {
            if (text) json::quote(o, *text); else json::quote(o, (const char16_t*)s.text, s.len);
        }
    }
    std::u16string text() const {
        std::u16string t;
        for (auto& s : segs)
            if (!s.kind && !s.removed) t.append((const char16_t*)s.text, s.len);
        return t;
    }
};

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) {
        h ^= b[i];
        h *= 0x100000001b3ull;
    }
    return h;
}
}  // namespace

static int doc_view(mte_engine* e, uint32_t doc, DocView& v) {
    if (!e) return MTE_E_ARG;
    int rc = ensure_download(e);
    if (rc) return rc;
    if (doc >= e->P.n_docs) return set_err(e, MTE_E_RANGE, "doc index out of range");
    v.e = e;
    v.d = doc;
    v.build();
    return MTE_OK;
}

int mte_doc_status(mte_engine* e, uint32_t doc, int32_t* code, int64_t* failing_seq) {
    if (!e) return MTE_E_ARG;
    if (!e->replayed) return set_err(e, MTE_E_STATE, "no replay results yet");
    if (doc >= e->res.size()) return set_err(e, MTE_E_RANGE, "doc index out of range");
    if (code) *code = e->res[doc].status;
    if (failing_seq) *failing_seq = e->res[doc].failing_seq;
    return MTE_OK;
}

int mte_text(mte_engine* e, uint32_t doc, uint16_t* buf, size_t cap, size_t* len) {
    DocView v;
    int rc = doc_view(e, doc, v);
    if (rc) return rc;
    std::u16string t = v.text();
    if (len) *len = t.size();
    if (!buf) return MTE_OK;
    if (cap < t.size()) return MTE_E_RANGE;
    memcpy(buf, t.data(), t.size() * 2);
    return MTE_OK;
}

int mte_length(mte_engine* e, uint32_t doc, uint64_t* len) {
    DocView v;
    int rc = doc_view(e, doc, v);
    if (rc) return rc;
    uint64_t n = 0;
    for (auto& sg : v.segs)
        if (!sg.removed) n += sg.len;  // a marker counts 1 (Marker.cachedLength, mergeTree.ts:649)
    if (len) *len = n;
    return MTE_OK;
}

int mte_segments(mte_engine* e, uint32_t doc, mte_seg_row* rows, size_t cap, size_t* n) {
    DocView v;
    int rc = doc_view(e, doc, v);
    if (rc) return rc;
    if (n) *n = v.segs.size();
    if (!rows) return MTE_OK;
    if (cap < v.segs.size()) return MTE_E_RANGE;
    uint32_t off = 0;
    for (size_t i = 0; i < v.segs.size(); i++) {
        const SegView& s = v.segs[i];
        mte_seg_row& r = rows[i];
        r.kind = s.kind;
        r.len = s.len;
        r.seq = s.seq;
        r.client = s.client;
        r.removed_seq = s.removed ? s.rseq : INT32_MIN;
        r.removed_client = s.removed ? s.rclient : -1;
        r.overlap_mask = s.ovl;
        r.text_off = off;
        r.ref_type = s.reftype;
        if (!s.kind) off += s.len;
    }
    return MTE_OK;
}

// Extra (non-header) helper used by the Python mirror: full segment dump as JSON rows.
int mte_segments_json(mte_engine* e, uint32_t doc, char* buf, size_t cap, size_t* len) {
    DocView v;
    int rc = doc_view(e, doc, v);
    if (rc) return rc;
    std::string o = "[";
    for (size_t i = 0; i < v.segs.size(); i++) {
        const SegView& s = v.segs[i];
        if (i) o += ",";
        o += "{\"kind\":";
        o += s.kind == 1 ? "\"M\"" : s.kind == 2 ? "\"P\"" : "\"T\"";
        if (s.kind == 1) o += ",\"refType\":" + std::to_string(s.reftype);
        else if (s.kind == 2) o += ",\"start\":" + std::to_string(s.reftype ? (int64_t)s.reftype : (int64_t)INT32_MIN);
        else {
            o += ",\"text\":";
            json::quote(o, (const char16_t*)s.text, s.len);
        }
        o += ",\"len\":" + std::to_string(s.len) + ",\"seq\":" + std::to_string(s.seq) + ",\"client\":";
        std::u16string cu;
        std::string c = v.long_id(s.client);
        json::decode_utf8(c.data(), c.size(), cu);
        json::quote(o, cu);
        if (s.removed) {
            o += ",\"removedSeq\":" + std::to_string(s.rseq) + ",\"removedClient\":";
            std::string rc2 = v.long_id(s.rclient);
            std::u16string ru;
            json::decode_utf8(rc2.data(), rc2.size(), ru);
            json::quote(o, ru);
        }
        o += ",\"overlap\":[";
        bool first = true;
        for (int b = 0; b < 128; b++)
            if ((b < 64 ? s.ovl >> b : s.ovl2 >> (b - 64)) & 1ull) {
                if (!first) o += ",";
                first = false;
                std::string nm = v.long_id(b);
                std::u16string nu;
                json::decode_utf8(nm.data(), nm.size(), nu);
                json::quote(o, nu);
            }
        o += "],\"props\":";
        if (s.props) {
            std::string pj;
            v.props_json(pj, s.props);
            std::u16string pu;
            json::decode_utf8(pj.data(), pj.size(), pu);
            json::quote(o, pu);
        } else {
            o += "null";
        }
        o += "}";
    }
    o += "]";
    if (len) *len = o.size();
    if (!buf) return MTE_OK;
    if (cap < o.size()) return MTE_E_RANGE;
    memcpy(buf, o.data(), o.size());
    return MTE_OK;
}

// SharedSegmentSequence.snapshotCore (sequence.ts:413-438): the interval-collection blob "header"
// (MapKernel.serialize of no collections: "{}"; interval ops are outside the path) and the merge-tree
// ITree as "content".
// The SnapshotV1 blobs the device wrote (emit.hip), downloaded once per replay on first use.
static int ensure_emit_download(mte_engine* e) {
    if (e->emit_downloaded) return MTE_OK;
    HIP_TRY(e, hipSetDevice(e->device));
    for (auto& pl : e->pool) {
        pl.h.resize(pl.used);
        pl.h_blob_off.resize(pl.blobs);
        if (pl.used) HIP_TRY(e, hipMemcpy(pl.h.data(), pl.out.p, pl.used, hipMemcpyDeviceToHost));
        if (pl.blobs) HIP_TRY(e, hipMemcpy(pl.h_blob_off.data(), pl.blob_off.p, pl.blobs * 8, hipMemcpyDeviceToHost));
    }
    e->emit_downloaded = true;
    return MTE_OK;
}
// Document d's blobs as (pointer, length); MTE_E_STATE when it has none (failed, or emission off).
static int doc_blobs(mte_engine* e, uint32_t d, std::vector<std::pair<const char*, size_t>>& out) {
    out.clear();
    int rc = ensure_emit_download(e);
    if (rc) return rc;
    if (d >= e->emit_pool_of.size() || e->emit_pool_of[d] == 255)
        return set_err(e, MTE_E_STATE, "no SnapshotV1 for this document (replay failed, or option emit is 0)");
    const auto& pl = e->pool[e->emit_pool_of[d]];
    const uint64_t o = e->h_out_off[d], n = e->h_emit_size[d], b0 = e->h_blob_base[d], nb = e->h_nblobs[d];
    for (uint64_t b = 0; b < nb; b++) {
        const uint64_t s0 = pl.h_blob_off[b0 + b], s1 = b + 1 < nb ? pl.h_blob_off[b0 + b + 1] : n;
        out.emplace_back(pl.h.data() + o + s0, (size_t)(s1 - s0));
    }
    return MTE_OK;
}

static int legacy_tree(mte_engine* e, uint32_t doc, const char* catch_up_name, std::string& o);

int mte_snapshot_shared_string(mte_engine* e, uint32_t doc, char* buf, size_t cap, size_t* len) {
    if (!e) return MTE_E_ARG;
    size_t n = 0;
    int rc;
    std::string inner;
    if (e->emitted_legacy) {
        if (doc >= e->P.n_docs) return set_err(e, MTE_E_RANGE, "doc index out of range");
        if ((rc = legacy_tree(e, doc, nullptr, inner))) return rc;
    } else {
        if ((rc = mte_snapshot_v1(e, doc, nullptr, 0, &n, nullptr))) return rc;
        inner.assign(n, '\0');
        if ((rc = mte_snapshot_v1(e, doc, &inner[0], n, &n, nullptr))) return rc;
    }
    std::string o = "{\"entries\":[{\"mode\":\"100644\",\"path\":\"header\",\"type\":\"Blob\",\"value\":"
                    "{\"contents\":\"{}\",\"encoding\":\"utf-8\"}},{\"mode\":\"040000\",\"path\":\"content\","
                    "\"type\":\"Tree\",\"value\":" + inner + "}],\"id\":null}";
    if (len) *len = o.size();
    if (!buf) return MTE_OK;
    if (cap < o.size()) return MTE_E_RANGE;
    memcpy(buf, o.data(), o.size());
    return MTE_OK;
}

int mte_snapshot_v1(mte_engine* e, uint32_t doc, char* buf, size_t cap, size_t* len, uint32_t* n_blobs) {
    if (!e) return MTE_E_ARG;
    if (doc >= e->P.n_docs) return set_err(e, MTE_E_RANGE, "doc index out of range");
    if (e->emitted_legacy) return set_err(e, MTE_E_STATE, "the last replay emitted SnapshotLegacy (snapshot_format 1)");
    std::vector<std::pair<const char*, size_t>> blobs;
    int rc = doc_blobs(e, doc, blobs);
    if (rc) return rc;
    std::string o = "{\"entries\":[";
    for (size_t i = 0; i < blobs.size(); i++) {
        if (i) o += ",";
        std::string path = i == 0 ? "header" : "body_" + std::to_string(i - 1);
        o += "{\"mode\":\"100644\",\"path\":\"" + path + "\",\"type\":\"Blob\",\"value\":{\"contents\":";
        std::u16string bu;
        json::decode_utf8(blobs[i].first, blobs[i].second, bu);
        json::quote(o, bu);
        o += ",\"encoding\":\"utf-8\"}}";
    }
    o += "],\"id\":null}";
    if (n_blobs) *n_blobs = (uint32_t)blobs.size();
    if (len) *len = o.size();
    if (!buf) return MTE_OK;
    if (cap < o.size()) return MTE_E_RANGE;
    memcpy(buf, o.data(), o.size());
    return MTE_OK;
}

// SparseArray2D's Morton keys (sparsearray2d.ts:10-41): the bits of a 16-bit row / col interleaved,
// row bits odd, col bits even.
static uint32_t interlace16(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}
static uint32_t morton2x16(uint32_t row, uint32_t col) { return (interlace16(row) << 1) | interlace16(col); }

// One SparseArray2D tile (256 entries): sub-tiles above the last level, values (val ids) in it.
struct CellTile {
    std::map<uint32_t, std::unique_ptr<CellTile>> sub;
    std::map<uint32_t, uint32_t> val;  // NONE: cleared (undefined)
    CellTile* at(uint32_t k) {
        std::unique_ptr<CellTile>& t = sub[k];
        if (!t) t.reset(new CellTile());
        return t.get();
    }
};
static void cell_tile_json(std::string& o, const CellTile& t, int depth, const HostBatch& hb) {
    o += '[';
    for (uint32_t i = 0; i < 256; i++) {
        if (i) o += ',';
        if (depth < 3) {
            auto it = t.sub.find(i);
            if (it == t.sub.end()) o += "null";
            else cell_tile_json(o, *it->second, depth + 1, hb);
        } else {
            auto it = t.val.find(i);
            if (it == t.val.end() || it->second == NONE) o += "null";
            else o.append(hb.val_text, hb.val_offsets[it->second], hb.val_offsets[it->second + 1] - hb.val_offsets[it->second]);
        }
    }
    o += ']';
}

// A vector's HandleTable as the device left it: the handles array (HandleTable.snapshot,
// handletable.ts:80-82) and the seq of each handle's last free.
static int read_handle_table(mte_engine* e, uint32_t doc, std::vector<uint32_t>& handles, std::vector<uint32_t>& freed) {
    handles.assign(1, 1u);  // new HandleTable(): [1]
    freed.clear();
    const DocCfg& c = e->cfg[doc];
    if (!c.ht_cap || !e->d_htab.p) return MTE_OK;
    std::vector<uint32_t> w(1 + 2 * (size_t)c.ht_cap);
    HIP_TRY(e, hipMemcpy(w.data(), e->d_htab.p + c.ht_off, w.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    const uint32_t len = w[0];
    if (len < 1 || len > c.ht_cap) return set_err(e, MTE_E_STATE, "handle table out of range");
    handles.assign(w.begin() + 1, w.begin() + 1 + len);
    freed.assign(w.begin() + 1 + c.ht_cap, w.end());
    return MTE_OK;
}

// SharedMatrix.snapshotCore (matrix.ts:405-430) over PermutationVector.snapshot (permutationvector.ts:260-273).
// The segments trees are the vectors' SnapshotV1 (the emission kernels); the handle tables and the
// cells come from the replay's device results: a gated set wrote cell (row handle, col handle) at its
// seq, and a zamboni UNLINK of the row (col) handle after that seq cleared it (onRowHandlesRecycled /
// onColHandlesRecycled, matrix.ts:626-640: clearRows / clearCols leave the tiles in place).
int mte_snapshot_matrix(mte_engine* e, uint32_t rows_doc, uint32_t cols_doc, char* buf, size_t cap, size_t* len) {
    if (!e) return MTE_E_ARG;
    if (rows_doc >= e->P.n_docs || cols_doc >= e->P.n_docs) return MTE_E_RANGE;
    std::string o = "{\"entries\":[";
    const uint32_t docs[2] = {rows_doc, cols_doc};
    std::vector<uint32_t> handles[2], freed[2];
    for (int i = 0; i < 2; i++) {
        size_t n = 0;
        int rc = mte_snapshot_v1(e, docs[i], nullptr, 0, &n, nullptr);
        if (rc) return rc;
        std::string seg(n, '\0');
        if ((rc = mte_snapshot_v1(e, docs[i], &seg[0], n, &n, nullptr))) return rc;
        if ((rc = read_handle_table(e, docs[i], handles[i], freed[i]))) return rc;
        std::string ht = "[";
        for (size_t q = 0; q < handles[i].size(); q++) {
            if (q) ht += ',';
            ht += std::to_string(handles[i][q]);
        }
        ht += ']';
        o += std::string("{\"mode\":\"040000\",\"path\":\"") + (i ? "cols" : "rows") + "\",\"type\":\"Tree\",\"value\":";
        o += "{\"entries\":[{\"mode\":\"040000\",\"path\":\"segments\",\"type\":\"Tree\",\"value\":" + seg +
             "},{\"mode\":\"100644\",\"path\":\"handleTable\",\"type\":\"Blob\",\"value\":{\"contents\":\"" + ht +
             "\",\"encoding\":\"utf-8\"}}],\"id\":null}},";
    }
    // cells: JSON.stringify([cells.snapshot(), pending.snapshot()]); pending stays [undefined] for an
    // observer (it only holds unACKed local writes)
    std::map<uint32_t, CellTile> root;  // keyHi -> level-0 tile
    uint32_t root_len = 1;
    // a matrix loaded from a summary starts from its SparseArray2D (SparseArray2D.load keeps every
    // tile); a loaded cell is cleared when a zamboni of the replay freed its row or col handle
    auto mi = e->mx_init.find(rows_doc);
    if (mi != e->mx_init.end()) {
        root_len = mi->second.root_len;
        for (const auto& t : mi->second.tiles) {
            CellTile* x = &root[t[0]];
            for (uint32_t dd = 0; dd < t[1]; dd++) x = x->at((t[2] >> (16 - 8 * dd)) & 0xFFu);
        }
        for (const auto& c : mi->second.cells) {
            const uint32_t rh = c[0], ch = c[1];
            const uint32_t hi = morton2x16(rh >> 16, ch >> 16), lo = morton2x16(rh, ch);
            CellTile* t = root[hi].at(lo >> 24)->at((lo >> 16) & 0xFFu)->at((lo >> 8) & 0xFFu);
            const bool gone = (rh < freed[0].size() && freed[0][rh]) || (ch < freed[1].size() && freed[1][ch]);
            t->val[lo & 0xFFu] = gone ? NONE : c[2];
        }
    }
    auto it = e->cell_recs.find(rows_doc);
    if (it != e->cell_recs.end() && e->n_cells) {
        std::vector<uint32_t> h(2 * e->n_cells);
        HIP_TRY(e, hipMemcpy(h.data(), e->d_cell_h.p, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        for (const mte_engine::CellRec& r : it->second) {
            const uint32_t rh = h[2 * (size_t)r.cell], ch = h[2 * (size_t)r.cell + 1];
            if (!rh || !ch) continue;  // adjustPosition undefined in one of the vectors
            // setCell (sparsearray2d.ts:89-98): getLevel creates every tile on the path
            const uint32_t hi = morton2x16(rh >> 16, ch >> 16), lo = morton2x16(rh, ch);
            CellTile* t = root[hi].at(lo >> 24)->at((lo >> 16) & 0xFFu)->at((lo >> 8) & 0xFFu);
            const bool gone = (rh < freed[0].size() && (int32_t)freed[0][rh] > r.seq) ||
                              (ch < freed[1].size() && (int32_t)freed[1][ch] > r.seq);
            t->val[lo & 0xFFu] = gone ? NONE : r.val;
        }
    }
    std::string cells = "[[";
    if (root.empty() && root_len <= 1) {
        cells += "null";
    } else {
        const uint32_t top = std::max<uint32_t>(root.empty() ? 0u : root.rbegin()->first, root_len - 1);
        if (top > (1u << 20)) return set_err(e, MTE_E_UNSUPPORTED, "cell handles beyond 2^26");
        for (uint32_t k = 0; k <= top; k++) {
            if (k) cells += ',';
            auto r = root.find(k);
            if (r == root.end()) cells += "null";
            else cell_tile_json(cells, r->second, 0, e->hb);
        }
    }
    cells += "],[null]]";
    std::u16string cu;
    json::decode_utf8(cells.data(), cells.size(), cu);
    o += "{\"mode\":\"100644\",\"path\":\"cells\",\"type\":\"Blob\",\"value\":{\"contents\":";
    json::quote(o, cu);
    o += ",\"encoding\":\"utf-8\"}}],\"id\":null}";
    if (len) *len = o.size();
    if (!buf) return MTE_OK;
    if (cap < o.size()) return MTE_E_RANGE;
    memcpy(buf, o.data(), o.size());
    return MTE_OK;
}

// ---- SnapshotLegacy catch-up messages (sequence.ts:584-650) -------------------------------------
static int num_field(const json::Value& o, const char16_t* k, int32_t* out);
static void set_member(json::Value& o, const char16_t* k, json::Value v) {
    for (auto& m : o.members)
        if (m.first == k) {
            m.second = std::move(v);
            return;
        }
    o.members.emplace_back(k, std::move(v));
}
static json::Value jobj() {
    json::Value v;
    v.kind = json::Value::Object;
    return v;
}
static json::Value jnumv(double x) {
    json::Value v;
    v.kind = json::Value::Number;
    v.num = x;
    return v;
}
// one property map of document d from the device (map_words words: count, then (key, value) ids)
static int read_map(mte_engine* e, uint32_t d, uint32_t id, std::vector<std::pair<uint32_t, uint32_t>>& kv) {
    kv.clear();
    if (id == 0) return MTE_OK;
    const bool rr0 = d < e->map_rr_off.size() && e->map_rr_off[d] != UINT64_MAX;
    if (id >= (rr0 ? e->map_rr_cap[d] : e->cfg[d].map_cap))
        return set_err(e, MTE_E_STATE, "catch-up: property map id out of range");
    std::vector<uint32_t> w(e->map_words);
    const bool rr = d < e->map_rr_off.size() && e->map_rr_off[d] != UINT64_MAX;
    const uint32_t* base = rr ? e->d_maps_rr.p + e->map_rr_off[d] * e->map_words : e->d_maps.p + e->cfg[d].map_off * e->map_words;
    HIP_TRY(e, hipMemcpy(w.data(), base + (uint64_t)id * e->map_words, w.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < std::min<uint32_t>(w[0], (e->map_words - 1) / 2); i++) kv.emplace_back(w[1 + 2 * i], w[2 + 2 * i]);
    return MTE_OK;
}
static json::Value parse_text(const std::string& t) { return json::parse(t.data(), t.size()); }
// propertyDeltas keys of an annotate (segmentPropertiesManager.ts:65-106): with rewrite, the segment's
// keys (Object.keys order) whose new value is falsy or absent, then the op's keys; each key mapped to
// the segment's value after the op, or null (createOpsFromDelta, sequence.ts:62-81)
static int annotate_props(mte_engine* e, uint32_t d, const mte_op& op, uint32_t nmap, uint32_t omap, json::Value& props) {
    const HostBatch& hb = e->hb;
    std::vector<std::pair<uint32_t, uint32_t>> nk, ok;
    int rc;
    if ((rc = read_map(e, d, nmap, nk)) || (rc = read_map(e, d, omap, ok))) return rc;
    std::vector<uint32_t> keys;
    const mte_propset ps = op.props < hb.propsets.size() ? hb.propsets[op.props] : mte_propset{0, 0};
    auto in_new = [&](uint32_t k, uint32_t* v) {
        for (uint32_t q = 0; q < ps.count; q++)
            if (hb.prop_keys[ps.first + q] == k) {
                *v = hb.prop_vals[ps.first + q];
                return true;
            }
        return false;
    };
    if (op.flags & MTE_F_REWRITE) {
        std::vector<size_t> idx(ok.size());
        for (size_t i = 0; i < ok.size(); i++) idx[i] = i;
        std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {  // JS own-key order
            const uint32_t ka = ok[a].first, kb = ok[b].first;
            const bool ia = e->key_is_index[ka], ib = e->key_is_index[kb];
            if (ia != ib) return ia;
            return ia && e->key_index[ka] < e->key_index[kb];
        });
        for (size_t i : idx) {
            uint32_t v = 0;
            if (!in_new(ok[i].first, &v) || (e->val_flags[v] & 1u)) keys.push_back(ok[i].first);
        }
    }
    for (uint32_t q = 0; q < ps.count; q++) {
        const uint32_t k = hb.prop_keys[ps.first + q];
        if (std::find(keys.begin(), keys.end(), k) == keys.end()) keys.push_back(k);
    }
    props = jobj();
    for (uint32_t k : keys) {
        json::Value kv = parse_text(hb.key(k));
        json::Value val;  // null
        for (auto& p : nk)
            if (p.first == k) val = parse_text(hb.val(p.second));
        set_member(props, kv.str.c_str(), std::move(val));
    }
    return MTE_OK;
}
// segment.clone().toJSONObject() of an insert op's segment (textSegment.ts:48-54, mergeTree.ts:652-656)
static json::Value insert_seg_json(const mte_engine* e, uint32_t d, const mte_op& op) {
    const HostBatch& hb = e->hb;
    json::Value props = jobj();
    if (op.props && op.props < hb.propsets.size()) {
        const mte_propset ps = hb.propsets[op.props];
        for (uint32_t q = 0; q < ps.count; q++) {
            const uint32_t v = hb.prop_vals[ps.first + q];
            if (v == 0) continue;  // null deletes
            json::Value kv = parse_text(hb.key(hb.prop_keys[ps.first + q]));
            set_member(props, kv.str.c_str(), parse_text(hb.val(v)));
        }
    }
    json::Value seg;
    if (op.type == MTE_OP_INSERT_MARKER) {
        seg = jobj();
        json::Value mk = jobj();
        set_member(mk, u"refType", jnumv((double)(op.b & 0xFFFFu)));
        set_member(seg, u"marker", std::move(mk));
        if (op.props) set_member(seg, u"props", std::move(props));
        return seg;
    }
    json::Value text;
    text.kind = json::Value::String;
    const uint64_t p0 = hb.doc_payload_offsets[d] + (uint64_t)op.a;
    text.str.assign((const char16_t*)hb.payload.data() + p0, op.b);
    if (!op.props) return text;
    seg = jobj();
    set_member(seg, u"text", std::move(text));
    set_member(seg, u"props", std::move(props));
    return seg;
}
// The catch-up blob of document d: JSON.stringify(messagesSinceMSNChange) at snapshot time.
static int catch_up_json(mte_engine* e, uint32_t d, std::string& out) {
    if (int rc = ensure_host_ops(e)) return rc;
    const HostBatch& hb = e->hb;
    const DocRes& r = e->res[d];
    const int32_t minSeq = r.min_seq;
    const uint64_t m0 = hb.doc_msg_offsets[d], m1 = hb.doc_msg_offsets[d + 1];
    const uint64_t op0 = hb.doc_op_offsets[d], nops = hb.doc_op_offsets[d + 1] - op0;
    // every applied op above minSeq must have its message (generated logs have none)
    uint64_t need = 0, have = 0;
    for (uint64_t i = 0; e->cfg[d].collab && i < nops; i++) {  // local (non-collaborative) edits are not messages
        const mte_op& o = hb.ops[op0 + i];
        if ((o.flags & MTE_F_END_OF_MSG) && o.seq > minSeq && o.type <= MTE_OP_INSERT_MARKER) need++;
    }
    std::vector<uint4> rec(2 * (size_t)r.cu_n);
    if (r.cu_n) HIP_TRY(e, hipMemcpy(rec.data(), e->d_cu.p + 2 * e->cfg[d].cu_off, rec.size() * sizeof(uint4), hipMemcpyDeviceToHost));
    out = "[";
    size_t ri = 0;
    bool first = true;
    for (uint64_t i = m0; i < m1; i++) {
        json::Value m;
        try {
            m = parse_text(hb.message(i));
        } catch (std::exception& ex) {
            return set_err(e, MTE_E_PARSE, ex.what());
        }
        int32_t seq = 0, ref = 0;
        num_field(m, u"sequenceNumber", &seq);
        num_field(m, u"referenceSequenceNumber", &ref);
        const uint64_t f0 = hb.msg_first_op[i], f1 = i + 1 < m1 ? hb.msg_first_op[i + 1] : nops;
        while (ri < r.cu_n && rec[2 * ri].x < f0) ri++;
        if (seq <= minSeq) continue;
        have++;
        if (ref != seq - 1) {  // stashMessage = {...message, referenceSequenceNumber, contents}
            std::vector<json::Value> ops;
            for (; ri < r.cu_n && rec[2 * ri].x < f1; ri++) {
                const uint4 a = rec[2 * ri], b = rec[2 * ri + 1];
                const mte_op& op = hb.ops[op0 + a.x];
                const double pos = (double)(int32_t)a.y, len = (double)a.z;
                json::Value* last = ops.empty() ? nullptr : &ops.back();
                if (a.w == 0) {  // createInsertOp(r.position, segment.clone().toJSONObject())
                    json::Value o = jobj();
                    set_member(o, u"pos1", jnumv(pos));
                    set_member(o, u"seg", insert_seg_json(e, d, op));
                    set_member(o, u"type", jnumv(0));
                    ops.push_back(std::move(o));
                } else if (a.w == 1) {  // lastRem?.pos1 === r.position ? lastRem.pos2 += len : a new remove
                    const json::Value* p1 = last ? last->get(u"pos1") : nullptr;
                    if (p1 && p1->kind == json::Value::Number && p1->num == pos) {
                        const json::Value* p2 = last->get(u"pos2");
                        set_member(*last, u"pos2", jnumv(p2 && p2->kind == json::Value::Number ? p2->num + len : NAN));
                    } else {
                        json::Value o = jobj();
                        set_member(o, u"pos1", jnumv(pos));
                        set_member(o, u"pos2", jnumv(pos + len));
                        set_member(o, u"type", jnumv(1));
                        ops.push_back(std::move(o));
                    }
                } else {  // annotate: extend the last one when adjacent with matching props
                    json::Value props;
                    int rc = annotate_props(e, d, op, b.x, b.y, props);
                    if (rc) return rc;
                    const json::Value* p2 = last ? last->get(u"pos2") : nullptr;
                    const json::Value* lp = last ? last->get(u"props") : nullptr;
                    if (p2 && p2->kind == json::Value::Number && p2->num == pos && json::match_properties(lp, &props)) {
                        set_member(*last, u"pos2", jnumv(p2->num + len));
                    } else {
                        json::Value o = jobj();
                        set_member(o, u"pos1", jnumv(pos));
                        set_member(o, u"pos2", jnumv(pos + len));
                        set_member(o, u"props", std::move(props));
                        set_member(o, u"type", jnumv(2));
                        ops.push_back(std::move(o));
                    }
                }
            }
            set_member(m, u"referenceSequenceNumber", jnumv(seq - 1));
            if (ops.size() == 1) {
                set_member(m, u"contents", std::move(ops[0]));
            } else {  // createGroupOp(...ops)
                json::Value g = jobj(), arr;
                arr.kind = json::Value::Array;
                arr.items = std::move(ops);
                set_member(g, u"ops", std::move(arr));
                set_member(g, u"type", jnumv(3));
                set_member(m, u"contents", std::move(g));
            }
        }
        set_member(m, u"minimumSequenceNumber", jnumv(minSeq));  // sequence.ts:590
        if (!first) out += ",";
        first = false;
        json::stringify(out, m);
    }
    out += "]";
    if (have < need)
        return set_err(e, MTE_E_UNSUPPORTED, "legacy catch-up: ops above minSeq without their message JSON (generated log)");
    return MTE_OK;
}
static int legacy_tree(mte_engine* e, uint32_t doc, const char* catch_up_name, std::string& o) {
    if (!e->emitted_legacy) return set_err(e, MTE_E_STATE, "replay with snapshot_format 1 for SnapshotLegacy");
    std::vector<std::pair<const char*, size_t>> blobs;
    int rc = doc_blobs(e, doc, blobs);
    if (rc || (rc = ensure_download(e))) return rc;
    std::string cu;
    if ((rc = catch_up_json(e, doc, cu))) return rc;
    const std::string cname = catch_up_name && *catch_up_name ? catch_up_name : "catchupOps";
    o = "{\"entries\":[";
    auto entry = [&](const std::string& path, const char* p, size_t n) {
        o += "{\"mode\":\"100644\",\"path\":";
        std::u16string pu;
        json::decode_utf8(path.data(), path.size(), pu);
        json::quote(o, pu);
        o += ",\"type\":\"Blob\",\"value\":{\"contents\":";
        std::u16string bu;
        json::decode_utf8(p, n, bu);
        json::quote(o, bu);
        o += ",\"encoding\":\"utf-8\"}}";
    };
    for (size_t i = 0; i < blobs.size(); i++) {
        entry(i == 0 ? "header" : "body", blobs[i].first, blobs[i].second);
        o += ",";
    }
    entry(cname, cu.data(), cu.size());
    o += "],\"id\":null}";
    return MTE_OK;
}
int mte_snapshot_legacy(mte_engine* e, uint32_t doc, const char* catch_up_name, char* buf, size_t cap, size_t* len) {
    if (!e) return MTE_E_ARG;
    if (doc >= e->P.n_docs) return set_err(e, MTE_E_RANGE, "doc index out of range");
    std::string o;
    int rc = legacy_tree(e, doc, catch_up_name, o);
    if (rc) return rc;
    if (len) *len = o.size();
    if (!buf) return MTE_OK;
    if (cap < o.size()) return MTE_E_RANGE;
    memcpy(buf, o.data(), o.size());
    return MTE_OK;
}

int mte_summaries(mte_engine* e, mte_doc_summary* out, size_t cap) {
    if (!e || !out) return MTE_E_ARG;
    int rc = ensure_download(e);
    if (rc) return rc;
    const uint32_t nd = e->P.n_docs;
    if (cap < nd) return MTE_E_RANGE;
    if ((rc = ensure_emit_download(e))) return rc;
    std::atomic<uint32_t> next{0};
    auto work = [&]() {
        std::vector<std::pair<const char*, size_t>> blobs;
        for (uint32_t d; (d = next.fetch_add(1)) < nd;) {
            DocView v;
            v.e = e;
            v.d = d;
            v.build();
            std::u16string t = v.text();
            std::string t8 = json::to_utf8(t.data(), t.size());
            uint64_t h = fnv1a(0xcbf29ce484222325ull, t8.data(), t8.size());
            uint32_t sb = 0;
            if (e->res[d].status == 0 && e->emit_pool_of.size() > d && e->emit_pool_of[d] != 255) {
                const auto& pl = e->pool[e->emit_pool_of[d]];
                const uint64_t o = e->h_out_off[d], n = e->h_emit_size[d], b0 = e->h_blob_base[d], nb = e->h_nblobs[d];
                for (uint64_t b = 0; b < nb; b++) {
                    const uint64_t s0 = pl.h_blob_off[b0 + b], s1 = b + 1 < nb ? pl.h_blob_off[b0 + b + 1] : n;
                    uint8_t z = 0;
                    h = fnv1a(h, &z, 1);
                    h = fnv1a(h, pl.h.data() + o + s0, s1 - s0);
                }
                sb = (uint32_t)n;
            }
            mte_doc_summary& s = out[d];
            s.checksum = h;
            s.ops = e->res[d].ops;
            s.length = (uint32_t)t.size();
            s.segments = (uint32_t)v.segs.size();
            s.snapshot_bytes = sb;
            s.status = e->res[d].status;
            s.doc_id = e->cfg[d].gid;
        }
    };
    run_pool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())), work);
    return MTE_OK;
}

// ------------------------------------------------------------------------------------------------
// The one collective of the path: an all-gather of the per-document summary records over
// RCCL (xGMI on one node). librccl is opened on first use, so hosts that never gather (one GPU, the
// CPU tests) do not need it.
}  // extern "C"
namespace {
struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclGetErrorString) errStr = nullptr;
    bool ok() {
        if (h) return true;
        for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) return false;
        getUniqueId = (decltype(getUniqueId))dlsym(h, "ncclGetUniqueId");
        commInitRank = (decltype(commInitRank))dlsym(h, "ncclCommInitRank");
        commDestroy = (decltype(commDestroy))dlsym(h, "ncclCommDestroy");
        allGather = (decltype(allGather))dlsym(h, "ncclAllGather");
        errStr = (decltype(errStr))dlsym(h, "ncclGetErrorString");
        if (!getUniqueId || !commInitRank || !commDestroy || !allGather || !errStr) {
            dlclose(h);
            h = nullptr;
        }
        return h != nullptr;
    }
};
Rccl& rccl() {
    static Rccl r;
    return r;
}
std::mutex& rccl_mu() {
    static std::mutex m;
    return m;
}
}  // namespace
static_assert(sizeof(ncclUniqueId) == MTE_RCCL_ID_BYTES, "ncclUniqueId size");
extern "C" {

int mte_rccl_unique_id(uint8_t* id) {
    if (!id) return MTE_E_ARG;
    std::lock_guard<std::mutex> g(rccl_mu());
    if (!rccl().ok()) return MTE_E_UNSUPPORTED;
    ncclUniqueId u;
    if (rccl().getUniqueId(&u) != ncclSuccess) return MTE_E_HIP;
    memcpy(id, &u, sizeof u);
    return MTE_OK;
}

int mte_rccl_comm_create(mte_engine* e, const uint8_t* id, int rank, int world, void** comm) {
    if (!e || !id || !comm || world < 1 || rank < 0 || rank >= world) return MTE_E_ARG;
    *comm = nullptr;
    {
        std::lock_guard<std::mutex> g(rccl_mu());
        if (!rccl().ok()) return set_err(e, MTE_E_UNSUPPORTED, "librccl not available");
    }
    HIP_TRY(e, hipSetDevice(e->device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclComm_t c = nullptr;
    ncclResult_t r = rccl().commInitRank(&c, world, u, rank);
    if (r != ncclSuccess) return set_err(e, MTE_E_HIP, std::string("ncclCommInitRank: ") + rccl().errStr(r));
    *comm = (void*)c;
    return MTE_OK;
}

void mte_rccl_comm_destroy(void* comm) {
    if (comm && rccl().ok()) rccl().commDestroy((ncclComm_t)comm);
}

// The gather itself: every rank's records into `res` (rank order). One count all-gather and one
// record all-gather; the caller sizes nothing beforehand.
static int gather_all(mte_engine* e, int rank, int world, void* comm, std::vector<mte_doc_summary>& res) {
    if (!e || world < 1 || rank < 0 || rank >= world || (world > 1 && !comm)) return MTE_E_ARG;
    const size_t nd = e->P.n_docs;
    std::vector<mte_doc_summary> mine(nd);
    int rc = nd ? mte_summaries(e, mine.data(), nd) : MTE_OK;
    if (rc) return rc;
    if (world == 1) {
        res.swap(mine);
        return MTE_OK;
    }
    HIP_TRY(e, hipSetDevice(e->device));
    ncclComm_t c = (ncclComm_t)comm;
    // 1) every rank's record count, 2) the records padded to the largest count
    DevBuf<uint64_t> cnt, all_cnt;
    HIP_TRY(e, cnt.alloc(1));
    HIP_TRY(e, all_cnt.alloc((size_t)world));
    const uint64_t mine_n = nd;
    HIP_TRY(e, hipMemcpyAsync(cnt.p, &mine_n, 8, hipMemcpyHostToDevice, e->stream));
    ncclResult_t r = rccl().allGather(cnt.p, all_cnt.p, 1, ncclUint64, c, e->stream);
    if (r != ncclSuccess) return set_err(e, MTE_E_HIP, std::string("ncclAllGather: ") + rccl().errStr(r));
    std::vector<uint64_t> counts((size_t)world);
    HIP_TRY(e, hipMemcpyAsync(counts.data(), all_cnt.p, 8 * (size_t)world, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    const GatherPlan g = gather_plan(counts.data(), world);
    const size_t words = sizeof(mte_doc_summary) / 8;  // 32-B records as 4 u64 words
    std::vector<mte_doc_summary> blk(g.stride), flat(g.stride * (size_t)world);
    gather_pack(mine.data(), nd, g, blk.data());
    DevBuf<uint64_t> send, recv;
    HIP_TRY(e, send.alloc(g.stride * words));
    HIP_TRY(e, recv.alloc(g.stride * words * (size_t)world));
    HIP_TRY(e, hipMemcpyAsync(send.p, blk.data(), g.stride * sizeof(mte_doc_summary), hipMemcpyHostToDevice, e->stream));
    r = rccl().allGather(send.p, recv.p, g.stride * words, ncclUint64, c, e->stream);
    if (r != ncclSuccess) return set_err(e, MTE_E_HIP, std::string("ncclAllGather: ") + rccl().errStr(r));
    HIP_TRY(e, hipMemcpyAsync(flat.data(), recv.p, flat.size() * sizeof(mte_doc_summary), hipMemcpyDeviceToHost,
                              e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    res.resize(g.total);
    gather_concat(flat.data(), counts.data(), world, g, res.data());
    return MTE_OK;
}

int mte_gather_summaries(mte_engine* e, int rank, int world, void* comm, mte_doc_summary* out, size_t cap,
                         size_t* n) {
    if (!e || world < 1 || rank < 0 || rank >= world || (world > 1 && !comm)) return MTE_E_ARG;
    if (!out && world == 1) {  // size query on one rank: no collective
        if (n) *n = e->P.n_docs;
        return MTE_OK;
    }
    // (with world > 1 a size query runs the full record all-gather, like the call that follows it:
    // mte_gather_summaries_alloc does both in one collective)
    std::vector<mte_doc_summary> res;
    if (int rc = gather_all(e, rank, world, comm, res)) return rc;
    if (n) *n = res.size();
    if (!out) return MTE_OK;
    if (cap < res.size()) return MTE_E_RANGE;
    std::copy(res.begin(), res.end(), out);
    return MTE_OK;
}

int mte_gather_summaries_alloc(mte_engine* e, int rank, int world, void* comm, mte_doc_summary** out, size_t* n) {
    if (!out || !n) return MTE_E_ARG;
    *out = nullptr;
    *n = 0;
    std::vector<mte_doc_summary> res;
    if (int rc = gather_all(e, rank, world, comm, res)) return rc;
    void* p = malloc(res.empty() ? 1 : res.size() * sizeof(mte_doc_summary));
    if (!p) return set_err(e, MTE_E_NOMEM, "gather buffer");
    if (!res.empty()) memcpy(p, res.data(), res.size() * sizeof(mte_doc_summary));
    *out = (mte_doc_summary*)p;
    *n = res.size();
    return MTE_OK;
}

void mte_free(void* p) { free(p); }

// Extra helpers (not part of include/mte.h's contract; used by tests / bench for diagnostics).
int mte_doc_result(mte_engine* e, uint32_t doc, void* out, size_t sz) {
    if (!e || !e->replayed || doc >= e->res.size() || sz < sizeof(DocRes)) return MTE_E_ARG;
    memcpy(out, &e->res[doc], sizeof(DocRes));
    return MTE_OK;
}
// Diagnostics of the last replay/generate: documents that outgrew the LDS plan and ran the
// HBM-resident pass, and the two passes' kernel times.
int mte_run_info(mte_engine* e, uint32_t* spilled, double* lds_ms, double* hbm_ms, uint64_t* out_rows,
                 uint32_t* continued) {
    if (!e) return MTE_E_ARG;
    if (continued) *continued = e->last_continued;
    uint32_t ctr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (e->d_counters.p) HIP_TRY(e, hipMemcpy(ctr, e->d_counters.p, sizeof ctr, hipMemcpyDeviceToHost));
    if (spilled) *spilled = e->last_spilled;
    if (lds_ms) *lds_ms = e->last_lds_ms;
    if (hbm_ms) *hbm_ms = e->last_hbm_ms;
    if (out_rows) *out_rows = ctr[1];
    return MTE_OK;
}
// Phase cycle counters of the last run (libmte built with MTE_PROFILE; zeros otherwise):
// PROF_SLOTS u64 per document (engine.hpp ProfSlot).
int mte_profile(mte_engine* e, uint64_t* out, size_t cap) {
    if (!e || !out) return MTE_E_ARG;
    size_t n = (size_t)e->P.n_docs * PROF_SLOTS;
    if (cap < n) return MTE_E_RANGE;
    HIP_TRY(e, hipMemcpy(out, e->d_prof.p, n * 8, hipMemcpyDeviceToHost));
    return MTE_OK;
}
// Engine options (tests / tuning): "force_hbm" (1 = HBM-resident waves only), "pool_limit" (LDS
// leaf blocks usable per CU; 0 = all), "hbm_waves_per_cu" (HBM-resident waves beside each LDS
// workgroup; 0 = LDS waves only), "slot_budget_mb" (HBM for per-wave slots).
int mte_set_option(mte_engine* e, const char* key, int64_t value) {
    if (!e || !key) return MTE_E_ARG;
    std::string k(key);
    if (k == "force_hbm") e->force_hbm = value != 0;
    else if (k == "pool_limit") e->pool_limit = (uint32_t)std::max<int64_t>(0, value);
    else if (k == "hbm_waves_per_cu") {
        e->hbm_waves_per_cu = (uint32_t)std::min<int64_t>(std::max<int64_t>(0, value), 32);
        e->hbm_waves_set = true;
    }
    else if (k == "slot_budget_mb") e->slot_budget = (uint64_t)std::max<int64_t>(1, value) << 20;
    else if (k == "slot_ops_cap") e->slot_ops_cap = (uint64_t)std::max<int64_t>(64, value);  // next load
    else if (k == "slot_blk_limit") e->slot_blk_limit = (uint32_t)std::max<int64_t>(0, value);  // next load
    else if (k == "doc_id_base") e->doc_id_base = (uint64_t)std::max<int64_t>(0, value);  // next load
    else if (k == "solo_max") e->solo_max = (uint32_t)std::max<int64_t>(0, value);
    else if (k == "solo_min_ops") e->solo_min_ops = (uint64_t)std::max<int64_t>(1, value);
    else if (k == "lean") e->lean_opt = value != 0;
    else if (k == "reg_solo") e->reg_solo = value != 0;
    else if (k == "reg_lb_limit") e->reg_lb_limit = (uint32_t)std::max<int64_t>(0, value);
    else if (k == "emit") e->emit_opt = value != 0;  // SnapshotV1 emission on the device after replay
    else if (k == "xcd_align") e->xcd_align = value != 0;
    else if (k == "solo_gate") e->solo_gate = value != 0;
    else if (k == "rows_bulk") e->rows_bulk = value < 0 ? -1 : value == 0 ? 0 : value >= 12 ? 12 : value >= 8 ? 8 : 4;  // lean bulk on k_rows
    else if (k == "snapshot_format") e->legacy = value == 1;  // mte_config.snapshot_format
    else if (k == "rows_pool") e->rows_pool_lim = (uint32_t)std::max<int64_t>(0, value);  // k_rows pool rows per CU (0 = all)
    else if (k == "rows_mixed") e->rows_mixed = (int)std::min<int64_t>(std::max<int64_t>(value, 0), 2);
    else if (k == "retain") {  // incremental replay: checkpoints kept for a later pass over extended logs
        e->retain = value != 0;
        if (!e->retain) ck_forget(e);
    }
    else return set_err(e, MTE_E_ARG, "unknown option " + k);
    return MTE_OK;
}
// Wave plan and routing of the last run: "lds_groups", "hbm_waves", "hbm_docs" (documents taken by
// HBM-resident waves), "continued", "spilled", "slot_bytes", "slots".
int mte_get_info(mte_engine* e, const char* key, int64_t* value) {
    if (!e || !key || !value) return MTE_E_ARG;
    std::string k(key);
    if (k == "lds_groups") *value = e->last_lds_groups;
    else if (k == "hbm_waves") *value = e->last_hbm_waves;
    else if (k == "hbm_docs") *value = e->last_hbm_docs;
    else if (k == "continued") *value = e->last_continued;
    else if (k == "spilled") *value = e->last_spilled;
    else if (k == "slot_bytes") *value = (int64_t)e->P.slot_bytes;
    else if (k == "slots") *value = e->n_slots;
    else if (k == "solo") *value = e->last_solo;
    else if (k == "solo_us") *value = (int64_t)(e->last_solo_ms * 1000.0);  // the solo workgroups' pass (critical path)
    else if (k == "solo_lead_us") *value = (int64_t)(e->last_solo_lead_ms * 1000.0);
    else if (k == "solo_cycles") *value = (int64_t)e->last_solo_cycles;  // longest document's wave: s_memtime
    else if (k == "solo_ref_ticks") *value = (int64_t)e->last_solo_ref;  // ... and s_memrealtime (100 MHz)
    else if (k == "solo_start_delay_ticks") *value = e->last_solo_start_delay;  // vs the bulk kernel's start
    else if (k == "load_alloc_us") *value = (int64_t)(e->last_alloc_ms * 1000.0);
    else if (k == "load_stage_copy_us") *value = (int64_t)(e->stage_copy_ms * 1000.0);
    else if (k == "load_stage_wait_us") *value = (int64_t)(e->stage_wait_ms * 1000.0);
    else if (k == "solo_tail_us") *value = (int64_t)(e->last_solo_tail_ms * 1000.0);
    else if (k == "lean") *value = e->last_lean;
    else if (k == "rows") *value = e->last_rows;  // k_rows waves per CU of the last pass (0: not used)
    else if (k == "rows_mixed") *value = e->last_mixed;  // ... with documents handed over at op 0
    else if (k == "cell_pass_us") *value = (int64_t)(e->last_cell_pass_ms * 1000.0);  // SharedMatrix pass 1
    else if (k == "rows_restart_pushed" || k == "rows_restart_popped" || k == "rows_continued") {
        // k_rows' in-pass restart queue (counters[8] / [9]): documents given back when the row pool
        // was full, and restarts taken by a wave; counters[10]: documents that continued HBM-resident
        // in the pass after outgrowing the row plan (rows_continue, DocRes mode 6)
        uint32_t ctr[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        if (e->d_counters.p) HIP_TRY(e, hipMemcpy(ctr, e->d_counters.p, sizeof ctr, hipMemcpyDeviceToHost));
        *value = k == "rows_restart_pushed" ? ctr[8] : k == "rows_restart_popped" ? ctr[9] : ctr[10];
    }
    else if (k == "emit_us") *value = (int64_t)(e->last_emit_ms * 1000.0);  // emission after the replay pass
    else if (k == "resumed_docs") *value = e->last_resumed_docs;  // option retain: documents continued ...
    else if (k == "resumed_ops") *value = e->last_resumed_ops;    // ... and the op records they skipped
    else if (k == "ck_offered") *value = e->last_ck_offered;      // documents whose log extends the last pass's
    else if (k == "out_text") {  // UTF-16 units Engine::finish gathered (counters[6..7])
        uint32_t ctr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (e->d_counters.p) HIP_TRY(e, hipMemcpy(ctr, e->d_counters.p, sizeof ctr, hipMemcpyDeviceToHost));
        *value = (int64_t)(ctr[6] | ((uint64_t)ctr[7] << 32));
    }
    else return set_err(e, MTE_E_ARG, "unknown info key " + k);
    return MTE_OK;
}
int mte_wave_selftest(mte_engine* e, const uint32_t* in, uint32_t* out, uint32_t n_waves) {
    if (!e) return MTE_E_ARG;
    HIP_TRY(e, hipSetDevice(e->device));
    DevBuf<uint32_t> di, dout;
    HIP_TRY(e, di.alloc((size_t)n_waves * 64));
    HIP_TRY(e, dout.alloc((size_t)n_waves * 64 * 5));
    HIP_TRY(e, hipMemcpy(di.p, in, (size_t)n_waves * 64 * 4, hipMemcpyHostToDevice));
    HIP_TRY(e, launch_wave_selftest(di.p, dout.p, n_waves, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    HIP_TRY(e, hipMemcpy(out, dout.p, (size_t)n_waves * 64 * 5 * 4, hipMemcpyDeviceToHost));
    return MTE_OK;
}
// Replay kernel time of the last mte_replay, measured with HIP events on the engine stream.
double mte_last_kernel_ms(mte_engine* e) { return e ? e->last_kernel_ms : 0; }

// ------------------------------------------------------------------------------------------------
// Builder: ISequencedDocumentMessage JSON -> op records (client.ts:776-836; ops.ts:29-110)
int mte_builder_create(mte_builder** out) {
    if (!out) return MTE_E_ARG;
    *out = new mte_builder();
    return MTE_OK;
}
void mte_builder_destroy(mte_builder* b) { delete b; }
const char* mte_builder_error(const mte_builder* b) { return b ? b->err.c_str() : "null builder"; }

static int num_field(const json::Value& o, const char16_t* k, int32_t* out) {
    const json::Value* v = o.get(k);
    if (!v || v->kind != json::Value::Number) return 0;
    *out = (int32_t)v->num;
    return 1;
}

// Marker.getId (mergeTree.ts:690-695) of a segment's props: the "markerId" value when it is a
// non-empty string (a truthy non-string id is left unmapped: relative positions naming it fail).
static bool marker_id(const json::Value* props, std::u16string* id) {
    const json::Value* v = props && props->kind == json::Value::Object ? props->get(u"markerId") : nullptr;
    if (!v || v->kind != json::Value::String || v->str.empty()) return false;
    *id = v->str;
    return true;
}

// One document under construction: its records, payload and short-id table (observer = 0).
struct DocBuild {
    std::vector<mte_op> ops;
    std::vector<uint16_t> payload;
    std::vector<std::string> names;
    std::unordered_map<std::string, uint32_t> ids;
    bool collab = false;
    bool perm = false;  // a SharedMatrix row / col vector: PermutationSegment specs
    std::string err;
    // marker ids for relative positions (include/mte.h MTE_OP_RELPOS): id -> tag of the marker the
    // reference maps it to; ids tied to two markers, and every id after an annotate that sets a
    // "markerId" property, are ambiguous (blockUpdate re-maps live markers, mergeTree.ts:2748-2768)
    std::unordered_map<std::u16string, uint32_t> mk_tag;
    std::unordered_set<std::u16string> mk_amb;
    bool mk_annot = false;
    uint32_t n_tags = 0;
    // mapIdToSegment (mergeTree.ts:1185-1187) for a marker record: its tag into bits 16..31 of the
    // refType word *w
    void map_marker(const std::u16string& id, uint32_t* w) {
        if (mk_tag.count(id)) mk_amb.insert(id);
        if (n_tags >= 0xFFFFu) {
            mk_amb.insert(id);
            return;
        }
        mk_tag[id] = ++n_tags;
        *w = (*w & 0xFFFFu) | (n_tags << 16);
    }
    // posFromRelativePos's marker lookup (mergeTree.ts:1949-1951) -> tag, offset, before
    uint32_t rel_tag(const json::Value& rp, int32_t* off, bool* before) const {
        *off = 0;
        *before = false;
        if (rp.kind != json::Value::Object) return MTE_REL_UNMAPPED;
        const json::Value* id = rp.get(u"id");
        const json::Value* bf = rp.get(u"before");
        *before = bf && json::truthy(bf);
        num_field(rp, u"offset", off);
        if (!id || id->kind != json::Value::String || id->str.empty() || mk_annot || mk_amb.count(id->str))
            return MTE_REL_UNMAPPED;
        auto it = mk_tag.find(id->str);
        return it == mk_tag.end() ? MTE_REL_UNMAPPED : it->second;
    }
    // Windowed short ids: the engine's client field has MTE_MAX_CLIENTS values, the reference's
    // short-id map grows without bound (client.ts:644-668; a container log gets a new clientId per
    // reconnect). A client's id matters only while one of its ops is above minSeq: nodeLength
    // (mergeTree.ts:1659-1699) compares client ids only for segments whose seq / removedSeq is above
    // the op's refSeq >= minSeq (msn is the least refSeq of the quorum), and SnapshotV1 names clients
    // only above minSeq. So a slot whose client's last op is at or below minSeq is reused; `names`
    // holds each slot's last owner (the name every output above minSeq refers to). Concurrent
    // overlapping removers are all above minSeq while their removal matters. An op whose refSeq is
    // below minSeq after a reuse is reported unsupported (slot 255), as is a client with no free slot.
    // messagesSinceMSNChange (sequence.ts:597-650): op messages above the running minSeq, as
    // JSON.stringify(JSON.parse(message)), with the index of their first op record; the ones left at
    // commit are the legacy summary's catch-up messages
    struct Msg {
        int32_t seq;
        bool rewrite;  // refSeq != seq - 1: the legacy summary rewrites it from its delta ranges
        uint64_t first_op;
        std::string text;
    };
    std::deque<Msg> stash;
    void trim_stash() {
        while (!stash.empty() && stash.front().seq <= cur_min) stash.pop_front();
    }
    std::vector<int32_t> last_use;  // slot -> highest seq its owner used
    int32_t cur_min = 0;            // minSeq as the engine will have it at the next record
    bool loading = false;           // summary records: no reuse before LOAD_END
    bool reused = false;
    explicit DocBuild(const char* observer_name) {
        const std::string observer = observer_name ? observer_name : "";
        names.push_back(observer);
        last_use.push_back(INT32_MAX);  // the observer keeps slot 0
        ids[observer] = 0;
        collab = !observer.empty();
    }
    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    // getOrAddShortClientId (client.ts:644-668), windowed (above); `use` = the seq the id is used at
    int short_id(const std::string& name, uint32_t* out, int32_t use = 0) {
        auto it = ids.find(name);
        if (it != ids.end()) {
            *out = it->second;
            if (use > last_use[*out]) last_use[*out] = use;
            return MTE_OK;
        }
        uint32_t slot = NONE;
        if (names.size() < MTE_MAX_CLIENTS) {
            slot = (uint32_t)names.size();
            names.push_back(name);
            last_use.push_back(use);
        } else if (!loading) {
            for (uint32_t q = 1; q < MTE_MAX_CLIENTS && slot == NONE; q++)
                if (last_use[q] <= cur_min) slot = q;
            if (slot != NONE) {
                ids.erase(names[slot]);
                names[slot] = name;
                last_use[slot] = use;
                reused = true;
            }
        }
        // no slot free: the engine reports the document MTE_DOC_UNSUPPORTED at the first record
        // naming this client (255), the rest of the batch replays normally
        *out = slot == NONE ? 255u : slot;
        if (slot != NONE) ids[name] = slot;
        return MTE_OK;
    }
    void commit(HostBatch& hb) {
        trim_stash();
        for (size_t i = 0; i < stash.size(); i++) {
            const uint64_t end = i + 1 < stash.size() ? stash[i + 1].first_op : ops.size();
            if (stash[i].rewrite)
                for (uint64_t q = stash[i].first_op; q < end && q < ops.size(); q++)
                    if (ops[q].type <= MTE_OP_INSERT_MARKER) ops[q].flags |= MTE_F_CATCHUP;
            hb.msg_first_op.push_back(stash[i].first_op);
            hb.msg_text += stash[i].text;
            hb.msg_text_offsets.push_back(hb.msg_text.size());
        }
        hb.doc_msg_offsets.push_back(hb.msg_first_op.size());
        hb.ops.insert(hb.ops.end(), ops.begin(), ops.end());
        hb.doc_op_offsets.push_back(hb.ops.size());
        hb.payload.insert(hb.payload.end(), payload.begin(), payload.end());
        hb.doc_payload_offsets.push_back(hb.payload.size());
        for (auto& nm : names) {
            hb.client_names += nm;
            hb.client_name_offsets.push_back(hb.client_names.size());
        }
        hb.doc_client_offsets.push_back(hb.doc_client_offsets.back() + (uint32_t)names.size());
    }
};

// A JSON array of ISequencedDocumentMessage -> op records appended to `db`.
static int add_messages(mte_builder* b, const json::Value& doc, DocBuild& db) {
    std::vector<mte_op>& ops = db.ops;
    std::vector<uint16_t>& payload = db.payload;
    const bool collab = db.collab;
    auto fail = [&](int code, const std::string& m) { return db.fail(code, m); };
    if (doc.kind != json::Value::Array) return fail(MTE_E_PARSE, "op log must be a JSON array of messages");
    for (const json::Value& m : doc.items) {
        if (m.kind != json::Value::Object) return fail(MTE_E_PARSE, "message is not an object");
        mte_op base{};
        num_field(m, u"sequenceNumber", &base.seq);
        num_field(m, u"referenceSequenceNumber", &base.ref_seq);
        num_field(m, u"minimumSequenceNumber", &base.msn);
        const json::Value* cid = m.get(u"clientId");
        std::string name = (cid && cid->kind == json::Value::String) ? json::to_utf8(cid->str.data(), cid->str.size()) : "";
        if (!collab) name = "";
        uint32_t sid;
        if (int rc = db.short_id(name, &sid, base.seq)) return rc;
        base.client = (uint8_t)sid;
        const json::Value* type = m.get(u"type");
        const json::Value* contents = m.get(u"contents");
        std::vector<const json::Value*> members;
        bool isOp = type && type->kind == json::Value::String && type->str == u"op" && contents &&
                    contents->kind == json::Value::Object;
        if (isOp) {
            if (collab && sid == 0) return fail(MTE_E_UNSUPPORTED, "observer never submits ops (ack path)");
            if (db.reused && base.ref_seq < db.cur_min) base.client = 255;  // refSeq below minSeq after a reuse
            int32_t t = -1;
            num_field(*contents, u"type", &t);
            if (t == 3) {
                const json::Value* g = contents->get(u"ops");
                if (g && g->kind == json::Value::Array)
                    for (auto& x : g->items) members.push_back(&x);
            } else {
                members.push_back(contents);
            }
        }
        size_t first = ops.size();
        for (const json::Value* c : members) {
            if (c->kind != json::Value::Object) continue;
            if (c->get(u"register")) return fail(MTE_E_UNSUPPORTED, "registers are out of scope");
            mte_op o = base;
            std::u16string mkid;
            bool mapMarker = false;
            int32_t t = -1;
            num_field(*c, u"type", &t);
            num_field(*c, u"pos1", &o.pos1);
            if (t == 0) {
                const json::Value* seg = c->get(u"seg");
                if (!seg) continue;
                const json::Value* props = nullptr;
                if (db.perm) {  // PermutationSegment.fromJSONObject (permutationvector.ts:41-44): [length, start]
                    if (seg->kind != json::Value::Array || seg->items.empty() || seg->items[0].kind != json::Value::Number ||
                        seg->items[0].num < 0 || seg->items[0].num > 0x7FFFFFFF)
                        return fail(MTE_E_UNSUPPORTED, "not a PermutationSegment spec");
                    o.type = MTE_OP_INSERT;
                    o.flags |= MTE_F_PERM;  // handles reset on insert (onDelta, :302-309)
                    o.a = 0;
                    o.b = (uint32_t)seg->items[0].num;
                } else if (seg->kind == json::Value::String) {
                    o.type = MTE_OP_INSERT;
                    o.a = (int32_t)payload.size();
                    o.b = (uint32_t)seg->str.size();
                    payload.insert(payload.end(), seg->str.begin(), seg->str.end());
                } else if (seg->kind == json::Value::Object && seg->get(u"marker")) {
                    o.type = MTE_OP_INSERT_MARKER;
                    const json::Value* mk = seg->get(u"marker");
                    int32_t rt = 0;
                    if (mk->kind == json::Value::Object) num_field(*mk, u"refType", &rt);
                    if (rt < 0 || rt > 0xFFFF) return fail(MTE_E_UNSUPPORTED, "refType beyond 16 bits");
                    o.b = (uint32_t)rt;
                    props = seg->get(u"props");
                    mapMarker = marker_id(props, &mkid);
                } else if (seg->kind == json::Value::Object && seg->get(u"text") &&
                           seg->get(u"text")->kind == json::Value::String) {
                    const json::Value* tx = seg->get(u"text");
                    o.type = MTE_OP_INSERT;
                    o.a = (int32_t)payload.size();
                    o.b = (uint32_t)tx->str.size();
                    payload.insert(payload.end(), tx->str.begin(), tx->str.end());
                    props = seg->get(u"props");
                } else {
                    return fail(MTE_E_UNSUPPORTED, "unknown segment spec");
                }
                if (props && json::truthy(props)) {
                    if (props->kind != json::Value::Object) return fail(MTE_E_UNSUPPORTED, "non-object props");
                    o.props = b->in->propset(*props);
                }
            } else if (t == 1) {
                o.type = MTE_OP_REMOVE;
                num_field(*c, u"pos2", &o.a);
            } else if (t == 2) {
                o.type = MTE_OP_ANNOTATE;
                num_field(*c, u"pos2", &o.a);
                const json::Value* props = c->get(u"props");
                const json::Value* comb = c->get(u"combiningOp");
                if (comb) {
                    const json::Value* nm = comb->kind == json::Value::Object ? comb->get(u"name") : nullptr;
                    if (nm && nm->kind == json::Value::String && nm->str == u"rewrite") o.flags |= MTE_F_REWRITE;
                    else return fail(MTE_E_UNSUPPORTED, "combiningOp other than rewrite is out of scope");
                }
                json::Value empty;
                empty.kind = json::Value::Object;
                o.props = b->in->propset(props && props->kind == json::Value::Object ? *props : empty);
            } else {
                continue;
            }
            // relativePos1 / relativePos2 where pos1 / pos2 is undefined (client.ts:493-510): a RELPOS
            // record before the op (an insert uses only its start)
            const json::Value* rp1 = c->get(u"relativePos1");
            const json::Value* rp2 = c->get(u"relativePos2");
            const bool r1 = rp1 && json::truthy(rp1) && !c->get(u"pos1");
            const bool r2 = t != 0 && rp2 && json::truthy(rp2) && !c->get(u"pos2");
            if (r1 || r2) {
                mte_op r = base;
                r.type = MTE_OP_RELPOS;
                r.flags = 0;
                r.props = 0;
                r.msn = 0;
                bool before = false;
                int32_t off = 0;
                if (r1) {
                    r.pos1 = (int32_t)db.rel_tag(*rp1, &off, &before);
                    r.msn = off;
                    if (before) r.flags |= MTE_F_REL_BEFORE1;
                }
                if (r2) {
                    r.a = (int32_t)db.rel_tag(*rp2, &off, &before);
                    r.props = (uint32_t)off;
                    if (before) r.flags |= MTE_F_REL_BEFORE2;
                }
                ops.push_back(r);
                o.flags |= MTE_F_REL;
            }
            if (mapMarker) db.map_marker(mkid, &o.b);  // after the op's own position (insertSegments)
            if (t == 2) {
                const json::Value* ap = c->get(u"props");
                if (ap && ap->kind == json::Value::Object && ap->get(u"markerId")) db.mk_annot = true;
            }
            ops.push_back(o);
        }
        if (ops.size() == first) {  // no merge-tree op: still a sequenced message
            mte_op o = base;
            o.type = MTE_OP_NOOP;
            ops.push_back(o);
        }
        ops.back().flags |= MTE_F_END_OF_MSG;
        if (collab && base.msn > db.cur_min) db.cur_min = base.msn;  // setMinSeq after the message
        if (collab && type && type->kind == json::Value::String && type->str == u"op") {
            db.stash.push_back(DocBuild::Msg{base.seq, base.ref_seq != base.seq - 1, (uint64_t)first, json::stringify(m)});
            if (db.stash.size() > 64) db.trim_stash();
        }
    }
    return MTE_OK;
}

// documents are added before the first open one (mte_builder_open_doc): a batch lists the committed
// documents, then the open ones
static int builder_closed(mte_builder* b) {
    b->err = "documents cannot be added after an open document (mte_builder_open_doc)";
    return MTE_E_STATE;
}

int mte_builder_add_doc(mte_builder* b, const char* observer_name, const char* text, size_t len) {
    if (!b || !text) return MTE_E_ARG;
    if (!b->open.empty()) return builder_closed(b);
    json::Value doc;
    try {
        doc = json::parse(text, len);
    } catch (std::exception& ex) {
        b->err = ex.what();
        return MTE_E_PARSE;
    }
    DocBuild db(observer_name);
    if (int rc = add_messages(b, doc, db)) {
        b->err = db.err;
        return rc;
    }
    db.commit(b->hb);
    b->paths.emplace_back();
    return MTE_OK;
}

// ------------------------------------------------------------------------------------------------
// Resume from a summary: SnapshotLoader (snapshotLoader.ts:38-216) as LOAD records (include/mte.h).

// A segment spec (sequenceFactory.ts:31-37: string | {text, props} | {marker, props}) -> o.a/o.b/props.
static int load_spec(mte_builder* b, DocBuild& db, const json::Value& seg, mte_op& o, std::u16string* mkid = nullptr,
                     bool* hasId = nullptr) {
    const json::Value* props = nullptr;
    if (db.perm) {  // PermutationSegment.fromJSONObject (permutationvector.ts:41-44): [length, start]
        if (seg.kind != json::Value::Array || seg.items.empty() || seg.items[0].kind != json::Value::Number ||
            seg.items[0].num < 0 || seg.items[0].num > 0x7FFFFFFF)
            return db.fail(MTE_E_UNSUPPORTED, "not a PermutationSegment spec");
        const double st = seg.items.size() > 1 && seg.items[1].kind == json::Value::Number ? seg.items[1].num : -2147483648.0;
        if (st >= 1 && (st > 0x7FFFFFFF || st != (double)(int32_t)st)) return db.fail(MTE_E_UNSUPPORTED, "start handle");
        o.b = (uint32_t)seg.items[0].num;
        o.a = st >= 1 ? (int32_t)st : 0;  // a loaded run keeps its handles (no onDelta reset on load)
        o.flags |= MTE_F_PERM;
        return MTE_OK;
    }
    if (seg.kind == json::Value::String) {
        o.a = (int32_t)db.payload.size();
        o.b = (uint32_t)seg.str.size();
        db.payload.insert(db.payload.end(), seg.str.begin(), seg.str.end());
    } else if (seg.kind == json::Value::Object && seg.get(u"marker")) {
        const json::Value* mk = seg.get(u"marker");
        int32_t rt = 0;
        if (mk->kind == json::Value::Object) num_field(*mk, u"refType", &rt);
        if (rt < 0 || rt > 0xFFFF) return db.fail(MTE_E_UNSUPPORTED, "refType beyond 16 bits");
        o.a = rt;
        o.b = 1;
        o.flags |= MTE_F_LOAD_MARKER;
        props = seg.get(u"props");
        if (mkid && hasId) *hasId = marker_id(props, mkid);
    } else if (seg.kind == json::Value::Object && seg.get(u"text") && seg.get(u"text")->kind == json::Value::String) {
        const json::Value* tx = seg.get(u"text");
        o.a = (int32_t)db.payload.size();
        o.b = (uint32_t)tx->str.size();
        db.payload.insert(db.payload.end(), tx->str.begin(), tx->str.end());
        props = seg.get(u"props");
    } else {
        return db.fail(MTE_E_UNSUPPORTED, "unknown segment spec");
    }
    if (props && json::truthy(props)) {
        if (props->kind != json::Value::Object) return db.fail(MTE_E_UNSUPPORTED, "non-object props");
        o.props = b->in->propset(*props);
    }
    return MTE_OK;
}

static const json::Value* tree_entry(const json::Value& tree, const char16_t* path) {
    const json::Value* es = tree.kind == json::Value::Object ? tree.get(u"entries") : nullptr;
    if (!es || es->kind != json::Value::Array) return nullptr;
    for (const json::Value& e : es->items) {
        const json::Value* p = e.kind == json::Value::Object ? e.get(u"path") : nullptr;
        if (p && p->kind == json::Value::String && p->str == path) return &e;
    }
    return nullptr;
}

static json::Value jstr(const std::u16string& v) {
    json::Value x;
    x.kind = json::Value::String;
    x.str = v;
    return x;
}
static json::Value jnum(double v) {
    json::Value x;
    x.kind = json::Value::Number;
    x.num = v;
    return x;
}
// toLatestVersion for a legacy chunk (snapshotChunks.ts:135-176): segmentTexts -> segments, and for
// the header the metadata it carries or buildHeaderMetadataForLegecyChunk's (a "body" chunk when the
// header holds fewer chars than the document).
static int legacy_to_v1(const std::u16string& path, json::Value& c) {
    json::Value v1;
    v1.kind = json::Value::Object;
    v1.members.emplace_back(u"version", jstr(u"1"));
    for (auto& m : c.members) {
        if (m.first == u"segmentTexts") v1.members.emplace_back(u"segments", m.second);
        else if (m.first == u"headerMetadata") v1.members.emplace_back(u"headerMetadata", m.second);
    }
    if (path == u"header" && !c.get(u"headerMetadata")) {
        json::Value md, ids;
        md.kind = json::Value::Object;
        ids.kind = json::Value::Array;
        auto id = [&](const char16_t* n) {
            json::Value o;
            o.kind = json::Value::Object;
            o.members.emplace_back(u"id", jstr(n));
            ids.items.push_back(o);
        };
        id(u"header");
        const json::Value* cl = c.get(u"chunkLengthChars");
        const json::Value* tl = c.get(u"totalLengthChars");
        if (cl && tl && cl->num < tl->num) id(u"body");
        md.members.emplace_back(u"orderedChunkMetadata", ids);
        if (const json::Value* m = c.get(u"chunkMinSequenceNumber")) md.members.emplace_back(u"minSequenceNumber", *m);
        if (const json::Value* q = c.get(u"chunkSequenceNumber")) md.members.emplace_back(u"sequenceNumber", *q);
        if (tl) md.members.emplace_back(u"totalLength", *tl);
        if (const json::Value* ts = c.get(u"totalSegmentCount")) md.members.emplace_back(u"totalSegmentCount", *ts);
        v1.members.emplace_back(u"headerMetadata", md);
    }
    (void)jnum;
    c = v1;
    return MTE_OK;
}

// Buffer.toString("utf8") of the decoded base64 bytes (fromBase64ToUtf8, common-utils
// base64Encoding.ts): the WHATWG UTF-8 decoder, each maximal invalid subpart becomes U+FFFD.
// Re-encoded as UTF-8 for the JSON parser.
static std::string utf8_replace_invalid(const std::string& in) {
    std::string out;
    out.reserve(in.size());
    auto put = [&](u32 cp) {
        if (cp < 0x80) {
            out.push_back((char)cp);
        } else if (cp < 0x800) {
            out.push_back((char)(0xC0 | (cp >> 6)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        }
    };
    u32 need = 0, seen = 0, cp = 0, lo = 0x80, hi = 0xBF;
    for (size_t i = 0; i < in.size();) {
        const u32 b = (unsigned char)in[i];
        if (need == 0) {
            i++;
            if (b < 0x80) put(b);
            else if (b >= 0xC2 && b <= 0xDF) { need = 1; cp = b & 0x1F; }
            else if (b >= 0xE0 && b <= 0xEF) { if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; need = 2; cp = b & 0xF; }
            else if (b >= 0xF0 && b <= 0xF4) { if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; need = 3; cp = b & 0x7; }
            else put(0xFFFD);
            continue;
        }
        if (b < lo || b > hi) {  // the byte starts over (not consumed)
            need = seen = cp = 0;
            lo = 0x80;
            hi = 0xBF;
            put(0xFFFD);
            continue;
        }
        i++;
        lo = 0x80;
        hi = 0xBF;
        cp = (cp << 6) | (b & 0x3F);
        if (++seen == need) {
            put(cp);
            need = seen = cp = 0;
        }
    }
    if (need) put(0xFFFD);
    return out;
}

// An ITree blob's text (IBlob { contents, encoding: "utf-8" | "base64" }): what storage.read(path) +
// fromBase64ToUtf8 give the loader (snapshotV1.ts:255,267; snapshotLoader.ts:225). Base64 as Node's
// Buffer.from(s, "base64") reads it: standard or url-safe alphabet, whitespace skipped, '=' ends the
// data. Returns 0, or -1 for a missing blob, -2 for an unknown encoding, -3 for a bad character.
static int blob_utf8(const json::Value* v, std::string& out) {
    const json::Value* c = v && v->kind == json::Value::Object ? v->get(u"contents") : nullptr;
    const json::Value* enc = v && v->kind == json::Value::Object ? v->get(u"encoding") : nullptr;
    if (!c || c->kind != json::Value::String) return -1;
    if (!enc || (enc->kind == json::Value::String && enc->str == u"utf-8")) {
        out = json::to_utf8(c->str.data(), c->str.size());
        return 0;
    }
    if (!(enc->kind == json::Value::String && enc->str == u"base64")) return -2;
    out.clear();
    u32 acc = 0, nb = 0;
    for (char16_t ch : c->str) {
        int d;
        if (ch >= u'A' && ch <= u'Z') d = ch - u'A';
        else if (ch >= u'a' && ch <= u'z') d = ch - u'a' + 26;
        else if (ch >= u'0' && ch <= u'9') d = ch - u'0' + 52;
        else if (ch == u'+' || ch == u'-') d = 62;
        else if (ch == u'/' || ch == u'_') d = 63;
        else if (ch == u'=') break;
        else if (ch == u' ' || ch == u'\n' || ch == u'\r' || ch == u'\t') continue;
        else return -3;
        acc = (acc << 6) | (u32)d;
        nb += 6;
        if (nb >= 8) {
            nb -= 8;
            out.push_back((char)((acc >> nb) & 0xff));
        }
    }
    out = utf8_replace_invalid(out);
    return 0;
}
static int blob_text(DocBuild& db, const json::Value* v, std::string& out, const char* missing) {
    switch (blob_utf8(v, out)) {
        case 0: return MTE_OK;
        case -1: return db.fail(MTE_E_PARSE, missing);
        case -2: return db.fail(MTE_E_UNSUPPORTED, "blob encoding other than utf-8 / base64");
        default: return db.fail(MTE_E_PARSE, "bad base64 blob contents");
    }
}

// storage.read(path) + SnapshotV1.processChunk (snapshotV1.ts:249-270)
static int load_chunk(DocBuild& db, const json::Value& tree, const std::u16string& path, json::Value* out) {
    const json::Value* e = tree_entry(tree, path.c_str());
    const json::Value* v = e ? e->get(u"value") : nullptr;
    std::string text;
    if (int rc = blob_text(db, v, text, "summary blob missing")) return rc;
    try {
        *out = json::parse(text.data(), text.size());
    } catch (std::exception& ex) {
        return db.fail(MTE_E_PARSE, ex.what());
    }
    const json::Value* ver = out->kind == json::Value::Object ? out->get(u"version") : nullptr;
    if (!ver && out->kind == json::Value::Object && out->get(u"segmentTexts")) return legacy_to_v1(path, *out);
    if (!ver || ver->kind != json::Value::String || ver->str != u"1")
        return db.fail(MTE_E_UNSUPPORTED, "unsupported snapshot chunk version");
    return MTE_OK;
}

// NonCollabClient (constants.ts) as a short id: the name getLongClientId gives it (client.ts:653-659).
// SnapshotV1 never emits it: universal segments carry no merge info (snapshotV1.ts:219-223).
static const char* const kNonCollabName = "original";

// One summary segment spec -> a LOAD_SEG-shaped record (SnapshotLoader.specToSegment,
// snapshotLoader.ts:79-111): merge info gives client / seq / removedSeq / removedClient; a bare spec,
// or merge info without client and seq, is NonCollab at the universal seq (*batchable: loadBody's
// flushBatch test, :193-195).
struct MarkerId {  // a summary marker's Marker.getId, tagged when the record is emitted
    bool has = false;
    std::u16string id;
};
static int summary_seg(mte_builder* b, DocBuild& db, const json::Value& sp, mte_op& o, bool* info, bool* batchable,
                       MarkerId* mid) {
    const json::Value* js = sp.kind == json::Value::Object ? sp.get(u"json") : nullptr;  // hasMergeInfo
    if (int rc = load_spec(b, db, js ? *js : sp, o, &mid->id, &mid->has)) return rc;
    std::string client = kNonCollabName;
    bool hasClient = false, hasSeq = false;
    if (js) {
        const json::Value* c = sp.get(u"client");
        if (c && c->kind == json::Value::String) {
            client = json::to_utf8(c->str.data(), c->str.size());
            hasClient = true;
        }
        hasSeq = num_field(sp, u"seq", &o.seq) != 0;
    }
    uint32_t cid;
    if (int rc = db.short_id(client, &cid, o.seq)) return rc;
    o.client = (uint8_t)cid;
    if (js && num_field(sp, u"removedSeq", &o.ref_seq)) {
        o.flags |= MTE_F_LOAD_REMOVED;
        const json::Value* rc = sp.get(u"removedClient");
        std::string rn = rc && rc->kind == json::Value::String ? json::to_utf8(rc->str.data(), rc->str.size())
                                                               : kNonCollabName;
        uint32_t rid;
        if (int e = db.short_id(rn, &rid, o.ref_seq)) return e;
        o.pos1 = (int32_t)rid;
    }
    *info = js != nullptr;
    *batchable = !hasClient && (!hasSeq || o.seq == 0);
    return MTE_OK;
}

static int add_summary(mte_builder* b, const json::Value& summary, DocBuild& db) {
    if (!db.collab) return db.fail(MTE_E_ARG, "a summary is loaded by a collaborating client (observer name)");
    db.loading = true;  // no short-id reuse inside the load records
    const json::Value* t = &summary;
    const json::Value* content = tree_entry(summary, u"content");
    if (content && content->get(u"value")) t = content->get(u"value");  // SharedString summary (sequence.ts:413-438)
    json::Value header;
    if (int rc = load_chunk(db, *t, u"header", &header)) return rc;
    const json::Value* md = header.get(u"headerMetadata");
    if (!md || md->kind != json::Value::Object) return db.fail(MTE_E_PARSE, "header metadata not available");
    bool mergeInfo = false;
    const size_t first = db.ops.size();
    const json::Value* hs = header.get(u"segments");
    if (hs && hs->kind == json::Value::Array) {
        for (const json::Value& sp : hs->items) {
            mte_op o{};
            o.type = MTE_OP_LOAD_SEG;
            bool info, batchable;
            MarkerId mid;
            if (int rc = summary_seg(b, db, sp, o, &info, &batchable, &mid)) return rc;
            mergeInfo |= info;
            // reloadFromSegments maps the live markers (blockUpdate -> addNodeReferences, mergeTree.ts:275-284)
            if (mid.has && !(o.flags & MTE_F_LOAD_REMOVED)) {
                uint32_t w = (uint32_t)o.a;
                db.map_marker(mid.id, &w);
                o.a = (int32_t)w;
            }
            db.ops.push_back(o);
        }
    }
    const size_t nHeader = db.ops.size() - first;
    // loadBody (:150-216): nothing when the header holds every segment (:159-161; the shipAsserts on
    // the lengths only log, :152-157, :176-182); otherwise every later chunk's segments in order
    const json::Value* ocm = md->get(u"orderedChunkMetadata");
    int32_t segCount = -1, totalSegs = -2;
    num_field(header, u"segmentCount", &segCount);
    num_field(*md, u"totalSegmentCount", &totalSegs);
    std::vector<mte_op> body;
    std::vector<uint8_t> bodyBatchable;
    std::vector<MarkerId> bodyIds;
    if (segCount != totalSegs && ocm && ocm->kind == json::Value::Array) {
        for (size_t i = 1; i < ocm->items.size(); i++) {
            const json::Value* id = ocm->items[i].kind == json::Value::Object ? ocm->items[i].get(u"id") : nullptr;
            if (!id || id->kind != json::Value::String) return db.fail(MTE_E_PARSE, "chunk id");
            json::Value ch;
            if (int rc = load_chunk(db, *t, id->str, &ch)) return rc;
            const json::Value* cs = ch.get(u"segments");
            if (!cs || cs->kind != json::Value::Array) continue;
            for (const json::Value& sp : cs->items) {
                mte_op o{};
                bool info, batchable;
                MarkerId mid;
                if (int rc = summary_seg(b, db, sp, o, &info, &batchable, &mid)) return rc;
                mergeInfo |= info;
                body.push_back(o);
                bodyBatchable.push_back(batchable ? 1 : 0);
                bodyIds.push_back(std::move(mid));
            }
        }
    }
    // Without merge info every body segment is NonCollab at seq 0 and loadBody is ONE append at the
    // document end: LOAD_SEG records whose tree shape the builder computes below. With merge info,
    // the appends go through the insert walk on the device (LOAD_APPEND after LOAD_END), in the
    // order loadBody issues them.
    // The appended markers are mapped by insertSegments (blockInsert, mergeTree.ts:2199-2205).
    auto tag_body = [&](size_t i, mte_op& o) {
        if (!bodyIds[i].has) return;
        uint32_t w = (uint32_t)o.a;
        db.map_marker(bodyIds[i].id, &w);
        o.a = (int32_t)w;
    };
    if (!mergeInfo) {
        for (size_t i = 0; i < body.size(); i++) {
            mte_op o = body[i];
            if (o.b == 0) continue;  // blockInsert skips empty segments (mergeTree.ts:2196)
            o.type = MTE_OP_LOAD_SEG;
            o.flags |= MTE_F_LOAD_BODY;
            tag_body(i, o);
            db.ops.push_back(o);
        }
    }
    // The loaded tree's shape (child counts per level, document order): reloadFromSegments packs the
    // header 7 to a block, level by level; each body append then lands at the end of the last leaf
    // (insertingWalk at the document end) and a block reaching 8 children splits 4+4 up to the root
    // (mergeTree.ts:2446-2489, 1876-1887). Segment ids and text are not part of the shape.
    std::vector<std::vector<uint32_t>> lv(1);
    for (size_t i = 0; i < nHeader; i += 7) lv[0].push_back((uint32_t)std::min<size_t>(7, nHeader - i));
    if (lv[0].empty()) lv[0].push_back(0);
    while (lv.back().size() > 1) {
        const size_t m = lv.back().size();
        std::vector<uint32_t> up;
        for (size_t i = 0; i < m; i += 7) up.push_back((uint32_t)std::min<size_t>(7, m - i));
        lv.push_back(up);
    }
    for (size_t k = first + nHeader; k < db.ops.size(); k++) {
        size_t l = 0;
        for (lv[0].back()++; l < lv.size() && lv[l].back() == 8; l++) {
            lv[l].back() = 4;
            lv[l].push_back(4);
            if (l + 1 == lv.size()) lv.push_back({2});  // the root split: updateRoot
            else lv[l + 1].back()++;
        }
    }
    // leaf boundaries onto the LOAD_SEG records
    size_t k = first;
    for (size_t leaf = 0; leaf < lv[0].size(); leaf++) {
        if (leaf > 0 && k < db.ops.size()) db.ops[k].flags |= MTE_F_LOAD_LEAF;
        k += lv[0][leaf];
    }
    if (k != db.ops.size()) return db.fail(MTE_E_PARSE, "loaded tree shape does not cover the segments");
    uint32_t nodes = 0;
    for (size_t l = 1; l < lv.size(); l++)
        for (uint32_t c : lv[l]) {
            mte_op o{};
            o.type = MTE_OP_LOAD_NODE;
            o.a = (int32_t)l;
            o.b = c;
            db.ops.push_back(o);
            nodes++;
        }
    mte_op end{};
    end.type = MTE_OP_LOAD_END;
    end.a = (int32_t)nodes;
    num_field(*md, u"sequenceNumber", &end.seq);
    end.msn = end.seq;
    num_field(*md, u"minSequenceNumber", &end.msn);
    db.ops.push_back(end);
    if (mergeInfo && !body.empty()) {
        // loadBody's appends (:184-213): a batchable segment joins `batch`; any other flushes the batch
        // (append at root.cachedLength, NonCollab, seq 0) and is appended alone with its own client and
        // seq. flushBatch never clears `batch` (:196-199): each later flush appends every earlier
        // batched segment object again (MTE_F_APPEND_REPEAT) before the new ones.
        std::vector<size_t> batch;
        std::vector<uint8_t> linked(body.size(), 0);
        auto emit = [&](size_t i, bool firstOfCall, uint32_t client, int32_t seq) {
            if (body[i].b == 0) return;  // blockInsert skips empty segments: no walk, no position
            mte_op o = body[i];
            o.type = MTE_OP_LOAD_APPEND;
            o.client = (uint8_t)client;
            o.seq = seq;
            o.flags = (uint16_t)(o.flags & (MTE_F_LOAD_MARKER | MTE_F_LOAD_REMOVED | MTE_F_PERM));
            if (firstOfCall) o.flags |= MTE_F_APPEND_FIRST;
            if (linked[i]) o.flags |= MTE_F_APPEND_REPEAT;
            else tag_body(i, o);  // a repeat is the same object: mapped already
            linked[i] = 1;
            db.ops.push_back(o);
        };
        uint32_t nc;
        if (int rc = db.short_id(kNonCollabName, &nc)) return rc;
        auto flush = [&]() {
            bool firstOfCall = true;
            for (size_t i : batch) {
                const size_t before = db.ops.size();
                emit(i, firstOfCall, nc, 0);
                firstOfCall &= db.ops.size() == before;
            }
        };
        for (size_t i = 0; i < body.size(); i++) {
            if (bodyBatchable[i]) {
                batch.push_back(i);
            } else {
                flush();
                emit(i, true, body[i].client, body[i].seq);
            }
        }
        flush();
    }
    db.loading = false;
    db.cur_min = std::max(db.cur_min, end.msn);  // startOrUpdateCollaboration(minSeq)
    // loadBodyAndCatchupOps (snapshotLoader.ts:55-77): one blob beyond the chunks holds catch-up
    // messages (legacy summaries), applied after the load like any sequenced message; any other blob
    // count is an error
    const json::Value* es = t->get(u"entries");
    size_t nChunks = ocm && ocm->kind == json::Value::Array ? ocm->items.size() : 1, nBlobs = 0;
    const json::Value* extra = nullptr;
    static const std::vector<json::Value> none;
    for (const json::Value& e : es ? es->items : none) {  // (a reference: `extra` points into it)
        const json::Value* ty = e.get(u"type");
        const json::Value* pth = e.get(u"path");
        if (!ty || ty->kind != json::Value::String || ty->str != u"Blob" || !pth) continue;
        nBlobs++;
        bool isChunk = false;
        for (size_t i = 0; ocm && ocm->kind == json::Value::Array && i < ocm->items.size(); i++) {
            const json::Value* id = ocm->items[i].get(u"id");
            isChunk |= id && id->kind == json::Value::String && id->str == pth->str;
        }
        if (!isChunk) extra = &e;
    }
    if (nBlobs == nChunks + 1 && extra) {
        std::string text;
        if (int rc = blob_text(db, extra->get(u"value"), text, "catch-up ops blob")) return rc;
        json::Value msgs;
        try {
            msgs = json::parse(text.data(), text.size());
        } catch (std::exception& ex) {
            return db.fail(MTE_E_PARSE, ex.what());
        }
        if (int rc = add_messages(b, msgs, db)) return rc;
    } else if (nBlobs != nChunks) {
        return db.fail(MTE_E_PARSE, "Unexpected blobs in snapshot");
    }
    return MTE_OK;
}

int mte_builder_add_doc_from_summary(mte_builder* b, const char* observer_name, const char* summary,
                                     size_t summary_len, const char* ops, size_t ops_len) {
    if (!b || !summary) return MTE_E_ARG;
    if (!b->open.empty()) return builder_closed(b);
    DocBuild db(observer_name);
    json::Value s, log;
    try {
        s = json::parse(summary, summary_len);
        if (ops) log = json::parse(ops, ops_len);
    } catch (std::exception& ex) {
        b->err = ex.what();
        return MTE_E_PARSE;
    }
    int rc = add_summary(b, s, db);
    if (!rc && ops) rc = add_messages(b, log, db);
    if (rc) {
        b->err = db.err;
        return rc;
    }
    db.commit(b->hb);
    b->paths.emplace_back();
    return MTE_OK;
}

// ------------------------------------------------------------------------------------------------
// Container-level op logs (clientReplayTool.ts:113-192, 258-347; fileDeltaStorageService.ts:23-31).

static const char16_t* const kSharedStringType = u"https://graph.microsoft.com/types/mergeTree";  // SharedStringFactory.Type

static std::string u8(const std::u16string& s) { return json::to_utf8(s.data(), s.size()); }

// getDssTreesFromAttach + processAttachMessage: every SharedString tree of an attach snapshot, by
// full path (the attach id, then "/"-joined tree entry paths). Later attaches of a path replace it.
static void attach_trees(const json::Value& attach, const std::string& id, std::deque<json::Value>& store,
                         std::vector<std::pair<std::string, const json::Value*>>& out) {
    const json::Value* snap = attach.get(u"snapshot");
    if (!snap || snap->kind != json::Value::Object) return;
    store.push_back(*snap);
    auto put = [&](const std::string& path, const json::Value* tree) {
        for (auto& o : out)
            if (o.first == path) {
                o.second = tree;
                return;
            }
        out.emplace_back(path, tree);
    };
    const json::Value* ty = attach.get(u"type");
    if (ty && ty->kind == json::Value::String && ty->str == kSharedStringType) put(id, &store.back());
    std::deque<std::pair<std::string, const json::Value*>> q{{id, &store.back()}};
    while (!q.empty()) {
        auto [full, tree] = q.front();
        q.pop_front();
        const json::Value* es = tree->get(u"entries");
        if (!es || es->kind != json::Value::Array) continue;
        for (const json::Value& e : es->items) {
            const json::Value* t = e.get(u"type");
            const json::Value* p = e.get(u"path");
            const json::Value* v = e.get(u"value");
            if (!t || t->kind != json::Value::String || !p || p->kind != json::Value::String || !v) continue;
            if (t->str == u"Tree") {
                q.emplace_back(full + "/" + u8(p->str), v);
            } else if (t->str == u"Blob" && p->str == u".attributes") {
                std::string at_text;
                if (blob_utf8(v, at_text)) continue;
                try {
                    json::Value a = json::parse(at_text.c_str(), at_text.size());
                    const json::Value* at = a.get(u"type");
                    if (at && at->kind == json::Value::String && at->str == kSharedStringType) put(full, tree);
                } catch (std::exception&) {
                }
            }
        }
    }
}

int mte_builder_add_container_log(mte_builder* b, const char* observer_name, const char* text, size_t len,
                                  uint32_t* n_docs) {
    if (!b || !text) return MTE_E_ARG;
    if (!b->open.empty()) return builder_closed(b);
    if (n_docs) *n_docs = 0;
    json::Value log;
    try {
        log = json::parse(text, len);
    } catch (std::exception& ex) {
        b->err = ex.what();
        return MTE_E_PARSE;
    }
    if (log.kind != json::Value::Array) {
        b->err = "container log must be a JSON array of messages";
        return MTE_E_PARSE;
    }
    std::deque<json::Value> store;                                   // attach snapshots / parsed strings
    std::vector<std::pair<std::string, const json::Value*>> trees;   // mergeTreeAttachTrees (insertion order)
    std::unordered_map<std::string, std::vector<json::Value>> msgs;  // merge-tree messages by full path
    // ChunkedOp parts per client (clientReplayTool.ts:118-141: any order, each index once)
    std::unordered_map<std::string, std::pair<std::vector<std::u16string>, std::vector<bool>>> chunks;
    std::vector<uint8_t> have;
    auto parse_str = [&](const std::u16string& s) -> const json::Value* {
        const std::string t = u8(s);
        store.push_back(json::parse(t.data(), t.size()));
        return &store.back();
    };
    try {
        for (const json::Value& m0 : log.items) {
            if (m0.kind != json::Value::Object) continue;
            json::Value m = m0;
            const json::Value* ty = m.get(u"type");
            const json::Value* cid = m.get(u"clientId");
            const std::string client = cid && cid->kind == json::Value::String ? u8(cid->str) : "";
            if (ty && ty->kind == json::Value::String && ty->str == u"chunkedOp") {  // ChunkedOp reassembly
                const json::Value* c = m.get(u"contents");
                const json::Value* ch = c && c->kind == json::Value::String ? parse_str(c->str) : c;
                if (!ch || ch->kind != json::Value::Object) continue;
                int32_t id = 0, total = 0;
                num_field(*ch, u"chunkId", &id);
                num_field(*ch, u"totalChunks", &total);
                const json::Value* part = ch->get(u"contents");
                if (total <= 0 || id < 1 || id > total) throw std::runtime_error("chunk id out of range");
                auto& pending = chunks[client];  // (texts, assigned) by chunk index
                if (pending.first.empty()) {
                    pending.first.assign((size_t)total, std::u16string());
                    pending.second.assign((size_t)total, false);
                }
                if ((size_t)id > pending.first.size()) throw std::runtime_error("chunk id out of range");
                if (pending.second[(size_t)(id - 1)]) throw std::runtime_error("Chunk already assigned");
                pending.second[(size_t)(id - 1)] = true;
                pending.first[(size_t)(id - 1)] = part && part->kind == json::Value::String ? part->str : std::u16string();
                if (id != total) continue;
                std::u16string joined;
                for (size_t q = 0; q < pending.first.size(); q++) {
                    if (!pending.second[q]) throw std::runtime_error("Chunk not assigned");
                    joined += pending.first[q];
                }
                chunks.erase(client);
                // `ch` may point into m's own "contents" member (object-form chunks): copy what is
                // needed from it before m's members are rewritten
                const json::Value* origp = ch->get(u"originalType");
                const bool hasOrig = origp != nullptr;
                const json::Value orig = hasOrig ? *origp : json::Value();
                for (auto& mem : m.members) {
                    if (mem.first == u"contents") {
                        json::Value joinedv;
                        joinedv.kind = json::Value::String;
                        joinedv.str = joined;
                        mem.second = std::move(joinedv);
                    } else if (mem.first == u"type" && hasOrig) {
                        mem.second = orig;
                    }
                }
                ty = m.get(u"type");
            }
            if (!ty || ty->kind != json::Value::String) continue;
            const json::Value* contents = m.get(u"contents");
            if (ty->str == u"attach") {  // ContainerMessageType.Attach
                const json::Value* a = contents && contents->kind == json::Value::String ? parse_str(contents->str) : contents;
                const json::Value* id = a ? a->get(u"id") : nullptr;
                if (a && id && id->kind == json::Value::String) attach_trees(*a, u8(id->str), store, trees);
                continue;
            }
            if (ty->str != u"op" || !contents || contents->kind == json::Value::Null) continue;
            // address envelopes: {address, contents: {address, contents: ...}}
            std::vector<std::string> parts;
            const json::Value* cur = contents;
            do {
                if (cur->kind == json::Value::String) cur = parse_str(cur->str);
                const json::Value* ad = cur->get(u"address");
                parts.push_back(ad && ad->kind == json::Value::String ? u8(ad->str) : "undefined");
                cur = cur->get(u"contents");
                if (!cur) break;
            } while (cur->get(u"contents"));
            if (!cur) continue;
            auto join = [&](const std::string& last) {
                std::string o;
                for (auto& x : parts) o += x + "/";
                return o + last;
            };
            const json::Value* ity = cur->get(u"type");
            if (ity && ity->kind == json::Value::String && ity->str == u"attach") {  // legacy attach envelope
                const json::Value* a = cur->get(u"content");
                const json::Value* id = a ? a->get(u"id") : nullptr;
                if (a && id && id->kind == json::Value::String) attach_trees(*a, join(u8(id->str)), store, trees);
                continue;
            }
            const json::Value* content = cur->get(u"content");
            if (!content || content->kind != json::Value::Object) continue;
            const json::Value* ad = content->get(u"address");
            const std::string path = join(ad && ad->kind == json::Value::String ? u8(ad->str) : "undefined");
            bool known = false;
            for (auto& t : trees) known |= t.first == path;
            const json::Value* op = content->get(u"contents");
            if (!known || !op || op->kind != json::Value::Object || op->get(u"key")) continue;  // interval ops: "key"
            json::Value nm = m;
            for (auto& mem : nm.members)
                if (mem.first == u"contents") mem.second = *op;
            msgs[path].push_back(std::move(nm));
        }
    } catch (std::exception& ex) {
        b->err = ex.what();
        return MTE_E_PARSE;
    }
    uint32_t added = 0;
    // every channel's document is built before any is committed: a failing channel leaves the
    // builder as it was (interned property sets aside, which no document references)
    std::vector<std::unique_ptr<DocBuild>> built;
    for (auto& [path, tree] : trees) {
        built.emplace_back(new DocBuild(observer_name));
        DocBuild& db = *built.back();
        json::Value arr;
        arr.kind = json::Value::Array;
        auto it = msgs.find(path);
        if (it != msgs.end()) arr.items = std::move(it->second);
        int rc = add_summary(b, *tree, db);
        if (!rc) rc = add_messages(b, arr, db);
        if (rc) {
            b->err = path + ": " + db.err;
            return rc;
        }
    }
    for (size_t i = 0; i < built.size(); i++) {
        built[i]->commit(b->hb);
        b->paths.push_back(trees[i].first);
        added++;
    }
    if (n_docs) *n_docs = added;
    return MTE_OK;
}

const char* mte_builder_doc_path(const mte_builder* b, uint32_t doc) {
    return b && doc < b->paths.size() ? b->paths[doc].c_str() : nullptr;
}

// SharedMatrix.processCore (matrix.ts:548-560): rows then cols, each PermutationVector fed the
// messages that target it; a cell op (no target) becomes an MTE_OP_CELL record in both, in message order.
// SharedMatrix.processCore (matrix.ts:548-560) of a message log into the rows / cols documents: the
// messages that target a vector go to it; a cell op (no target) becomes an MTE_OP_CELL record in both,
// in message order.
static int matrix_messages(mte_builder* b, const json::Value& log, DocBuild* dbs[2], uint32_t& cells) {
    auto fail = [&](int code, const std::string& m) {
        b->err = m;
        return code;
    };
    json::Value one;
    one.kind = json::Value::Array;
    one.items.resize(1);
    for (const json::Value& m : log.items) {
        const json::Value* c = m.kind == json::Value::Object ? m.get(u"contents") : nullptr;
        const json::Value* t = c && c->kind == json::Value::Object ? c->get(u"target") : nullptr;
        if (t) {
            const int i = t->kind != json::Value::String ? -1 : t->str == u"rows" ? 0 : t->str == u"cols" ? 1 : -1;
            if (i < 0) continue;
            one.items[0] = m;
            if (int rc = add_messages(b, one, *dbs[i])) return fail(rc, dbs[i]->err);
            continue;
        }
        const json::Value* type = m.kind == json::Value::Object ? m.get(u"type") : nullptr;
        if (!c || c->kind != json::Value::Object || !type || type->kind != json::Value::String || type->str != u"op")
            continue;
        // the remote set (matrix.ts:575-601; an observer never submits, so never the ACK branch)
        int32_t op = -1, rc_[2] = {-1, -1};
        num_field(*c, u"type", &op);
        if (op != 2) return fail(MTE_E_UNSUPPORTED, "SharedMatrix op without target that is not a set");
        const json::Value* rc[2] = {c->get(u"row"), c->get(u"col")};
        for (int i = 0; i < 2; i++) {
            if (!rc[i] || rc[i]->kind != json::Value::Number || rc[i]->num < 0 || rc[i]->num > 0x7FFFFFFF ||
                rc[i]->num != (double)(int32_t)rc[i]->num)
                return fail(MTE_E_UNSUPPORTED, "set row / col must be an integer >= 0");
            rc_[i] = (int32_t)rc[i]->num;
        }
        const json::Value* v = c->get(u"value");
        const uint32_t val = v ? b->in->val(json::stringify(*v)) : 0u;  // undefined -> null in the blob
        const json::Value* cid = m.get(u"clientId");
        const std::string name = (cid && cid->kind == json::Value::String) ? json::to_utf8(cid->str.data(), cid->str.size()) : "";
        for (int i = 0; i < 2; i++) {
            DocBuild& db = *dbs[i];
            mte_op o{};
            num_field(m, u"sequenceNumber", &o.seq);
            num_field(m, u"referenceSequenceNumber", &o.ref_seq);
            num_field(m, u"minimumSequenceNumber", &o.msn);
            uint32_t sid = 0;
            if (db.collab) {  // getOrAddShortClientId (matrix.ts:576, 580)
                if (int e2 = db.short_id(name, &sid, o.seq)) return fail(e2, db.err);
                if (sid == 0) return fail(MTE_E_UNSUPPORTED, "observer never submits ops (ack path)");
                if (db.reused && o.ref_seq < db.cur_min) sid = 255;
            }
            o.client = (uint8_t)sid;
            o.type = MTE_OP_CELL;
            o.flags = i ? MTE_F_CELL_COL : 0;
            o.pos1 = rc_[i];
            o.b = cells;
            o.props = val;
            db.ops.push_back(o);
        }
        cells++;
    }
    return MTE_OK;
}

int mte_builder_add_matrix_log(mte_builder* b, const char* observer_name, const char* text, size_t len) {
    if (!b || !text) return MTE_E_ARG;
    if (!b->open.empty()) return builder_closed(b);
    json::Value log;
    try {
        log = json::parse(text, len);
    } catch (std::exception& ex) {
        b->err = ex.what();
        return MTE_E_PARSE;
    }
    if (log.kind != json::Value::Array) {
        b->err = "matrix log must be a JSON array of messages";
        return MTE_E_PARSE;
    }
    std::vector<std::unique_ptr<DocBuild>> dbs;
    for (int i = 0; i < 2; i++) {
        dbs.emplace_back(new DocBuild(observer_name));
        dbs.back()->perm = true;
    }
    uint32_t cells = b->n_cells;
    DocBuild* two[2] = {dbs[0].get(), dbs[1].get()};
    if (int rc = matrix_messages(b, log, two, cells)) return rc;
    for (int i = 0; i < 2; i++) {
        dbs[i]->commit(b->hb);
        b->paths.emplace_back(i ? "cols" : "rows");
    }
    b->n_cells = cells;
    return MTE_OK;
}

// de-interleave a 32-bit Morton key into its odd (row) and even (col) 16-bit halves
static void unmorton(uint32_t k, uint32_t* r, uint32_t* c) {
    uint32_t rr = 0, cc = 0;
    for (int i = 0; i < 16; i++) {
        cc |= ((k >> (2 * i)) & 1u) << i;
        rr |= ((k >> (2 * i + 1)) & 1u) << i;
    }
    *r = rr;
    *c = cc;
}

// SharedMatrix.loadCore (matrix.ts:528-546) + processCore of the suffix (include/mte.h).
int mte_builder_add_matrix_from_summary(mte_builder* b, const char* observer_name, const char* summary,
                                        size_t summary_len, const char* ops, size_t ops_len) {
    if (!b || !summary) return MTE_E_ARG;
    if (!b->open.empty()) return builder_closed(b);
    json::Value s, log;
    try {
        s = json::parse(summary, summary_len);
        if (ops) log = json::parse(ops, ops_len);
    } catch (std::exception& ex) {
        b->err = ex.what();
        return MTE_E_PARSE;
    }
    if (ops && log.kind != json::Value::Array) {
        b->err = "matrix log must be a JSON array of messages";
        return MTE_E_PARSE;
    }
    auto fail = [&](int code, const std::string& m) {
        b->err = m;
        return code;
    };
    std::vector<std::unique_ptr<DocBuild>> dbs;
    const char16_t* paths[2] = {u"rows", u"cols"};
    for (int i = 0; i < 2; i++) {
        dbs.emplace_back(new DocBuild(observer_name));
        DocBuild& db = *dbs.back();
        db.perm = true;
        // PermutationVector.load (permutationvector.ts:284-294): the handle table, then the segments
        const json::Value* e = tree_entry(s, paths[i]);
        const json::Value* vt = e ? e->get(u"value") : nullptr;
        if (!vt) return fail(MTE_E_PARSE, "matrix summary without its rows / cols tree");
        const json::Value* he = tree_entry(*vt, u"handleTable");
        const json::Value* se = tree_entry(*vt, u"segments");
        std::string ht;
        if (!he || !se || !se->get(u"value")) return fail(MTE_E_PARSE, "vector summary entries");
        if (int rc = blob_text(db, he->get(u"value"), ht, "handleTable blob missing")) return fail(rc, db.err);
        json::Value hv;
        try {
            hv = json::parse(ht.data(), ht.size());
        } catch (std::exception& ex) {
            return fail(MTE_E_PARSE, ex.what());
        }
        if (hv.kind != json::Value::Array || hv.items.empty()) return fail(MTE_E_PARSE, "handleTable is not an array");
        if (int rc = add_summary(b, *se->get(u"value"), db)) return fail(rc, db.err);
        for (size_t h = 0; h < hv.items.size(); h++) {
            const json::Value& x = hv.items[h];
            if (x.kind != json::Value::Number || x.num < 0 || x.num > 0x7FFFFFFF) return fail(MTE_E_UNSUPPORTED, "handle value");
            mte_op o{};
            o.type = MTE_OP_NOOP;
            o.flags = MTE_F_MX_HANDLE;
            o.pos1 = (int32_t)h;
            o.a = (int32_t)x.num;
            db.ops.push_back(o);
        }
    }
    // SparseArray2D.load (sparsearray2d.ts:232-235) of [cells, pending][0]: every tile and cell
    const json::Value* ce = tree_entry(s, u"cells");
    std::string ct;
    if (!ce) return fail(MTE_E_PARSE, "cells blob missing");
    if (int rc = blob_text(*dbs[0], ce->get(u"value"), ct, "cells blob missing")) return fail(rc, dbs[0]->err);
    json::Value cv;
    try {
        cv = json::parse(ct.data(), ct.size());
    } catch (std::exception& ex) {
        return fail(MTE_E_PARSE, ex.what());
    }
    if (cv.kind != json::Value::Array || cv.items.empty() || cv.items[0].kind != json::Value::Array)
        return fail(MTE_E_PARSE, "cells blob is not [cells, pending]");
    DocBuild& rows = *dbs[0];
    std::function<int(const json::Value&, uint32_t, uint32_t, uint32_t)> tile = [&](const json::Value& a, uint32_t hi,
                                                                                  uint32_t depth, uint32_t pre) -> int {
        if (a.kind != json::Value::Array || a.items.size() > 256) return fail(MTE_E_PARSE, "cells tile");
        mte_op t{};
        t.type = MTE_OP_NOOP;
        t.flags = MTE_F_MX_TILE;
        t.pos1 = (int32_t)hi;
        t.a = (int32_t)pre;
        t.b = depth;
        rows.ops.push_back(t);
        for (uint32_t i = 0; i < a.items.size(); i++) {
            const json::Value& x = a.items[i];
            if (x.kind == json::Value::Null) continue;
            if (depth < 3) {
                if (int rc = tile(x, hi, depth + 1, pre | (i << (16 - 8 * depth)))) return rc;
                continue;
            }
            const uint32_t lo = (pre << 8) | i;  // the low key's bytes 0..3
            uint32_t rh, ch, rl, cl;
            unmorton(hi, &rh, &ch);
            unmorton(lo, &rl, &cl);
            mte_op o{};
            o.type = MTE_OP_NOOP;
            o.flags = MTE_F_MX_CELL;
            o.pos1 = (int32_t)((rh << 16) | rl);
            o.a = (int32_t)((ch << 16) | cl);
            o.props = b->in->val(json::stringify(x));
            rows.ops.push_back(o);
        }
        return MTE_OK;
    };
    const json::Value& root = cv.items[0];
    for (uint32_t k = 0; k < root.items.size(); k++)
        if (root.items[k].kind != json::Value::Null)
            if (int rc = tile(root.items[k], k, 0, 0)) return rc;
    if (root.items.size() > 1) {  // the root's length (trailing undefined entries included)
        mte_op t{};
        t.type = MTE_OP_NOOP;
        t.flags = MTE_F_MX_TILE;
        t.pos1 = (int32_t)root.items.size() - 1;
        t.b = 4;  // (no tile: only the root's extent)
        rows.ops.push_back(t);
    }
    uint32_t cells = b->n_cells;
    if (ops) {
        DocBuild* two[2] = {dbs[0].get(), dbs[1].get()};
        if (int rc = matrix_messages(b, log, two, cells)) return rc;
    }
    for (int i = 0; i < 2; i++) {
        dbs[i]->commit(b->hb);
        b->paths.emplace_back(i ? "cols" : "rows");
    }
    b->n_cells = cells;
    return MTE_OK;
}

// An open document (Client.applyMsg one message batch at a time, client.ts:805-836): its log grows
// by mte_builder_append_messages; every mte_builder_batch sees it as it is then (commit of a copy: the
// messages above minSeq at the end of the log so far are its catch-up messages).
int mte_builder_open_doc(mte_builder* b, const char* observer_name, uint32_t* doc) {
    if (!b || !doc) return MTE_E_ARG;
    *doc = b->hb.n_docs() + (uint32_t)b->open.size();
    b->open.emplace_back(new DocBuild(observer_name));
    b->paths.emplace_back();
    return MTE_OK;
}
int mte_builder_append_messages(mte_builder* b, uint32_t doc, const char* text, size_t len) {
    if (!b || !text) return MTE_E_ARG;
    const uint32_t nc = b->hb.n_docs();
    if (doc < nc || doc - nc >= b->open.size()) {
        b->err = "not an open document";
        return MTE_E_ARG;
    }
    json::Value msgs;
    try {
        msgs = json::parse(text, len);
    } catch (std::exception& ex) {
        b->err = ex.what();
        return MTE_E_PARSE;
    }
    DocBuild& db = *b->open[doc - nc];
    // all or nothing: a message the builder refuses leaves the document as it was
    DocBuild keep = db;
    if (int rc = add_messages(b, msgs, db)) {
        b->err = db.err;
        db = std::move(keep);
        return rc;
    }
    return MTE_OK;
}
mte_builder::~mte_builder() = default;

int mte_builder_batch(mte_builder* b, mte_batch* out) {
    if (!b || !out) return MTE_E_ARG;
    if (b->open.empty()) {
        b->hb.view(out);
        return MTE_OK;
    }
    b->view = b->hb;
    for (auto& d : b->open) {
        DocBuild c = *d;
        c.commit(b->view);
    }
    b->view.view(out);
    return MTE_OK;
}

}  // extern "C"
