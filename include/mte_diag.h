/* mte_diag.h — diagnostics and tuning entry points of libmte (not part of the reference boundary:
 * no reference interface corresponds to them; tests, bench.py and tools/ use them to route and
 * measure the replay). Same conventions as mte.h: MTE_OK (0) or a negative MTE_E_* code. */
#ifndef MTE_DIAG_H
#define MTE_DIAG_H
#include "mte.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Raw per-document result record of the last run (engine_types.hpp DocRes, sz bytes). */
int mte_doc_result(mte_engine* e, uint32_t doc, void* out, size_t sz);
/* Last run: documents re-run HBM-resident by the host, pass times, final rows, documents that
 * continued HBM-resident in their wave. */
int mte_run_info(mte_engine* e, uint32_t* spilled, double* lds_ms, double* hbm_ms, uint64_t* out_rows,
                 uint32_t* continued);
/* Wave plan / routing of the last run by key: "lds_groups", "hbm_waves", "hbm_docs", "continued",
 * "spilled", "slot_bytes", "slots", "solo", "lean", "rows" (k_rows waves per CU, 0 = not used),
 * "rows_restart_pushed" / "rows_restart_popped" (k_rows' in-pass restart queue), "rows_continued"
 * (k_rows documents that continued HBM-resident in the pass, DocRes mode 6), pass timings ("solo_us",
 * "emit_us", ...). DocRes::spill_why's low byte says why a k_rows document went to the host's re-run:
 * 1 no free HBM slot, 2 the slot too small for its state, 3 no pool row held, 4 the pool full inside
 * an op, 5 the shared-pool route (no in-pass continuation). "resumed_docs" / "resumed_ops" /
 * "ck_offered": with mte_retain, documents the last pass continued from a checkpoint, the op records
 * they did not replay again, and documents whose log extended the previous pass's. */
int mte_get_info(mte_engine* e, const char* key, int64_t* value);
/* Tuning: "force_hbm", "pool_limit", "hbm_waves_per_cu", "slot_budget_mb"; "retain" = mte_retain. */
int mte_set_option(mte_engine* e, const char* key, int64_t value);
/* Phase cycle counters (profiling build only): PROF_SLOTS u64 per document. */
int mte_profile(mte_engine* e, uint64_t* out, size_t cap);
/* Wave64 primitive self-test: 5 x 64 outputs per wave. */
int mte_wave_selftest(mte_engine* e, const uint32_t* in, uint32_t* out, uint32_t n_waves);
/* Kernel time of the last replay/generate in ms (HIP events). */
double mte_last_kernel_ms(mte_engine* e);

#ifdef __cplusplus
}
#endif
#endif /* MTE_DIAG_H */
