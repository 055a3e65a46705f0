/*
 * N-API addon over libmte.so (include/mte.h): the Node/TypeScript host binding of the MI355X
 * merge-tree replay engine. It is the drop-in a SharedSegmentSequence / replay tool binds instead of
 * driving @fluidframework/merge-tree's Client (client.ts:805-836) message by message.
 * Plain C, NAPI_VERSION 8 (Node >= 12.22). Errors are thrown as JS Errors carrying mte_last_error.
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/mte.h"
#include "../../../include/mte_diag.h"

#define CHECK(env, call)                                                       \
    do {                                                                       \
        if ((call) != napi_ok) {                                               \
            napi_throw_error((env), NULL, "N-API call failed: " #call);        \
            return NULL;                                                       \
        }                                                                      \
    } while (0)

static napi_value throw_mte(napi_env env, const char* what, int rc, const char* detail) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s failed (%d)%s%s", what, rc, detail ? ": " : "", detail ? detail : "");
    napi_throw_error(env, NULL, buf);
    return NULL;
}

static void finalize_engine(napi_env env, void* data, void* hint) {
    (void)env;
    (void)hint;
    mte_destroy((mte_engine*)data);
}
static void finalize_builder(napi_env env, void* data, void* hint) {
    (void)env;
    (void)hint;
    mte_builder_destroy((mte_builder*)data);
}

static int get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return 0;
    return argc >= want;
}

static void* get_external(napi_env env, napi_value v) {
    void* p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok) return NULL;
    return p;
}

static char* get_string(napi_env env, napi_value v, size_t* len_out) {
    size_t len = 0;
    if (napi_get_value_string_utf8(env, v, NULL, 0, &len) != napi_ok) return NULL;
    char* s = (char*)malloc(len + 1);
    napi_get_value_string_utf8(env, v, s, len + 1, &len);
    if (len_out) *len_out = len;
    return s;
}

static napi_value make_u32(napi_env env, uint32_t v) {
    napi_value r;
    napi_create_uint32(env, v, &r);
    return r;
}
static napi_value make_f64(napi_env env, double v) {
    napi_value r;
    napi_create_double(env, v, &r);
    return r;
}

/* abiVersion(): number */
static napi_value js_abi_version(napi_env env, napi_callback_info info) {
    (void)info;
    return make_u32(env, (uint32_t)mte_abi_version());
}

/* buildInfo(): string */
static napi_value js_build_info(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value r;
    CHECK(env, napi_create_string_utf8(env, mte_build_info(), NAPI_AUTO_LENGTH, &r));
    return r;
}

/* createEngine(device, chunkSize, snapshotFormat): External — new Client(...) for a whole batch;
 * snapshotFormat 1 = SnapshotLegacy (the reference's default, client.ts:930-941) */
static napi_value js_create_engine(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    mte_config cfg;
    memset(&cfg, 0, sizeof cfg);
    size_t argc = 3;
    napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
    if (argc >= 2) {
        napi_get_value_int32(env, argv[0], &cfg.device);
        napi_get_value_uint32(env, argv[1], &cfg.chunk_size);
    }
    if (argc >= 3) napi_get_value_uint32(env, argv[2], &cfg.snapshot_format);
    mte_engine* e = NULL;
    int rc = mte_create(&cfg, &e);
    if (rc) return throw_mte(env, "mte_create", rc, "no HIP device (MI355X/gfx950 required; no CPU fallback)");
    napi_value ext;
    CHECK(env, napi_create_external(env, e, finalize_engine, NULL, &ext));
    return ext;
}

/* createBuilder(): External */
static napi_value js_create_builder(napi_env env, napi_callback_info info) {
    (void)info;
    mte_builder* b = NULL;
    int rc = mte_builder_create(&b);
    if (rc) return throw_mte(env, "mte_builder_create", rc, NULL);
    napi_value ext;
    CHECK(env, napi_create_external(env, b, finalize_builder, NULL, &ext));
    return ext;
}

/* builderAddDoc(builder, observerName, messagesJson): void */
static napi_value js_builder_add_doc(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) {
        napi_throw_type_error(env, NULL, "builderAddDoc(builder, observer, json)");
        return NULL;
    }
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    size_t len = 0;
    char* obs = get_string(env, argv[1], NULL);
    char* json = get_string(env, argv[2], &len);
    int rc = (b && obs && json) ? mte_builder_add_doc(b, obs, json, len) : MTE_E_ARG;
    free(obs);
    free(json);
    if (rc) return throw_mte(env, "mte_builder_add_doc", rc, b ? mte_builder_error(b) : NULL);
    return NULL;
}

/* builderAddDocFromSummary(builder, observerName, summaryJson, messagesJson | null): void
 * (SnapshotLoader.initialize + applyMsg of the catch-up suffix, snapshotLoader.ts:38-216) */
static napi_value js_builder_add_doc_from_summary(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) {
        napi_throw_type_error(env, NULL, "builderAddDocFromSummary(builder, observer, summary, json|null)");
        return NULL;
    }
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    size_t slen = 0, mlen = 0;
    napi_valuetype t = napi_undefined;
    napi_typeof(env, argv[3], &t);
    char* obs = get_string(env, argv[1], NULL);
    char* summ = get_string(env, argv[2], &slen);
    char* msgs = t == napi_string ? get_string(env, argv[3], &mlen) : NULL;
    int rc = (b && obs && summ) ? mte_builder_add_doc_from_summary(b, obs, summ, slen, msgs, mlen) : MTE_E_ARG;
    free(obs);
    free(summ);
    free(msgs);
    if (rc) return throw_mte(env, "mte_builder_add_doc_from_summary", rc, b ? mte_builder_error(b) : NULL);
    return NULL;
}

/* builderAddContainerLog(builder, observerName, containerMessagesJson): string[] (channel paths)
 * (clientReplayTool.ts:113-192: chunk reassembly, envelope unwrapping, attach snapshots) */
static napi_value js_builder_add_container_log(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) {
        napi_throw_type_error(env, NULL, "builderAddContainerLog(builder, observer, json)");
        return NULL;
    }
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    size_t len = 0;
    uint32_t n = 0;
    char* obs = get_string(env, argv[1], NULL);
    char* json = get_string(env, argv[2], &len);
    int rc = (b && obs && json) ? mte_builder_add_container_log(b, obs, json, len, &n) : MTE_E_ARG;
    free(obs);
    free(json);
    if (rc) return throw_mte(env, "mte_builder_add_container_log", rc, b ? mte_builder_error(b) : NULL);
    mte_batch batch;
    mte_builder_batch(b, &batch);
    napi_value arr;
    CHECK(env, napi_create_array_with_length(env, n, &arr));
    for (uint32_t i = 0; i < n; i++) {
        const char* p = mte_builder_doc_path(b, batch.n_docs - n + i);
        napi_value sv;
        CHECK(env, napi_create_string_utf8(env, p ? p : "", NAPI_AUTO_LENGTH, &sv));
        CHECK(env, napi_set_element(env, arr, i, sv));
    }
    return arr;
}

/* builderAddMatrixLog(builder, observerName, matrixMessagesJson): void — two documents, the rows then
 * the cols PermutationVector of a SharedMatrix (matrix.ts:548-560) */
static napi_value js_builder_add_matrix_log(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) {
        napi_throw_type_error(env, NULL, "builderAddMatrixLog(builder, observer, json)");
        return NULL;
    }
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    size_t len = 0;
    char* obs = get_string(env, argv[1], NULL);
    char* json = get_string(env, argv[2], &len);
    int rc = (b && obs && json) ? mte_builder_add_matrix_log(b, obs, json, len) : MTE_E_ARG;
    free(obs);
    free(json);
    if (rc) return throw_mte(env, "mte_builder_add_matrix_log", rc, b ? mte_builder_error(b) : NULL);
    return NULL;
}

/* builderAddMatrixFromSummary(builder, observerName, summaryJson, messagesJson | null): void — a
 * SharedMatrix loaded from its summary (loadCore, matrix.ts:528-546) then its message suffix: two
 * documents, rows then cols */
static napi_value js_builder_add_matrix_from_summary(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) {
        napi_throw_type_error(env, NULL, "builderAddMatrixFromSummary(builder, observer, summary, messages)");
        return NULL;
    }
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    size_t slen = 0, mlen = 0;
    napi_valuetype t;
    char* obs = get_string(env, argv[1], NULL);
    char* summ = get_string(env, argv[2], &slen);
    char* msgs = NULL;
    if (napi_typeof(env, argv[3], &t) == napi_ok && t == napi_string) msgs = get_string(env, argv[3], &mlen);
    int rc = (b && obs && summ) ? mte_builder_add_matrix_from_summary(b, obs, summ, slen, msgs, mlen) : MTE_E_ARG;
    free(obs);
    free(summ);
    free(msgs);
    if (rc) return throw_mte(env, "mte_builder_add_matrix_from_summary", rc, b ? mte_builder_error(b) : NULL);
    return NULL;
}

/* snapshotMatrix(engine, rowsDoc, colsDoc): string — SharedMatrix.snapshotCore (matrix.ts:405-430) */
static napi_value js_snapshot_matrix(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t r, c;
    napi_get_value_uint32(env, argv[1], &r);
    napi_get_value_uint32(env, argv[2], &c);
    size_t n = 0;
    int rc = mte_snapshot_matrix(e, r, c, NULL, 0, &n);
    if (rc) return throw_mte(env, "mte_snapshot_matrix", rc, mte_last_error(e));
    char* buf = (char*)malloc(n + 1);
    rc = mte_snapshot_matrix(e, r, c, buf, n + 1, &n);
    napi_value sv;
    if (!rc) napi_create_string_utf8(env, buf, n, &sv);
    free(buf);
    if (rc) return throw_mte(env, "mte_snapshot_matrix", rc, mte_last_error(e));
    return sv;
}

/* builderOpenDoc(builder, observerName): number — an open document (its log grows) */
static napi_value js_builder_open_doc(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) {
        napi_throw_type_error(env, NULL, "builderOpenDoc(builder, observer)");
        return NULL;
    }
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    char* obs = get_string(env, argv[1], NULL);
    uint32_t doc = 0;
    int rc = (b && obs) ? mte_builder_open_doc(b, obs, &doc) : MTE_E_ARG;
    free(obs);
    if (rc) return throw_mte(env, "mte_builder_open_doc", rc, b ? mte_builder_error(b) : NULL);
    return make_u32(env, doc);
}

/* builderAppendMessages(builder, doc, messagesJson): void — Client.applyMsg of more messages */
static napi_value js_builder_append_messages(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) {
        napi_throw_type_error(env, NULL, "builderAppendMessages(builder, doc, json)");
        return NULL;
    }
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    uint32_t doc = 0;
    napi_get_value_uint32(env, argv[1], &doc);
    size_t len = 0;
    char* json = get_string(env, argv[2], &len);
    int rc = (b && json) ? mte_builder_append_messages(b, doc, json, len) : MTE_E_ARG;
    free(json);
    if (rc) return throw_mte(env, "mte_builder_append_messages", rc, b ? mte_builder_error(b) : NULL);
    return NULL;
}

/* retain(engine, on): void — mte_retain (incremental replay of extended logs) */
static napi_value js_retain(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    bool on = false;
    napi_get_value_bool(env, argv[1], &on);
    int rc = e ? mte_retain(e, on ? 1 : 0) : MTE_E_ARG;
    if (rc) return throw_mte(env, "mte_retain", rc, e ? mte_last_error(e) : NULL);
    return NULL;
}

/* getInfo(engine, key): number — mte_get_info (routing and counters of the last pass) */
static napi_value js_get_info(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    char* key = get_string(env, argv[1], NULL);
    int64_t v = 0;
    int rc = (e && key) ? mte_get_info(e, key, &v) : MTE_E_ARG;
    free(key);
    if (rc) return throw_mte(env, "mte_get_info", rc, e ? mte_last_error(e) : NULL);
    return make_f64(env, (double)v);
}

/* builderDocCount(builder): number */
static napi_value js_builder_doc_count(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    mte_builder* b = (mte_builder*)get_external(env, argv[0]);
    mte_batch batch;
    if (!b || mte_builder_batch(b, &batch)) return throw_mte(env, "mte_builder_batch", MTE_E_ARG, NULL);
    return make_u32(env, batch.n_docs);
}

/* load(engine, builder): void */
static napi_value js_load(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    mte_builder* b = (mte_builder*)get_external(env, argv[1]);
    mte_batch batch;
    if (!e || !b || mte_builder_batch(b, &batch)) return throw_mte(env, "load", MTE_E_ARG, NULL);
    int rc = mte_load(e, &batch);
    if (rc) return throw_mte(env, "mte_load", rc, mte_last_error(e));
    return NULL;
}

/* generate(engine, kind, nDocs, nOps, nClients, seed): void */
static napi_value js_generate(napi_env env, napi_callback_info info) {
    napi_value argv[6];
    if (!get_args(env, info, 6, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t kind, nd, no, nc;
    int64_t seed;
    napi_get_value_uint32(env, argv[1], &kind);
    napi_get_value_uint32(env, argv[2], &nd);
    napi_get_value_uint32(env, argv[3], &no);
    napi_get_value_uint32(env, argv[4], &nc);
    napi_get_value_int64(env, argv[5], &seed);
    int rc = mte_generate(e, kind, nd, no, NULL, nc, (uint64_t)seed);
    if (rc) return throw_mte(env, "mte_generate", rc, mte_last_error(e));
    return NULL;
}

/* replay(engine): {docs, ops, messages, failedDocs, kernelMs} — Client.applyMsg for every message */
static napi_value js_replay(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    mte_stats st;
    int rc = mte_replay(e, &st);
    if (rc) return throw_mte(env, "mte_replay", rc, mte_last_error(e));
    napi_value o;
    CHECK(env, napi_create_object(env, &o));
    napi_set_named_property(env, o, "docs", make_f64(env, (double)st.docs));
    napi_set_named_property(env, o, "ops", make_f64(env, (double)st.ops));
    napi_set_named_property(env, o, "messages", make_f64(env, (double)st.messages));
    napi_set_named_property(env, o, "failedDocs", make_f64(env, (double)st.failed_docs));
    napi_set_named_property(env, o, "kernelMs", make_f64(env, st.kernel_ms));
    return o;
}

/* replayAsync(engine): Promise<{docs, ops, messages, failedDocs, kernelMs}> — mte_replay on a libuv
 * worker thread (napi_create_async_work), so a long replay does not block the event loop. The engine
 * is referenced until the work completes; the JS facade keeps calls on one engine from overlapping
 * (mte.h: engine calls are not re-entrant). */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref engine_ref;
    mte_engine* e;
    mte_stats st;
    int rc;
    char err[512];
} ReplayJob;

static napi_value stats_object(napi_env env, const mte_stats* st) {
    napi_value o;
    if (napi_create_object(env, &o) != napi_ok) return NULL;
    napi_set_named_property(env, o, "docs", make_f64(env, (double)st->docs));
    napi_set_named_property(env, o, "ops", make_f64(env, (double)st->ops));
    napi_set_named_property(env, o, "messages", make_f64(env, (double)st->messages));
    napi_set_named_property(env, o, "failedDocs", make_f64(env, (double)st->failed_docs));
    napi_set_named_property(env, o, "kernelMs", make_f64(env, st->kernel_ms));
    return o;
}

static void replay_execute(napi_env env, void* data) {
    (void)env;
    ReplayJob* j = (ReplayJob*)data;
    j->rc = mte_replay(j->e, &j->st);
    if (j->rc) snprintf(j->err, sizeof j->err, "mte_replay failed (%d): %s", j->rc, mte_last_error(j->e));
}

static void replay_complete(napi_env env, napi_status status, void* data) {
    ReplayJob* j = (ReplayJob*)data;
    if (status != napi_ok && !j->rc) {
        j->rc = MTE_E_STATE;
        snprintf(j->err, sizeof j->err, "replayAsync: work cancelled");
    }
    if (j->rc) {
        napi_value msg, err;
        napi_create_string_utf8(env, j->err, NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &err);
        napi_reject_deferred(env, j->deferred, err);
    } else {
        napi_resolve_deferred(env, j->deferred, stats_object(env, &j->st));
    }
    napi_delete_reference(env, j->engine_ref);
    napi_delete_async_work(env, j->work);
    free(j);
}

static napi_value js_replay_async(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    if (!e) return throw_mte(env, "replayAsync", MTE_E_ARG, NULL);
    ReplayJob* j = (ReplayJob*)calloc(1, sizeof *j);
    j->e = e;
    napi_value promise, name;
    CHECK(env, napi_create_promise(env, &j->deferred, &promise));
    CHECK(env, napi_create_reference(env, argv[0], 1, &j->engine_ref));
    CHECK(env, napi_create_string_utf8(env, "mte_replay", NAPI_AUTO_LENGTH, &name));
    CHECK(env, napi_create_async_work(env, NULL, name, replay_execute, replay_complete, j, &j->work));
    CHECK(env, napi_queue_async_work(env, j->work));
    return promise;
}

/* getLength(engine, doc): number — Client.getLength (markers count 1, mergeTree.ts:1577-1584) */
static napi_value js_length(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t d;
    napi_get_value_uint32(env, argv[1], &d);
    uint64_t n = 0;
    int rc = mte_length(e, d, &n);
    if (rc) return throw_mte(env, "mte_length", rc, mte_last_error(e));
    return make_f64(env, (double)n);
}

/* docStatus(engine, doc): [code, failingSeq] */
static napi_value js_doc_status(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t d;
    napi_get_value_uint32(env, argv[1], &d);
    int32_t code;
    int64_t seq;
    int rc = mte_doc_status(e, d, &code, &seq);
    if (rc) return throw_mte(env, "mte_doc_status", rc, mte_last_error(e));
    napi_value arr;
    CHECK(env, napi_create_array_with_length(env, 2, &arr));
    napi_set_element(env, arr, 0, make_f64(env, code));
    napi_set_element(env, arr, 1, make_f64(env, (double)seq));
    return arr;
}

/* getText(engine, doc): string (UTF-16, MergeTreeTextHelper.getText) */
static napi_value js_text(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t d;
    napi_get_value_uint32(env, argv[1], &d);
    size_t n = 0;
    int rc = mte_text(e, d, NULL, 0, &n);
    if (rc) return throw_mte(env, "mte_text", rc, mte_last_error(e));
    uint16_t* buf = (uint16_t*)malloc((n + 1) * 2);
    rc = mte_text(e, d, buf, n, &n);
    napi_value s;
    if (!rc) napi_create_string_utf16(env, (const char16_t*)buf, n, &s);
    free(buf);
    if (rc) return throw_mte(env, "mte_text", rc, mte_last_error(e));
    return s;
}

/* snapshotV1(engine, doc): string — the SnapshotV1.emit ITree as JSON */
static napi_value js_snapshot(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t d;
    napi_get_value_uint32(env, argv[1], &d);
    size_t n = 0;
    uint32_t nb = 0;
    int rc = mte_snapshot_v1(e, d, NULL, 0, &n, &nb);
    if (rc) return throw_mte(env, "mte_snapshot_v1", rc, mte_last_error(e));
    char* buf = (char*)malloc(n + 1);
    rc = mte_snapshot_v1(e, d, buf, n + 1, &n, &nb);
    napi_value s;
    if (!rc) napi_create_string_utf8(env, buf, n, &s);
    free(buf);
    if (rc) return throw_mte(env, "mte_snapshot_v1", rc, mte_last_error(e));
    return s;
}

/* snapshotLegacy(engine, doc, catchUpBlobName): string — the SnapshotLegacy.emit ITree as JSON */
static napi_value js_snapshot_legacy(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    size_t argc = 3;
    napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
    if (argc < 2) {
        napi_throw_type_error(env, NULL, "snapshotLegacy(engine, doc, catchUpBlobName?)");
        return NULL;
    }
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t d;
    napi_get_value_uint32(env, argv[1], &d);
    char name[256] = "catchupOps";
    size_t nl = 0;
    if (argc >= 3) napi_get_value_string_utf8(env, argv[2], name, sizeof name, &nl);
    size_t n = 0;
    int rc = mte_snapshot_legacy(e, d, name, NULL, 0, &n);
    if (rc) return throw_mte(env, "mte_snapshot_legacy", rc, mte_last_error(e));
    char* buf = (char*)malloc(n + 1);
    rc = mte_snapshot_legacy(e, d, name, buf, n + 1, &n);
    napi_value s;
    if (!rc) napi_create_string_utf8(env, buf, n, &s);
    free(buf);
    if (rc) return throw_mte(env, "mte_snapshot_legacy", rc, mte_last_error(e));
    return s;
}

/* summaries(engine, nDocs): Buffer of 32-byte mte_doc_summary records */
static napi_value js_summaries(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    uint32_t nd;
    napi_get_value_uint32(env, argv[1], &nd);
    void* data = NULL;
    napi_value buf;
    CHECK(env, napi_create_buffer(env, (size_t)nd * sizeof(mte_doc_summary), &data, &buf));
    int rc = mte_summaries(e, (mte_doc_summary*)data, nd);
    if (rc) return throw_mte(env, "mte_summaries", rc, mte_last_error(e));
    return buf;
}

/* Multi-GPU (mte.h mte_rccl_* / mte_gather_summaries): rank 0 makes the id, the host sends its bytes to
 * every rank (worker_threads message, IPC, ...), each rank creates its communicator on its engine's
 * device and every rank calls gatherSummaries (a collective). */
typedef struct comm_box {  /* the handle's payload: destroyed once, by rcclCommDestroy or the GC */
    void* comm;
} comm_box;
static void finalize_comm(napi_env env, void* data, void* hint) {
    (void)env;
    (void)hint;
    comm_box* c = (comm_box*)data;
    if (c && c->comm) mte_rccl_comm_destroy(c->comm);
    free(c);
}
static void* get_comm(napi_env env, napi_value v) {
    comm_box* c = (comm_box*)get_external(env, v);
    return c ? c->comm : NULL;
}

/* rcclUniqueId(): Buffer of MTE_RCCL_ID_BYTES */
static napi_value js_rccl_unique_id(napi_env env, napi_callback_info info) {
    (void)info;
    void* data = NULL;
    napi_value buf;
    CHECK(env, napi_create_buffer(env, MTE_RCCL_ID_BYTES, &data, &buf));
    int rc = mte_rccl_unique_id((uint8_t*)data);
    if (rc) return throw_mte(env, "mte_rccl_unique_id", rc, NULL);
    return buf;
}

/* rcclCommCreate(engine, idBuffer, rank, world): communicator handle (destroyed by rcclCommDestroy or
 * by the garbage collector) */
static napi_value js_rccl_comm_create(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return throw_mte(env, "rcclCommCreate", -1, "expects (engine, id, rank, world)");
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    void* id = NULL;
    size_t idlen = 0;
    bool isbuf = false;
    napi_is_buffer(env, argv[1], &isbuf);
    if (!e || !isbuf || napi_get_buffer_info(env, argv[1], &id, &idlen) != napi_ok || idlen != MTE_RCCL_ID_BYTES)
        return throw_mte(env, "rcclCommCreate", -1, "expects an engine and a Buffer from rcclUniqueId()");
    int32_t rank = 0, world = 0;
    napi_get_value_int32(env, argv[2], &rank);
    napi_get_value_int32(env, argv[3], &world);
    void* comm = NULL;
    int rc = mte_rccl_comm_create(e, (const uint8_t*)id, rank, world, &comm);
    if (rc) return throw_mte(env, "mte_rccl_comm_create", rc, mte_last_error(e));
    comm_box* box = (comm_box*)malloc(sizeof *box);
    if (!box) {
        mte_rccl_comm_destroy(comm);
        return throw_mte(env, "rcclCommCreate", -1, "out of memory");
    }
    box->comm = comm;
    napi_value out;
    if (napi_create_external(env, box, finalize_comm, NULL, &out) != napi_ok) {
        finalize_comm(env, box, NULL);
        return throw_mte(env, "rcclCommCreate", -1, "napi_create_external");
    }
    return out;
}

/* rcclCommDestroy(comm): releases the communicator now (the handle must not be used again) */
static napi_value js_rccl_comm_destroy(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    comm_box* c = (comm_box*)get_external(env, argv[0]);
    if (c && c->comm) {
        mte_rccl_comm_destroy(c->comm);
        c->comm = NULL;
    }
    return NULL;
}

/* gatherSummaries(engine, rank, world, comm|null): Buffer of every rank's 32-byte records, rank order */
static napi_value js_gather_summaries(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return throw_mte(env, "gatherSummaries", -1, "expects (engine, rank, world, comm)");
    mte_engine* e = (mte_engine*)get_external(env, argv[0]);
    int32_t rank = 0, world = 0;
    napi_get_value_int32(env, argv[1], &rank);
    napi_get_value_int32(env, argv[2], &world);
    napi_valuetype t = napi_undefined;
    napi_typeof(env, argv[3], &t);
    void* comm = t == napi_external ? get_comm(env, argv[3]) : NULL;
    if (!e || world < 1 || rank < 0 || rank >= world || (world > 1 && !comm))
        return throw_mte(env, "gatherSummaries", -1, "expects an engine, 0 <= rank < world and a live communicator when world > 1");
    /* one collective call (the library allocates): a failure below leaves no rank waiting */
    mte_doc_summary* recs = NULL;
    size_t n = 0;
    int rc = mte_gather_summaries_alloc(e, rank, world, comm, &recs, &n);
    if (rc) return throw_mte(env, "mte_gather_summaries_alloc", rc, mte_last_error(e));
    napi_value buf;
    napi_status st = napi_create_buffer_copy(env, n * sizeof(mte_doc_summary), recs, NULL, &buf);
    mte_free(recs);
    if (st != napi_ok) return throw_mte(env, "gatherSummaries", -1, "napi_create_buffer_copy");
    return buf;
}

static napi_value init(napi_env env, napi_value exports) {
    napi_property_descriptor props[] = {
        {"abiVersion", 0, js_abi_version, 0, 0, 0, napi_default, 0},
        {"buildInfo", 0, js_build_info, 0, 0, 0, napi_default, 0},
        {"createEngine", 0, js_create_engine, 0, 0, 0, napi_default, 0},
        {"createBuilder", 0, js_create_builder, 0, 0, 0, napi_default, 0},
        {"builderAddDoc", 0, js_builder_add_doc, 0, 0, 0, napi_default, 0},
        {"builderAddDocFromSummary", 0, js_builder_add_doc_from_summary, 0, 0, 0, napi_default, 0},
        {"builderAddContainerLog", 0, js_builder_add_container_log, 0, 0, 0, napi_default, 0},
        {"builderAddMatrixLog", 0, js_builder_add_matrix_log, 0, 0, 0, napi_default, 0},
        {"builderAddMatrixFromSummary", 0, js_builder_add_matrix_from_summary, 0, 0, 0, napi_default, 0},
        {"snapshotMatrix", 0, js_snapshot_matrix, 0, 0, 0, napi_default, 0},
        {"builderDocCount", 0, js_builder_doc_count, 0, 0, 0, napi_default, 0},
        {"builderOpenDoc", 0, js_builder_open_doc, 0, 0, 0, napi_default, 0},
        {"builderAppendMessages", 0, js_builder_append_messages, 0, 0, 0, napi_default, 0},
        {"retain", 0, js_retain, 0, 0, 0, napi_default, 0},
        {"getInfo", 0, js_get_info, 0, 0, 0, napi_default, 0},
        {"load", 0, js_load, 0, 0, 0, napi_default, 0},
        {"generate", 0, js_generate, 0, 0, 0, napi_default, 0},
        {"replay", 0, js_replay, 0, 0, 0, napi_default, 0},
        {"replayAsync", 0, js_replay_async, 0, 0, 0, napi_default, 0},
        {"getLength", 0, js_length, 0, 0, 0, napi_default, 0},
        {"docStatus", 0, js_doc_status, 0, 0, 0, napi_default, 0},
        {"getText", 0, js_text, 0, 0, 0, napi_default, 0},
        {"snapshotV1", 0, js_snapshot, 0, 0, 0, napi_default, 0},
        {"snapshotLegacy", 0, js_snapshot_legacy, 0, 0, 0, napi_default, 0},
        {"summaries", 0, js_summaries, 0, 0, 0, napi_default, 0},
        {"rcclUniqueId", 0, js_rccl_unique_id, 0, 0, 0, napi_default, 0},
        {"rcclCommCreate", 0, js_rccl_comm_create, 0, 0, 0, napi_default, 0},
        {"rcclCommDestroy", 0, js_rccl_comm_destroy, 0, 0, 0, napi_default, 0},
        {"gatherSummaries", 0, js_gather_summaries, 0, 0, 0, napi_default, 0},
    };
    napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
