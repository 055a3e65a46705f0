/*
 * mte.h — C ABI of the MI355X batched merge-tree replay engine ("mte").
 *
 * Drop-in boundary for the sequenced-op replay path of @fluidframework/merge-tree 0.31.0
 * (reference: /root/reference/packages/dds/merge-tree/src). The reference boundary is an
 * in-process TypeScript class API; each entry point below names the reference interface it
 * stands in for. The N-API addon (packages/merge-tree-native) and the Python host mirror
 * (fluidframework_amd/) bind exactly these symbols; INTEGRATION.md shows the bindings.
 *
 * Conventions
 *   - Plain C types only: pointers + sizes, no torch / STL types.
 *   - Every call returns int: 0 = ok, <0 = MTE_E_* engine error (message via mte_last_error).
 *     Per-document replay failures never abort a batch: they are recorded as a per-doc status
 *     (mte_doc_status), mirroring the throw points of the reference (e.g. "MergeTree insert
 *     failed", mergeTree.ts:2210-2216).
 *   - One engine per GPU per process; calls on one engine are not re-entrant.
 *   - Strings in op payloads are UTF-16 code units (JavaScript string semantics: lengths and
 *     positions are UTF-16 units, lone surrogates allowed).
 */
#ifndef MTE_H
#define MTE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTE_ABI_VERSION 2  /* 2: mte_batch gained the catch-up message fields, mte_config.snapshot_format */

/* ---- status codes ------------------------------------------------------------------------ */
enum {
    MTE_OK = 0,
    MTE_E_ARG = -1,          /* bad argument */
    MTE_E_NOMEM = -2,        /* host or device allocation failed */
    MTE_E_HIP = -3,          /* HIP runtime error (no device, launch failure, ...) */
    MTE_E_STATE = -4,        /* call out of order (e.g. mte_text before mte_replay) */
    MTE_E_PARSE = -5,        /* malformed op-log JSON */
    MTE_E_UNSUPPORTED = -6,  /* op-log feature outside the engine's scope */
    MTE_E_RANGE = -7,        /* index out of range / buffer too small (required size returned) */
};

/* per-document replay status (mte_doc_status) */
enum {
    MTE_DOC_OK = 0,
    MTE_DOC_INSERT_FAILED = 1,   /* mergeTree.ts:2210-2216 "MergeTree insert failed" */
    MTE_DOC_SEQ_ORDER = 2,       /* client.ts:469-472,832-834 sequencing asserts */
    MTE_DOC_CAPACITY = 3,        /* engine arena exhausted (sizing bug; never silent) */
    MTE_DOC_UNSUPPORTED = 4,     /* > 127 writers in one window, > MTE_MAX_PROPS keys on a segment, ... */
    MTE_DOC_NOT_RUN = 5,
};

#define MTE_MAX_CLIENTS 128      /* short ids 0..127 (observer = 0) in a collaboration window; removedClientOverlap
                                    kept as masks (clients 64..127: a second per-segment word, only in documents
                                    whose window holds more than 64 clients) */
#define MTE_MAX_PROPS 63         /* keys per segment property map on the device; the map records of a
                                    batch are as wide as its widest document needs (its distinct keys) */

/* ---- op records (one per merge-tree delta op; 32 bytes) ---------------------------------- */
/* Types follow ops.ts:29-34 (MergeTreeDeltaType) plus two engine-level kinds. */
enum {
    MTE_OP_INSERT = 0,        /* insert text segment: a = payload offset, b = length */
    MTE_OP_REMOVE = 1,        /* remove [pos1, a) */
    MTE_OP_ANNOTATE = 2,      /* annotate [pos1, a) with prop set `props` */
    MTE_OP_INSERT_MARKER = 3, /* insert Marker: b = refType | tag << 16 (MTE_OP_RELPOS), props = marker props */
    MTE_OP_NOOP = 4,          /* sequenced message with no merge-tree op (only seq/msn advance) */
    /* Resume from a summary (SnapshotLoader, snapshotLoader.ts:98-216); records precede the op log.
     * LOAD_SEG: one segment in document order (specToSegment :79-111): a = payload offset (text) or
     *   refType (marker, MTE_F_LOAD_MARKER), b = length, seq = seg.seq (0 = universal), client =
     *   seg.clientId, props; MTE_F_LOAD_REMOVED: ref_seq = removedSeq, pos1 = removedClient;
     *   MTE_F_LOAD_LEAF: starts a new leaf block; MTE_F_LOAD_BODY: a body-chunk segment (loadBody,
     *   :166-213: insertSegments at the end, refSeq 0, client NonCollab, seq 0).
     * LOAD_NODE: one interior node of the loaded tree: a = level (1 = parent of leaves), b = child
     *   count; in level order, then document order. The shape is that of reloadFromSegments
     *   (mergeTree.ts:1195-1251) over the header followed by the body appends (8 -> 4+4 splits).
     * LOAD_END: a = number of LOAD_NODE records just before it; links the tree, then
     *   startOrUpdateCollaboration(minSeq = msn, currentSeq = seq) (snapshotLoader.ts:126-140). */
    MTE_OP_LOAD_SEG = 5,
    MTE_OP_LOAD_END = 6,
    MTE_OP_LOAD_NODE = 7,
    /* LOAD_APPEND: one segment of loadBody's appends (snapshotLoader.ts:166-213) for a summary with
     *   merge info: insertSegments(pos, [seg], refSeq 0, client, seq) through the ordinary insert walk,
     *   after LOAD_END. Fields as LOAD_SEG (a, b, props, MTE_F_LOAD_MARKER / _REMOVED: ref_seq, pos1),
     *   client/seq = the append's. MTE_F_APPEND_FIRST: first segment of an append call, pos =
     *   root.cachedLength; otherwise pos = the previous record's pos + its length. MTE_F_APPEND_REPEAT:
     *   the segment object was appended before (flushBatch never clears its batch, :196-199): the
     *   reference re-links that object if the walk finds pos -- one object in two places, which the
     *   engine does not model (MTE_DOC_UNSUPPORTED) -- and skips it otherwise. */
    MTE_OP_LOAD_APPEND = 8,
    /* RELPOS: the relativePos1 / relativePos2 of the op record right after it (ops.ts:66-94), which
     *   carries MTE_F_REL; Client.getValidOpRange (client.ts:493-510) takes a position from it only where
     *   pos1 / pos2 is undefined. pos1 / a = the tag of the marker for position 1 / 2 (0 = the op's own
     *   pos1 / pos2; MTE_REL_UNMAPPED = an id the builder cannot tie to one marker), msn / props (as
     *   int32) = offset 1 / 2, MTE_F_REL_BEFORE1 / 2 = relativePos.before; seq, ref_seq, client = the
     *   op's. posFromRelativePos (mergeTree.ts:1943-1966): pos = getPosition(marker) - offset when
     *   before, getPosition(marker) + 1 + offset otherwise.
     *   Marker tags: the builder numbers the markers whose props carry a truthy "markerId"
     *   (Marker.getId, mergeTree.ts:690-695) 1, 2, ... per document in the order the reference maps
     *   them (mapIdToSegment at insert, mergeTree.ts:2074-2078 / 2199-2205; live loaded markers,
     *   addNodeReferences :275-284) and stores the tag in bits 16..31 of the marker's refType field
     *   (INSERT_MARKER b, LOAD_SEG / LOAD_APPEND a); refType itself must fit 16 bits. An id is
     *   MTE_REL_UNMAPPED when it was never mapped, was mapped to two markers (blockUpdate re-maps live
     *   markers, :2748-2768, so the winner depends on block-update order), an annotate before the op
     *   set a "markerId" property, or the marker count passed 65535. A document fails
     *   MTE_DOC_UNSUPPORTED at an op whose marker is unmapped, or whose position comes out below 0.
     *   A marker zamboni dropped is unlinked (scourNode sets its parent undefined, mergeTree.ts:1317),
     *   so getPosition gives 0 for it: position 1 + offset after it, 0 - offset before it. */
    MTE_OP_RELPOS = 9,
    /* CELL: a SharedMatrix cell `set` (matrix.ts:560-601) as one of its two PermutationVectors sees it
     *   (both the rows and the cols document carry one, in message order): pos1 = the op's row (rows
     *   document) or col (cols document, MTE_F_CELL_COL), ref_seq / client = the message's (client: the
     *   vector's short id, getOrAddShortClientId), seq = its sequence number, b = the cell's index among
     *   the batch's cell ops (the same in both records), props = the value id (val_text, canonical
     *   JSON; 0 = null / undefined). The vector applies no merge-tree op for it and its currentSeq /
     *   minSeq do not move (the message is not the vector's). The engine runs adjustPosition
     *   (permutationvector.ts:198-209) in both vectors and, when both are defined, getAllocatedHandle
     *   (:176-196: split at the position, take a handle from the HandleTable free list,
     *   handletable.ts:35-59); zamboni's UNLINK frees a removed run's handles (:357-382). */
    MTE_OP_CELL = 10,
};
#define MTE_REL_UNMAPPED 0xFFFFFFFFu

/* flags */
#define MTE_F_END_OF_MSG 0x1u   /* last op of its ISequencedDocumentMessage: currentSeq=seq, setMinSeq(msn) */
#define MTE_F_REWRITE 0x2u      /* annotate combiningOp {name:"rewrite"} (segmentPropertiesManager.ts:65-78) */
#define MTE_F_LOAD_MARKER 0x4u  /* LOAD_SEG: a Marker (a = refType, length 1) */
#define MTE_F_LOAD_REMOVED 0x8u /* LOAD_SEG: removed (ref_seq = removedSeq, pos1 = removedClient) */
#define MTE_F_LOAD_LEAF 0x10u   /* LOAD_SEG: first segment of a new leaf block */
#define MTE_F_LOAD_BODY 0x20u   /* LOAD_SEG: appended from a body chunk */
#define MTE_F_APPEND_FIRST 0x40u  /* LOAD_APPEND: first segment of an append call (pos = root.cachedLength) */
#define MTE_F_APPEND_REPEAT 0x80u /* LOAD_APPEND: a segment object appended before (see MTE_OP_LOAD_APPEND) */
#define MTE_F_REL 0x100u          /* op: positions from the MTE_OP_RELPOS record just before it */
#define MTE_F_REL_BEFORE1 0x200u  /* RELPOS: relativePos1.before */
#define MTE_F_REL_BEFORE2 0x400u  /* RELPOS: relativePos2.before */
#define MTE_F_PERM 0x1000u        /* INSERT: a PermutationSegment of a SharedMatrix row / col vector
                                     (permutationvector.ts:37-127): b = length, no text, handles unallocated */
#define MTE_F_CELL_COL 0x2000u    /* CELL: the record of the cols vector (else rows) */
/* SharedMatrix summary state (mte_builder_add_matrix_from_summary), NOOP records (no merge-tree op,
 * no seq / msn movement) after a vector's load records, read by the host only:
 *   MX_HANDLE: HandleTable.load (handletable.ts:84-86): handles[pos1] = a (both vectors);
 *   MX_CELL:   SparseArray2D.load (sparsearray2d.ts:232-235): cell (row handle pos1, col handle a) =
 *              value id props (the rows document);
 *   MX_TILE:   a tile the loaded SparseArray2D holds: key hi pos1, depth b (0..3), the first `depth`
 *              bytes of the low key in a (bits 16..23, 8..15, 0..7) (the rows document).
 * A LOAD_SEG / LOAD_APPEND with MTE_F_PERM is a loaded PermutationSegment ([length, start]): b =
 * length, a = its start handle (0 = Handle.unallocated), kept as loaded. */
#define MTE_F_MX_HANDLE 0x4000u
#define MTE_F_MX_CELL 0x8000u
#define MTE_F_MX_TILE 0xC000u
#define MTE_F_MX_MASK 0xC000u
#define MTE_F_CATCHUP 0x800u      /* op of a catch-up message the legacy summary rewrites (refSeq != seq - 1,
                                     sequence.ts:603-625): the engine records its delta ranges */

typedef struct mte_op {
    int32_t seq;        /* sequenceNumber */
    int32_t ref_seq;    /* referenceSequenceNumber */
    int32_t msn;        /* minimumSequenceNumber */
    int32_t pos1;
    int32_t a;          /* REMOVE/ANNOTATE: pos2; INSERT: payload offset (UTF-16 units, doc-relative) */
    uint32_t b;         /* INSERT: payload length; INSERT_MARKER: refType */
    uint32_t props;     /* prop-set id (0 = no props object; see mte_propset) */
    uint8_t type;       /* MTE_OP_* */
    uint8_t client;     /* short client id (first-appearance order, observer = 0; client.ts:644-668) */
    uint16_t flags;     /* MTE_F_* */
} mte_op;

/* An interned property set: the entries of one `props` object in JS Object.keys order.
 * kv[first .. first+count) index mte_batch.prop_keys / prop_vals. value id 0 == JSON null. */
typedef struct mte_propset {
    uint32_t first;
    uint32_t count;
} mte_propset;

/* A batch of documents (host memory, borrowed for the duration of mte_load). */
typedef struct mte_batch {
    uint32_t n_docs;
    const uint64_t* doc_op_offsets;       /* n_docs+1 prefix offsets into ops */
    const mte_op* ops;
    const uint64_t* doc_payload_offsets;  /* n_docs+1 prefix offsets (UTF-16 units) into payload */
    const uint16_t* payload;              /* UTF-16 text arena */
    /* property interning (shared by all docs) */
    uint32_t n_propsets;                  /* propset id 0 is reserved (= no props) */
    const mte_propset* propsets;
    const uint32_t* prop_keys;            /* key id per kv entry */
    const uint32_t* prop_vals;            /* value id per kv entry (0 = null / delete) */
    uint32_t n_keys;                      /* key strings: JSON-escaped, quoted ("\"bold\"") */
    const uint64_t* key_offsets;          /* n_keys+1 byte offsets into key_text */
    const char* key_text;
    uint32_t n_vals;                      /* value texts: canonical JSON.stringify output; id 0 = "null" */
    const uint64_t* val_offsets;          /* n_vals+1 byte offsets into val_text */
    const char* val_text;
    /* client names: per doc, short id order (index 0 = observer) */
    const uint32_t* doc_client_offsets;   /* n_docs+1 prefix offsets into client_name_offsets */
    const uint64_t* client_name_offsets;  /* (total names)+1 byte offsets into client_names */
    const char* client_names;             /* UTF-8 */
    /* SnapshotLegacy catch-up messages (messagesSinceMSNChange, sequence.ts:597-650): per doc the op
     * messages above its log's final MSN, JSON.stringify(JSON.parse(message)) text, and the
     * doc-relative index of each one's first op record. All NULL: none kept. */
    const uint64_t* doc_msg_offsets;      /* n_docs+1 prefix offsets into msg_first_op / msg_text_offsets */
    const uint64_t* msg_first_op;
    const uint64_t* msg_text_offsets;     /* (total msgs)+1 byte offsets into msg_text */
    const char* msg_text;
} mte_batch;

/* ---- engine ------------------------------------------------------------------------------ */
typedef struct mte_engine mte_engine;

typedef struct mte_config {
    int32_t device;             /* HIP device ordinal */
    uint32_t chunk_size;        /* SnapshotV1 chunk size (snapshotV1.ts:40); 0 => 10000 */
    uint32_t snapshot_format;   /* 0: SnapshotV1 (runtime option newMergeTreeSnapshotFormat: true);
                                   1: SnapshotLegacy (the reference's default, client.ts:930-941) */
    uint32_t reserved[5];
} mte_config;

typedef struct mte_stats {
    uint64_t docs;
    uint64_t ops;               /* merge-tree ops applied (all docs) */
    uint64_t messages;          /* sequenced messages applied */
    uint64_t failed_docs;
    double kernel_ms;           /* replay kernel time (HIP events on the engine stream) */
    double h2d_ms;              /* upload time of the last mte_load */
} mte_stats;

typedef struct mte_doc_summary {   /* 32-B record gathered across ranks */
    uint64_t checksum;             /* FNV-1a-64(UTF-8 text ‖ 0 ‖ blob0 ‖ 0 ‖ blob1 ...) */
    uint32_t ops;
    uint32_t length;
    uint32_t segments;
    uint32_t snapshot_bytes;
    int32_t status;
    uint32_t doc_id;
} mte_doc_summary;

typedef struct mte_seg_row {       /* parity dump row (walkAllSegments order, mergeTree.ts:2969) */
    uint32_t kind;                 /* 0 text, 1 marker, 2 permutation run */
    uint32_t len;
    int32_t seq;
    int32_t client;                /* short id (-1 local, -2 non-collab) */
    int32_t removed_seq;           /* INT32_MIN when not removed */
    int32_t removed_client;
    uint64_t overlap_mask;         /* removedClientOverlap as a short-id set (ids 0..63; mte_segments_json lists all) */
    uint32_t text_off;             /* offset into the text returned by mte_segment_text */
    uint32_t ref_type;             /* marker: refType; permutation run: its start handle (0 = unallocated) */
} mte_seg_row;

/* Library identity / capability */
int mte_abi_version(void);
const char* mte_build_info(void);     /* "gfx950 hip <ver>" */

/* new Client(specToSegment, logger, options) + startOrUpdateCollaboration(observer)
 * (client.ts:74-83, 1059-1079) — one engine replays many documents at once. */
int mte_create(const mte_config* cfg, mte_engine** out);
void mte_destroy(mte_engine* e);
const char* mte_last_error(const mte_engine* e);

/* Stage a batch on the device (copies host buffers; returns after the upload). */
int mte_load(mte_engine* e, const mte_batch* batch);

/* Client.applyMsg for every message of every document (client.ts:805-836), on the GPU.
 * Blocking. Per-doc failures are recorded, never thrown. */
int mte_replay(mte_engine* e, mte_stats* out);
/* Incremental replay (Client.applyMsg is incremental, client.ts:805-836): on = 1 keeps each document's
 * replay state after every mte_replay, so the next mte_load of logs that EXTEND the last pass's (the
 * same documents, each log the old one plus new messages; the engine checks the prefix) replays only
 * the new ops of every document the row engines held; any other document replays from op 0. The
 * results are the full replay's either way. on = 0 drops the kept state. Off by default: a replay
 * of the same batch again would otherwise only re-read its results. */
int mte_retain(mte_engine* e, int on);

/* Synthetic workload: generate op logs on the device and leave them loaded, as if
 * by mte_load. kind: 2 = C2 (insert/remove), 3 = C3 (annotate + ties), 5 = C5-style.
 * ops_per_doc may be NULL (uniform n_ops) or per-doc counts. */
int mte_generate(mte_engine* e, uint32_t kind, uint32_t n_docs, uint32_t n_ops,
                 const uint32_t* ops_per_doc, uint32_t n_clients, uint64_t seed_base);

/* As mte_generate, with the GLOBAL id of each document (NULL = 0..n_docs-1): a document's log
 * depends only on (kind, its op count, its global id, n_clients, seed_base), so a multi-GPU run that
 * shards documents by id generates exactly the documents a single GPU would. The ids are also the
 * doc_id of the summary records (mte_summaries). */
int mte_generate_ids(mte_engine* e, uint32_t kind, uint32_t n_docs, uint32_t n_ops, const uint32_t* ops_per_doc,
                     const uint32_t* doc_ids, uint32_t n_clients, uint64_t seed_base);

/* Copy the (generated or loaded) op logs back to the host in mte_batch form. Buffers are owned by
 * the engine and stay valid until the next load/generate/destroy. */
int mte_export_batch(mte_engine* e, mte_batch* out);

/* Results (after mte_replay). */
int mte_doc_status(mte_engine* e, uint32_t doc, int32_t* code, int64_t* failing_seq);
/* MergeTreeTextHelper.getText(currentSeq, observer) (textSegment.ts:154-172), UTF-16. */
int mte_text(mte_engine* e, uint32_t doc, uint16_t* buf, size_t cap, size_t* len);
/* Client.getLength() (client.ts:1057 -> MergeTree.getLength(currentSeq, observer), mergeTree.ts:1577-1584):
 * the observer's visible length in UTF-16 units, a marker counting 1. */
int mte_length(mte_engine* e, uint32_t doc, uint64_t* len);
/* Final segment table (parity dump). rows may be NULL to query *n. */
int mte_segments(mte_engine* e, uint32_t doc, mte_seg_row* rows, size_t cap, size_t* n);
/* SnapshotV1.extractSync + emit (snapshotV1.ts:85-247): the ITree as JSON
 * {"entries":[{"mode":"100644","path":"header","type":"Blob","value":{"contents":...,"encoding":"utf-8"}},...],"id":null}
 * buf may be NULL to query *len. */
int mte_snapshot_v1(mte_engine* e, uint32_t doc, char* buf, size_t cap, size_t* len, uint32_t* n_blobs);
/* SharedSegmentSequence.snapshotCore (sequence.ts:413-438): the SharedString summary tree, "header"
 * (interval collections: "{}") + "content" (the tree of mte_snapshot_v1, or of mte_snapshot_legacy
 * after a replay with snapshot_format 1). buf may be NULL. */
int mte_snapshot_shared_string(mte_engine* e, uint32_t doc, char* buf, size_t cap, size_t* len);
/* SnapshotLegacy.extractSync + emit (snapshotlegacy.ts:103-238) after a replay with snapshot_format 1:
 * the ITree JSON {"entries":[header, body?, <catch_up_name>]} -- the view at minSeq in
 * MergeTreeChunkLegacy chunks (serializeAsMinSupportedVersion, snapshotChunks.ts:75-111) and the
 * catch-up messages above minSeq (sequence.ts:584-634: minimumSequenceNumber set to minSeq; a message
 * whose refSeq is not seq - 1 rewritten to refSeq seq - 1 with contents rebuilt from its delta
 * ranges, createOpsFromDelta sequence.ts:58-100). catch_up_name NULL => "catchupOps". buf may be NULL.
 * MTE_E_UNSUPPORTED when the document has ops above minSeq but no message JSON (generated logs). */
int mte_snapshot_legacy(mte_engine* e, uint32_t doc, const char* catch_up_name, char* buf, size_t cap, size_t* len);
/* SharedMatrix.snapshotCore (matrix.ts:405-430) of a rows / cols document pair from
 * mte_builder_add_matrix_log: each PermutationVector.snapshot (permutationvector.ts:260-273: SnapshotV1
 * under "segments" + the "handleTable" blob: the HandleTable's array, free-list head first,
 * handletable.ts:19-86) and the "cells" blob (JSON.stringify([cells, pending]) of the two SparseArray2D,
 * sparsearray2d.ts:57-235: 4 levels of 256-entry Morton tiles; pending is [null] for an observer).
 * buf may be NULL. */
int mte_snapshot_matrix(mte_engine* e, uint32_t rows_doc, uint32_t cols_doc, char* buf, size_t cap, size_t* len);
/* Per-doc summaries for all docs of the batch (checksum over text + snapshot blobs). */
int mte_summaries(mte_engine* e, mte_doc_summary* out, size_t cap);

/* Multi-GPU: documents are sharded by id across ranks (one process per GPU) and the
 * only collective of the path is this all-gather of the per-document summary records, over RCCL
 * (xGMI inside a node). The communicator is RCCL's own: rank 0 makes an id (mte_rccl_unique_id),
 * the host passes the same MTE_RCCL_ID_BYTES to every rank over its own channel, and each rank calls
 * mte_rccl_comm_create on its engine's device. librccl is opened on first use.
 * mte_gather_summaries: every rank's mte_summaries records, concatenated in rank order (ranks may
 * hold different document counts; each record carries its global doc_id). out may be NULL to query
 * *n; world == 1 needs no communicator. Collective: every rank must call it. */
#define MTE_RCCL_ID_BYTES 128
int mte_rccl_unique_id(uint8_t* id);
int mte_rccl_comm_create(mte_engine* e, const uint8_t* id, int rank, int world, void** comm);
void mte_rccl_comm_destroy(void* comm);
int mte_gather_summaries(mte_engine* e, int rank, int world, void* rccl_comm, mte_doc_summary* out, size_t cap,
                         size_t* n);
/* The same gather as ONE collective call: the records land in a buffer the library allocates
 * (*out, *n records; release it with mte_free). A binding that sizes its own buffer from the result
 * cannot leave the other ranks waiting in a second collective when its allocation fails. */
int mte_gather_summaries_alloc(mte_engine* e, int rank, int world, void* rccl_comm, mte_doc_summary** out,
                               size_t* n);
void mte_free(void* p);

/* Op-log ingestion: build a batch from per-doc JSON arrays of ISequencedDocumentMessage
 * (protocol.ts:126-166). The builder owns the memory. */
typedef struct mte_builder mte_builder;
int mte_builder_create(mte_builder** out);
int mte_builder_add_doc(mte_builder* b, const char* observer_name, const char* json, size_t len);
/* Catch-up from a summary: SharedSegmentSequence.load + SnapshotLoader.initialize
 * (sequence.ts:593-633, snapshotLoader.ts:38-216) then applyMsg for the op-log suffix.
 * summary: the ITree JSON of mte_snapshot_v1 ({"entries":[header, body_0, ...]}) or a SharedString
 * tree holding it under "content", or a SnapshotLegacy tree (chunks converted by toLatestVersion,
 * snapshotChunks.ts:135-176; its catch-up ops blob applied after the load). Blobs are IBlob
 * { contents, encoding }: "utf-8", or "base64" as storage returns them (fromBase64ToUtf8,
 * snapshotV1.ts:267). ops may be NULL (no suffix). MTE_E_UNSUPPORTED for chunk versions other than
 * "1" / legacy and for other blob encodings; MTE_E_PARSE for malformed JSON or base64. */
int mte_builder_add_doc_from_summary(mte_builder* b, const char* observer_name, const char* summary,
                                     size_t summary_len, const char* ops, size_t ops_len);
/* Container-level op log (clientReplayTool.ts:113-192,258-347 over FileDeltaStorageService's
 * messages*.json, fileDeltaStorageService.ts:23-31): a JSON array of container messages is split into
 * one document per attached SharedString channel — ChunkedOp reassembly (containerRuntime.ts:1445-1460),
 * address-envelope unwrapping, the attach snapshot as the summary, the channel's merge-tree ops (not
 * interval-collection "key" ops) as the suffix. *n_docs (may be NULL) = documents added, in attach
 * order; mte_builder_doc_path names each one's channel ("" for documents added otherwise). */
int mte_builder_add_container_log(mte_builder* b, const char* observer_name, const char* json, size_t len,
                                  uint32_t* n_docs);
const char* mte_builder_doc_path(const mte_builder* b, uint32_t doc);
/* SharedMatrix op log (matrix.ts:548-560): a JSON array of its sequenced messages becomes TWO documents,
 * the rows then the cols PermutationVector (permutationvector.ts:129-146; paths "rows", "cols"), each
 * fed the messages whose contents.target names it. Segments are PermutationSegment runs
 * ([length, start] specs). A cell ("set") op becomes an MTE_OP_CELL record in both documents
 * (processCore's remote branch, matrix.ts:575-601); its row / col must be integers >= 0
 * (MTE_E_UNSUPPORTED otherwise). */
int mte_builder_add_matrix_log(mte_builder* b, const char* observer_name, const char* json, size_t len);
/* SharedMatrix.loadCore (matrix.ts:528-546) then processCore of a message suffix: the summary ITree
 * (snapshotCore, matrix.ts:405-433: "rows" / "cols" PermutationVector trees -- SnapshotV1 "segments"
 * and the "handleTable" blob, permutationvector.ts:269-294 -- and the "cells" blob [cells, pending])
 * becomes the rows and the cols document (LOAD records of PermutationSegment runs with their start
 * handles, the HandleTables and the cells as MTE_F_MX_* records), then `ops` (a JSON array of
 * messages, may be NULL) as in mte_builder_add_matrix_log. mte_snapshot_matrix of the pair is the
 * matrix's summary after the suffix. */
int mte_builder_add_matrix_from_summary(mte_builder* b, const char* observer_name, const char* summary,
                                        size_t summary_len, const char* ops, size_t ops_len);
/* An open document: Client.applyMsg fed one message batch at a time (client.ts:805-836). *doc = its
 * index in the batch (after every document added before it; no other document may be added after
 * it). mte_builder_append_messages parses one more JSON array of messages onto its log (all or none
 * of them: a refused message leaves the log as it was); each mte_builder_batch sees the log as it is.
 * With retain on (mte_retain), mte_load + mte_replay of the extended log continue every
 * document whose log extends the last pass's from that pass's state (replaying only the new ops). */
int mte_builder_open_doc(mte_builder* b, const char* observer_name, uint32_t* doc);
int mte_builder_append_messages(mte_builder* b, uint32_t doc, const char* json, size_t len);
int mte_builder_batch(mte_builder* b, mte_batch* out);   /* view valid until destroy */
const char* mte_builder_error(const mte_builder* b);
void mte_builder_destroy(mte_builder* b);

#ifdef __cplusplus
}
#endif
#endif /* MTE_H */
