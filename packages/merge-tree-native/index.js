"use strict";
/**
 * @fluidframework/merge-tree-native — batched, GPU-resident replay of merge-tree op logs.
 *
 * Mirrors the slice of @fluidframework/merge-tree's Client API that the replay / summarize path uses
 * (client.ts:805-836 applyMsg, textSegment.ts:154-172 getText, snapshotV1.ts:85-247 SnapshotV1 emit),
 * but for many documents at once: messages are staged per document and replayed on the MI355X in one
 * launch. There is no CPU fallback — without a HIP device createEngine throws.
 */
const path = require("path");
const addon = require(path.join(__dirname, "build", "mte_native.node"));

const DocStatus = Object.freeze({ Ok: 0, InsertFailed: 1, SequenceOrder: 2, Capacity: 3, Unsupported: 4 });

class BatchedMergeEngine {
    constructor(options = {}) {
        this.device = options.device || 0;
        this.chunkSize = options.chunkSize || 10000;  // SnapshotV1.chunkSize (snapshotV1.ts:40)
        // newMergeTreeSnapshotFormat (client.ts:930-941): SnapshotV1 only when it is true, else the
        // reference's default, SnapshotLegacy
        this.legacyFormat = options.newMergeTreeSnapshotFormat !== true;
        this._engine = addon.createEngine(this.device, this.chunkSize, this.legacyFormat ? 1 : 0);
        this._docs = 0;
    }
    /** Stage per-document logs: docs = [{ observer, messages: ISequencedDocumentMessage[], summary? }]
     *  summary (optional): a SnapshotV1 ITree to resume from (SnapshotLoader); messages are the suffix. */
    load(docs) {
        this._idle();
        const b = addon.createBuilder();
        for (const d of docs) {
            const obs = d.observer === undefined ? "__observer__" : d.observer;
            if (d.matrix !== undefined && d.summary !== undefined) {  // SharedMatrix summary + suffix
                const s = typeof d.summary === "string" ? d.summary : JSON.stringify(d.summary);
                addon.builderAddMatrixFromSummary(b, obs, s, JSON.stringify(d.matrix));
            } else if (d.matrix !== undefined) {  // SharedMatrix messages: two documents, rows then cols
                addon.builderAddMatrixLog(b, obs, JSON.stringify(d.matrix));
            } else if (d.summary !== undefined) {
                const s = typeof d.summary === "string" ? d.summary : JSON.stringify(d.summary);
                addon.builderAddDocFromSummary(b, obs, s, d.messages ? JSON.stringify(d.messages) : null);
            } else {
                addon.builderAddDoc(b, obs, JSON.stringify(d.messages));
            }
        }
        addon.load(this._engine, b);
        this._docs = addon.builderDocCount(b);
    }
    generate(kind, nDocs, nOps, nClients = 8, seed = 0) {
        this._idle();
        addon.generate(this._engine, kind, nDocs, nOps, nClients, seed);
        this._docs = nDocs;
    }
    replay() {
        this._idle();
        return addon.replay(this._engine);
    }
    /** mte_replay on a worker thread (N-API async work): the event loop keeps running. While it is
     *  pending, every other call on this engine throws (the engine is not re-entrant). */
    replayAsync() {
        this._idle();
        this._busy = true;
        return addon.replayAsync(this._engine).finally(() => { this._busy = false; });
    }
    _idle() { if (this._busy) throw new Error("BatchedMergeEngine: a replayAsync() is still running"); }
    /** Client.getLength() of a document: the observer's visible length, markers counting 1. */
    getLength(doc) { this._idle(); return addon.getLength(this._engine, doc); }
    docStatus(doc) { this._idle(); return addon.docStatus(this._engine, doc); }
    getText(doc) { this._idle(); return addon.getText(this._engine, doc); }
    /** The ITree SnapshotV1.emit(serializer) returns: { entries: [...], id: null } */
    snapshotV1(doc) { this._idle(); return JSON.parse(addon.snapshotV1(this._engine, doc)); }
    /** SharedMatrix summary of a { matrix } document pair (its rows and cols PermutationVectors) */
    snapshotMatrix(rowsDoc, colsDoc) { this._idle(); return JSON.parse(addon.snapshotMatrix(this._engine, rowsDoc, colsDoc)); }
    /** SnapshotLegacy ITree (snapshotlegacy.ts:103-182): header, body, catch-up messages */
    snapshotLegacy(doc, catchUpBlobName = "catchupOps") {
        this._idle();
        return JSON.parse(addon.snapshotLegacy(this._engine, doc, catchUpBlobName));
    }
    /** 32-byte records {checksum u64, ops, length, segments, snapshotBytes, status, docId} */
    summaries() {
        this._idle();
        return parseSummaries(addon.summaries(this._engine, this._docs));
    }
    /**
     * Multi-GPU (one process per GPU, documents sharded by id): every rank's summaries in rank order,
     * all-gathered over RCCL (mte_gather_summaries). A collective: every rank calls it after its replay.
     * comm: rcclCommCreate(...) of this engine; null when world is 1.
     */
    gatherSummaries(rank, world, comm = null) {
        this._idle();
        return parseSummaries(addon.gatherSummaries(this._engine, rank, world, comm));
    }
    /** This rank's RCCL communicator on the engine's device, from the id rank 0 made (rcclUniqueId()). */
    rcclCommCreate(id, rank, world) { this._idle(); return addon.rcclCommCreate(this._engine, id, rank, world); }
}

function parseSummaries(buf) {
    const out = [];
    for (let o = 0; o + 32 <= buf.length; o += 32) {
        out.push({
            checksum: buf.readBigUInt64LE ? buf.readBigUInt64LE(o) : buf.toString("hex", o, o + 8),
            ops: buf.readUInt32LE(o + 8), length: buf.readUInt32LE(o + 12), segments: buf.readUInt32LE(o + 16),
            snapshotBytes: buf.readUInt32LE(o + 20), status: buf.readInt32LE(o + 24), docId: buf.readUInt32LE(o + 28),
        });
    }
    return out;
}

/**
 * Client-shaped facade for one document (client.ts:42): applyMsg, getText, getLength, snapshot.
 *
 * Batch semantics (documented contract): messages are STAGED by applyMsg/applyMsgs and replayed on
 * the GPU, from the summary (or empty) state, the next time an output is read; reads without new
 * messages reuse that replay. A replay is a kernel launch over the whole log, so read after a batch
 * of messages (a catch-up or summarization step), not after every message: reading after each of n
 * messages replays O(n^2) ops in total. Continuous per-message use belongs to the reference Client.
 */
class MergeTreeClient {
    constructor(observer = "__observer__", options = {}) {
        this.observer = observer;
        this.options = options;
        this.messages = [];
        this.summary = undefined;
        this._engine = undefined;
        this._version = 0;        // bumped by every staged change
        this._replayed = -1;      // the version the engine's results belong to
        this._flushing = null;    // pending flush() promise
    }
    get _dirty() { return this._version !== this._replayed; }
    /** Client.load / SnapshotLoader (client.ts:944-952): resume from a summary ITree before applyMsg. */
    load(summary) { this.summary = summary; this.messages = []; this._version++; }
    applyMsg(msg) { this.messages.push(msg); this._version++; }
    /** Stage a batch of sequenced messages at once (one replay serves them all). */
    applyMsgs(msgs) { for (const m of msgs) this.messages.push(m); this._version++; }
    _check(version) {
        const [code, seq] = this._engine.docStatus(0);
        if (code === DocStatus.InsertFailed) throw new Error(`MergeTree insert failed at seq ${seq}`);
        if (code !== DocStatus.Ok) throw new Error(`replay failed (status ${code}) at seq ${seq}`);
        this._replayed = version;  // messages staged during an async flush keep the client dirty
    }
    _stage() {
        if (!this._engine) this._engine = new BatchedMergeEngine(this.options);
        this._engine.load([{ observer: this.observer, messages: this.messages.slice(), summary: this.summary }]);
        return this._version;
    }
    _run() {
        if (this._flushing) throw new Error("MergeTreeClient: a flush() is still running; await it first");
        if (this._dirty) {
            const v = this._stage();
            this._engine.replay();
            this._check(v);
        }
        return this._engine;
    }
    /** Replay the staged messages off the event loop; resolves when outputs can be read. Reads while
     *  it is pending throw (the engine is not re-entrant); a second flush() waits for the first. */
    async flush() {
        while (this._flushing) await this._flushing.catch(() => {});
        if (!this._dirty) return;
        const v = this._stage();
        this._flushing = this._engine.replayAsync();
        try {
            await this._flushing;
        } finally {
            this._flushing = null;
        }
        this._check(v);
    }
    getText() { return this._run().getText(0); }
    /** Client.getLength (client.ts:1057): markers count 1, unlike getText().length. */
    getLength() { return this._run().getLength(0); }
    /** Client.snapshot (client.ts:907-942): SnapshotV1, or SnapshotLegacy with its catch-up messages
     *  when the options say newMergeTreeSnapshotFormat: false. */
    snapshot() {
        const e = this._run();
        return e.legacyFormat ? e.snapshotLegacy(0, this.options.catchUpBlobName) : e.snapshotV1(0);
    }
}

module.exports = {
    BatchedMergeEngine, MergeTreeClient, DocStatus,
    abiVersion: addon.abiVersion, buildInfo: addon.buildInfo,
    createBuilder: addon.createBuilder, builderAddDoc: addon.builderAddDoc, builderDocCount: addon.builderDocCount,
    builderAddDocFromSummary: addon.builderAddDocFromSummary, builderAddContainerLog: addon.builderAddContainerLog,
    builderAddMatrixLog: addon.builderAddMatrixLog,
    builderAddMatrixFromSummary: addon.builderAddMatrixFromSummary,
    /** rank 0: the RCCL id (Buffer) to send to every rank; rcclCommDestroy(comm) releases a communicator */
    rcclUniqueId: addon.rcclUniqueId, rcclCommDestroy: addon.rcclCommDestroy,
    /** low level: (engine handle, rank, world, comm) -> Buffer of 32-byte records */
    gatherSummariesRaw: addon.gatherSummaries, rcclCommCreateRaw: addon.rcclCommCreate,
};
