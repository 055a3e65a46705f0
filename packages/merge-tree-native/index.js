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
    _loadBuilder(b) {
        this._idle();
        addon.load(this._engine, b);
        this._docs = addon.builderDocCount(b);
    }
    /** mte_retain: keep each document's state after a replay, so replaying logs that extend the last
     *  pass's replays only their new ops (Client.applyMsg's incremental cost, client.ts:805-836). */
    retain(on = true) { this._idle(); addon.retain(this._engine, on); }
    /** op records the last replay did not replay again (continued from the pass before) */
    resumedOps() { this._idle(); return addon.getInfo(this._engine, "resumed_ops"); }
    /** mte_get_info: routing and counters of the last pass ("resumed_docs", "rows", "solo", ...) */
    getInfo(key) { this._idle(); return addon.getInfo(this._engine, key); }
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
 * Incremental like Client.applyMsg (client.ts:805-836): applyMsg stages a message; the next read
 * parses the staged messages onto the document's open log (builderAppendMessages) and replays on the
 * GPU only the ops since the previous read, continuing the document's state from that pass (the
 * engine's retain mode, mte_retain). Reads without new messages reuse the last results. A document
 * loaded from a summary, or one the row engines cannot hold (relative positions, 64+ clients, ...),
 * replays from its first op on each read instead: the same results, not incremental.
 */
class MergeTreeClient {
    constructor(observer = "__observer__", options = {}) {
        this.observer = observer;
        this.options = options;
        this.pending = [];
        this.summary = undefined;
        this.messages = [];       // (summary mode only: the suffix replayed with it)
        this._builder = addon.createBuilder();
        this._doc = addon.builderOpenDoc(this._builder, observer);
        this._engine = undefined;
        this._version = 0;        // bumped by every staged change
        this._replayed = -1;      // the version the engine's results belong to
        this._flushing = null;    // pending flush() promise
        this.replays = 0;
    }
    get _dirty() { return this._version !== this._replayed; }
    /** Client.load / SnapshotLoader (client.ts:944-952): resume from a summary ITree before applyMsg. */
    load(summary) { this.summary = summary; this.messages = []; this.pending = []; this._version++; }
    applyMsg(msg) { this.pending.push(msg); this._version++; }
    /** Stage a batch of sequenced messages at once (one replay serves them all). */
    applyMsgs(msgs) { for (const m of msgs) this.pending.push(m); this._version++; }
    _check(version) {
        const [code, seq] = this._engine.docStatus(0);
        if (code === DocStatus.InsertFailed) throw new Error(`MergeTree insert failed at seq ${seq}`);
        if (code !== DocStatus.Ok) throw new Error(`replay failed (status ${code}) at seq ${seq}`);
        this._replayed = version;  // messages staged during an async flush keep the client dirty
        this.replays++;
    }
    _stage() {
        if (!this._engine) {
            this._engine = new BatchedMergeEngine(this.options);
            addon.retain(this._engine._engine, true);
        }
        if (this.summary !== undefined) {  // SnapshotLoader + suffix: a whole replay per read
            for (const m of this.pending) this.messages.push(m);
            this.pending = [];
            this._engine.load([{ observer: this.observer, messages: this.messages.slice(), summary: this.summary }]);
        } else {
            if (this.pending.length) {
                addon.builderAppendMessages(this._builder, this._doc, JSON.stringify(this.pending));
                this.pending = [];
            }
            this._engine._loadBuilder(this._builder);
        }
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
    /** op records the last read continued past instead of replaying again */
    resumedOps() { this._run(); return this._engine.resumedOps(); }
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
    builderOpenDoc: addon.builderOpenDoc, builderAppendMessages: addon.builderAppendMessages,
    builderAddDocFromSummary: addon.builderAddDocFromSummary, builderAddContainerLog: addon.builderAddContainerLog,
    builderAddMatrixLog: addon.builderAddMatrixLog,
    builderAddMatrixFromSummary: addon.builderAddMatrixFromSummary,
    /** rank 0: the RCCL id (Buffer) to send to every rank; rcclCommDestroy(comm) releases a communicator */
    rcclUniqueId: addon.rcclUniqueId, rcclCommDestroy: addon.rcclCommDestroy,
    /** low level: (engine handle, rank, world, comm) -> Buffer of 32-byte records */
    gatherSummariesRaw: addon.gatherSummaries, rcclCommCreateRaw: addon.rcclCommCreate,
};
