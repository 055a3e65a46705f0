// Type declarations for @fluidframework/merge-tree-native (see index.js).
import { ISequencedDocumentMessage, ITree } from "@fluidframework/protocol-definitions";

export declare const DocStatus: { Ok: 0; InsertFailed: 1; SequenceOrder: 2; Capacity: 3; Unsupported: 4 };

export interface ReplayStats { docs: number; ops: number; messages: number; failedDocs: number; kernelMs: number; }
export interface DocSummary {
    checksum: bigint | string; ops: number; length: number; segments: number;
    snapshotBytes: number; status: number; docId: number;
}
/** summary: a SnapshotV1 ITree to resume from (SnapshotLoader); messages then are the catch-up suffix. */
export interface DocLog { observer?: string; messages?: ISequencedDocumentMessage[]; summary?: ITree | string;
    /** SharedMatrix messages: this entry loads as two documents, the rows then the cols vector; with
     *  `summary` (a SharedMatrix summary ITree, SharedMatrix.loadCore) they are the suffix after it */
    matrix?: ISequencedDocumentMessage[]; }

export declare class BatchedMergeEngine {
    constructor(options?: { device?: number; chunkSize?: number; newMergeTreeSnapshotFormat?: boolean });
    load(docs: DocLog[]): void;
    generate(kind: 2 | 3 | 5, nDocs: number, nOps: number, nClients?: number, seed?: number): void;
    replay(): ReplayStats;
    /** mte_replay on a worker thread (N-API async work); other calls on the engine throw meanwhile. */
    replayAsync(): Promise<ReplayStats>;
    docStatus(doc: number): [number, number];
    getText(doc: number): string;
    /** Client.getLength: the observer's visible length, markers counting 1. */
    getLength(doc: number): number;
    snapshotV1(doc: number): ITree;
    /** A { matrix } entry of load() adds two documents: its rows then its cols PermutationVector. */
    snapshotMatrix(rowsDoc: number, colsDoc: number): ITree;
    /** After a replay with newMergeTreeSnapshotFormat: false. */
    snapshotLegacy(doc: number, catchUpBlobName?: string): ITree;
    summaries(): DocSummary[];
    /** Multi-GPU collective: every rank's summaries in rank order, all-gathered over RCCL (mte_gather_summaries).
     *  comm: this engine's communicator (rcclCommCreate), or null when world is 1. */
    gatherSummaries(rank: number, world: number, comm?: RcclComm | null): DocSummary[];
    /** This rank's RCCL communicator on the engine's device, from rank 0's rcclUniqueId(). */
    rcclCommCreate(id: Buffer, rank: number, world: number): RcclComm;
    /** mte_retain: keep each document's state, so a load of logs extending the last pass's replays
     *  only their new ops (Client.applyMsg's incremental cost). */
    retain(on?: boolean): void;
    /** op records the last replay continued past instead of replaying (mte_get_info "resumed_ops") */
    resumedOps(): number;
    /** mte_get_info: routing and counters of the last pass ("resumed_docs", "rows", "solo", ...) */
    getInfo(key: string): number;
}

/** An RCCL communicator handle (released by rcclCommDestroy or when collected). */
export type RcclComm = { readonly __rcclComm: unique symbol };
/** Rank 0 makes the id (MTE_RCCL_ID_BYTES = 128 bytes) and sends it to every rank. */
export declare function rcclUniqueId(): Buffer;
export declare function rcclCommDestroy(comm: RcclComm): void;

/** Client-shaped facade (merge-tree client.ts:42) for one document, incremental like
 *  Client.applyMsg (client.ts:805-836): a read after new messages replays only them on the GPU,
 *  continuing the document's state from the previous read (see index.js). */
export declare class MergeTreeClient {
    constructor(observer?: string, options?: { device?: number; chunkSize?: number });
    load(summary: ITree | string): void;
    applyMsg(msg: ISequencedDocumentMessage): void;
    applyMsgs(msgs: ISequencedDocumentMessage[]): void;
    /** Replay the staged messages off the event loop. */
    flush(): Promise<void>;
    getText(): string;
    getLength(): number;
    snapshot(): ITree;
    /** op records the last read did not replay again */
    resumedOps(): number;
    /** GPU passes run so far (one per read after new messages) */
    readonly replays: number;
}

export declare function abiVersion(): number;
export declare function buildInfo(): string;

/** Low-level builder (the addon's own surface): container logs split per SharedString channel. */
export declare function createBuilder(): unknown;
/** An open document (its log grows by builderAppendMessages); returns its index in the batch. */
export declare function builderOpenDoc(builder: unknown, observer: string): number;
export declare function builderAppendMessages(builder: unknown, doc: number, messagesJson: string): void;
export declare function builderAddContainerLog(builder: unknown, observer: string, containerMessagesJson: string): string[];
