// CPU-only checks: the addon loads, binds every entry point, and the host-side builder works.
"use strict";
const assert = require("assert");
const m = require("..");
assert.strictEqual(m.abiVersion(), 2);
assert.ok(/gfx950/.test(m.buildInfo()));
for (const f of ["BatchedMergeEngine", "MergeTreeClient", "createBuilder", "builderAddDoc", "builderDocCount",
    "builderOpenDoc", "builderAppendMessages"]) {
    assert.strictEqual(typeof m[f], "function", f);
}
const b = m.createBuilder();
const msg = (c, s, r, contents) => ({ clientId: c, sequenceNumber: s, referenceSequenceNumber: r,
    minimumSequenceNumber: 0, type: "op", contents });
m.builderAddDoc(b, "__observer__", JSON.stringify([msg("a", 1, 0, { pos1: 0, seg: "hi", type: 0 })]));
m.builderAddDoc(b, "__observer__", JSON.stringify([msg("a", 1, 0, { pos1: 0, pos2: 1, type: 1 })]));
assert.strictEqual(m.builderDocCount(b), 2);
assert.throws(() => m.builderAddDoc(b, "__observer__", "[{]"), /mte_builder_add_doc/);
// resume from a reference SnapshotV1 fixture, then a catch-up suffix
const fs = require("fs");
const summary = fs.readFileSync(__dirname + "/../../../tests/golden/v1/headerOnly.json", "utf8");
m.builderAddDocFromSummary(b, "catchup", summary, JSON.stringify([msg("w", 1, 0, { pos1: 0, seg: "x", type: 0 })]));
m.builderAddDocFromSummary(b, "catchup", summary, null);
assert.strictEqual(m.builderDocCount(b), 4);
assert.throws(() => m.builderAddDocFromSummary(b, "catchup", "{\"entries\":[]}", null), /mte_builder_add_doc_from_summary/);
assert.deepStrictEqual(m.builderAddContainerLog(b, "readonly", "[]"), []);
// a SharedMatrix log: rows and cols vectors (two documents), cell sets as records in both
const splice = (t, p, n) => ({ target: t, pos1: p, seg: [n, -2147483648], type: 0 });
m.builderAddMatrixLog(b, "readonly", JSON.stringify([msg("a", 1, 0, splice("rows", 0, 3)), msg("a", 2, 1, splice("cols", 0, 2)),
    msg("a", 3, 2, { type: 2, row: 0, col: 1, value: 1 })]));
assert.strictEqual(m.builderDocCount(b), 6);
assert.throws(() => m.builderAddMatrixLog(b, "readonly", JSON.stringify([msg("a", 1, 0, { type: 2, row: -1, col: 0, value: 1 })])),
    /mte_builder_add_matrix_log/);
// multi-GPU entry points (the collective itself needs GPUs: parity.gpu.js runs world 1)
for (const f of ["rcclUniqueId", "rcclCommDestroy", "gatherSummariesRaw", "rcclCommCreateRaw"]) {
    assert.strictEqual(typeof m[f], "function", f);
}
assert.strictEqual(typeof m.BatchedMergeEngine.prototype.gatherSummaries, "function");
assert.strictEqual(typeof m.BatchedMergeEngine.prototype.rcclCommCreate, "function");
assert.throws(() => m.gatherSummariesRaw(null, 0, 1, null), /gatherSummaries/);
assert.throws(() => m.rcclCommCreateRaw(null, Buffer.alloc(128), 0, 2), /rcclCommCreate/);
assert.throws(() => m.rcclCommCreateRaw(null, Buffer.alloc(3), 0, 2), /rcclCommCreate/);
// an open document (Client.applyMsg one batch at a time): nothing is added after it
const ob = m.createBuilder();
m.builderAddDoc(ob, "__observer__", "[]");
assert.strictEqual(m.builderOpenDoc(ob, "obs"), 1);
m.builderAppendMessages(ob, 1, JSON.stringify([msg("a", 1, 0, { pos1: 0, seg: "hi", type: 0 })]));
assert.throws(() => m.builderAddDoc(ob, "__observer__", "[]"), /mte_builder_add_doc/);
assert.throws(() => m.builderAppendMessages(ob, 0, "[]"), /mte_builder_append_messages/);
assert.strictEqual(m.builderDocCount(ob), 2);
console.log("exports ok");
