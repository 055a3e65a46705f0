// GPU: the Node path replays the reference's markRangeRemoved / snapshot spec scenarios on the MI355X
// (mergeTree.markRangeRemoved.spec.ts:67-106) and a generated batch, printing checksums for pytest.
"use strict";
const assert = require("assert");
const { BatchedMergeEngine, MergeTreeClient } = require("..");
const msg = (c, s, r, contents, msn = 0) => ({ clientId: c, sequenceNumber: s, referenceSequenceNumber: r,
    minimumSequenceNumber: msn, type: "op", contents });
const hello = [];
for (const [i, ch] of [..."hello world"].entries()) hello.push(msg("local", i + 1, i, { pos1: i, seg: ch, type: 0 }));
const c1 = new MergeTreeClient();
for (const m of hello) c1.applyMsg(m);
c1.applyMsg(msg("remote2", 12, 11, { pos1: 0, pos2: 11, type: 1 }));
c1.applyMsg(msg("remote", 13, 11, { pos1: 0, seg: "text", type: 0 }));
assert.strictEqual(c1.getText(), "text");
const tree = c1.snapshot();
assert.strictEqual(tree.entries[0].path, "header");
// Client.load (SnapshotLoader) from a reference v1 fixture: re-emits the same tree, then catches up
const fixture = JSON.parse(require("fs").readFileSync(__dirname + "/../../../tests/golden/v1/withAnnotations.json", "utf8"));
const c2 = new MergeTreeClient("catchup", { newMergeTreeSnapshotFormat: true });
c2.load(fixture);
assert.deepStrictEqual(c2.snapshot(), fixture.entries[1].value);
const len0 = c2.getLength();
c2.applyMsg(msg("w", 1, 0, { pos1: 3, seg: "XYZ", type: 0 }));
assert.strictEqual(c2.getLength(), len0 + 3);
assert.strictEqual(c2.getText().slice(3, 6), "XYZ");
// Client.getLength counts a marker as 1 (mergeTree.ts:1577-1584): getText().length + markers
const mk = JSON.parse(require("fs").readFileSync(__dirname + "/../../../tests/golden/v1/withMarkers.json", "utf8"));
const c3 = new MergeTreeClient("catchup");
c3.load(mk);
let markers = 0;
for (const ent of mk.entries[1].value.entries) {
    for (const sg of JSON.parse(ent.value.contents).segments) if (sg.marker || (sg.json && sg.json.marker)) markers++;
}
assert.ok(markers > 0);
assert.strictEqual(c3.getLength(), c3.getText().length + markers);
// newMergeTreeSnapshotFormat: false -> SnapshotLegacy (client.ts:930-941): the reference's legacy fixture
const legacyFix = JSON.parse(require("fs").readFileSync(__dirname + "/../../../tests/golden/legacyWithCatchUp/headerOnly.json", "utf8"));
const lc = new MergeTreeClient("", { newMergeTreeSnapshotFormat: false });
for (let i = 0; i < 1250; i++) lc.applyMsg(msg("", i + 1, i, { pos1: 0, seg: `text${i}`, type: 0 }));
const lt = lc.snapshot();
assert.deepStrictEqual(lt.entries.map((x) => [x.path, x.value.contents]),
    legacyFix.entries[1].value.entries.map((x) => [x.path, x.value.contents]));
// the reference's default summary format is SnapshotLegacy (client.ts:930-941)
assert.strictEqual(new MergeTreeClient()._engine, undefined);
assert.strictEqual(c1._engine.legacyFormat, true);
// SharedMatrix with cell sets (matrix.ts:575-601): rows [3], cols [2], set (0,0)=5 and (2,1)="x" --
// rows 0 and 2 take handles 1 and 2 (split out of the unallocated run), cols 0 and 1 settle into one
// run [2, 1]; the cells sit at Morton keys 3 and 12 of the first tile
const UN = -2147483648;
const mx = new BatchedMergeEngine({ newMergeTreeSnapshotFormat: true });
mx.load([{ observer: "obs", matrix: [
    msg("w", 1, 0, { target: "rows", pos1: 0, seg: [3, UN], type: 0 }, 1),
    msg("w", 2, 1, { target: "cols", pos1: 0, seg: [2, UN], type: 0 }, 2),
    msg("w", 3, 2, { type: 2, row: 0, col: 0, value: 5 }, 3),
    msg("w", 4, 3, { type: 2, row: 2, col: 1, value: "x" }, 4)] }]);
assert.strictEqual(mx.replay().failedDocs, 0);
const mt = mx.snapshotMatrix(0, 1);
const vec = (i) => JSON.parse(mt.entries[i].value.entries[0].value.entries[0].value.contents).segments;
assert.deepStrictEqual(vec(0), [[1, 1], [1, UN], [1, 2]]);
assert.deepStrictEqual(vec(1), [[2, 1]]);
assert.deepStrictEqual(mt.entries.slice(0, 2).map((x) => x.value.entries[1].value.contents), ["[3,0,0]", "[3,0,0]"]);
const [cells, pending] = JSON.parse(mt.entries[2].value.contents);
assert.deepStrictEqual(pending, [null]);
assert.deepStrictEqual(cells[0][0][0][0].flatMap((v, i) => (v === null ? [] : [[i, v]])), [[3, 5], [12, "x"]]);
const e = new BatchedMergeEngine({ newMergeTreeSnapshotFormat: true });
e.generate(2, 8, 500, 8, 3);
const st = e.replay();
assert.strictEqual(st.failedDocs, 0);
const sums = e.summaries();
// the multi-GPU gather at world 1 (no communicator) is this engine's own records, rank order
assert.deepStrictEqual(e.gatherSummaries(0, 1, null).map((x) => [x.checksum.toString(), x.docId]),
    sums.map((x) => [x.checksum.toString(), x.docId]));
assert.throws(() => e.gatherSummaries(0, 2, null), /communicator/);
(async () => {
    // replayAsync: the same replay on a worker thread while the event loop keeps turning
    const big = new BatchedMergeEngine();
    big.generate(2, 2048, 10000, 8, 9);
    const syncSums = (big.replay(), big.summaries().map((s) => s.checksum.toString()));
    let ticks = 0;
    const timer = setInterval(() => { ticks++; }, 0);
    const pending = big.replayAsync();
    assert.throws(() => big.getText(0), /still running/);
    assert.throws(() => big.load([]), /still running/);
    assert.throws(() => big.snapshotV1(0), /still running/);
    assert.throws(() => big.summaries(), /still running/);
    const st2 = await pending;
    clearInterval(timer);
    assert.strictEqual(st2.failedDocs, 0);
    assert.deepStrictEqual(big.summaries().map((s) => s.checksum.toString()), syncSums);
    const c4 = new MergeTreeClient();
    c4.applyMsgs(hello);
    const fl = c4.flush();
    assert.throws(() => c4.getText(), /flush\(\) is still running/);
    c4.applyMsg(msg("late", 12, 11, { pos1: 11, seg: "!", type: 0 }));  // staged during the flush
    await fl;
    assert.strictEqual(c4.getText(), "hello world!");  // the late message makes the client dirty again
    // Client.applyMsg interleaved with getText (client.ts:805-836): 10^4 messages of three writers, each
    // op in the view of every message before it (refSeq = seq - 1), minSeq 16 behind; a read at random
    // points equals the edited string and replays only the messages since the read before it
    const ic = new MergeTreeClient("obs");
    let text = "", prev = 0, reads = 0, rnd = 12345;
    const rand = (n) => { rnd = (rnd * 1103515245 + 12345) & 0x7fffffff; return rnd % n; };
    for (let seq = 1; seq <= 10000; seq++) {
        let c;
        if (text.length > 0 && rand(10) < 4) {
            const a = rand(text.length), b = Math.min(text.length, a + 1 + rand(5));
            c = { pos1: a, pos2: b, type: 1 };
            text = text.slice(0, a) + text.slice(b);
        } else {
            const p = rand(text.length + 1), sg = "abcdef".slice(0, 1 + rand(6));
            c = { pos1: p, seg: sg, type: 0 };
            text = text.slice(0, p) + sg + text.slice(p);
        }
        ic.applyMsg(msg("w" + rand(3), seq, seq - 1, c, Math.max(0, seq - 16)));
        if (rand(400) === 0 || seq === 10000) {
            assert.strictEqual(ic.getText(), text);
            assert.strictEqual(ic.getLength(), text.length);
            assert.strictEqual(ic.resumedOps(), reads ? prev : 0);
            prev = seq;
            reads++;
        }
    }
    assert.strictEqual(ic.replays, reads);
    console.log(JSON.stringify({ ops: st.ops, checksums: sums.map((s) => s.checksum.toString()), async_ticks: ticks,
        interleaved_reads: reads }));
})().catch((err) => { console.error(err); process.exit(1); });
