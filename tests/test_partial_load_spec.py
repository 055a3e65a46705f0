"""Restatement of the reference's sequence/src/test/partialLoad.spec.ts "Validate Full Load" (:86-105,
legacy summary format) and "Validate New Format Load" (:107-126, SnapshotV1) as observer logs.

The spec drives one SharedString through MockContainerRuntimeFactory (test-runtime-utils mocks.ts:
191-240) with `applyOperations` (:18-41) until its length reaches 3 x mergeTreeSnapshotChunkSize (5),
summarizes the SECOND, never-writing client with chunk size 5 -- so the summary has body chunks and a
collaboration window -- loads a third client from that summary and asserts its text equals the
summarizer's. The mock sequences each processAllMessages batch with refSeq = the last sequence number
the writer had seen and minimumSequenceNumber = the least refSeq of the clients that ever submitted
(only the writer here; 0 stays 0, mocks.ts:201-211,228-236).

Here the log is replayed by the observer (the summarizer) on the oracle and on the GPU, summarized
at chunk size 5 in both formats, and loaded again; the loaded text must equal the replayed text and
the text the spec's own operations produce (tracked below as a plain list)."""
import json

import pytest

from oracle import OracleDoc
from tests.oplog import dumps, ins, msg, rem

CHUNK = 5  # mergeTreeSnapshotChunkSize (:43)
WRITER, SUMMARIZER = "client1", "client2"


def partial_load_log():
    """(messages, expected text): applyOperations (:18-41) until getLength() >= 15 (:74-77)."""
    items = []  # the writer's view: characters, and None for a marker (getLength counts it, getText not)
    msgs, seq = [], 0
    while len(items) < CHUNK * 3:
        content = str(len(items))  # content = sharedString.getLength().toString()
        ref = seq  # every op of this batch is submitted before processAllMessages
        batch = []
        mod = len(items) % 4
        if mod == 0:
            batch.append(ins(0, content))
            items[0:0] = list(content)
        elif mod == 1:
            pos = len(items) // mod
            batch.append(ins(pos, {"marker": {"refType": 0}}))  # ReferenceType.Simple
            items.insert(pos, None)
        else:
            if mod == 2:
                batch.append(ins(len(items), content))
                items.extend(content)
                pos = len(items) // mod
                batch.append(rem(pos, pos + 1))
                del items[pos]
            batch.append(ins(len(items), content))  # (case 2 falls through)
            items.extend(content)
        for c in batch:
            seq += 1
            msgs.append(msg(WRITER, seq, ref, c, ref))  # msn: the writer's refSeq (the only submitter)
    return msgs, "".join(x for x in items if x is not None)


def test_partial_load_log_shape():
    msgs, text = partial_load_log()
    o = OracleDoc(SUMMARIZER)
    o.apply_json(dumps(msgs))
    assert o.status()[0] == 0 and o.text() == text
    assert len(text) >= 10 and len(msgs) > 6
    # chunk size 5: the SnapshotV1 summary has body chunks, with segments above minSeq (merge info)
    tree = json.loads(o.snapshot_json(CHUNK))
    assert len(tree["entries"]) > 1


@pytest.mark.parametrize("fmt", ["legacy", "v1"])
def test_partial_load_on_the_oracle(fmt):
    """The oracle's summary of the summarizer at chunk size 5, loaded by a new client, has the text."""
    msgs, text = partial_load_log()
    o = OracleDoc(SUMMARIZER)
    o.apply_json(dumps(msgs))
    summ = o.snapshot_json(CHUNK) if fmt == "v1" else o.snapshot_legacy_json(CHUNK)
    c = OracleDoc("client3")
    assert c.load_summary(summ) == 0, c.status()
    assert c.text() == text


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [1, 0])
def test_partial_load_on_gpu(fmt):
    """On the GPU: replay the log as the summarizer, summarize (SnapshotLegacy for "Validate Full
    Load", SnapshotV1 for "Validate New Format Load") at chunk size 5, load a new document from that
    summary, replay it: its text is the summarizer's; the summaries equal the oracle's byte for byte."""
    from fluidframework_amd import mte

    msgs, text = partial_load_log()
    e = mte.Engine(0, chunk_size=CHUNK, snapshot_format=fmt)
    b = mte.Builder()
    b.add_doc(msgs, observer=SUMMARIZER)
    e.load(b.batch())
    e.replay()
    assert e.status(0)[0] == 0 and e.text(0) == text
    o = OracleDoc(SUMMARIZER)
    o.apply_json(dumps(msgs))
    summ = e.snapshot_legacy(0) if fmt == 1 else e.snapshot_json(0)
    assert summ == (o.snapshot_legacy_json(CHUNK) if fmt == 1 else o.snapshot_json(CHUNK))
    e2 = mte.Engine(0, chunk_size=CHUNK, snapshot_format=fmt)
    b2 = mte.Builder()
    b2.add_doc_from_summary(summ, None, observer="client3")
    e2.load(b2.batch())
    e2.replay()
    assert e2.status(0)[0] == 0 and e2.text(0) == text
    e.close()
    e2.close()
