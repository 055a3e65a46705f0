"""The reference's client.getPosition and client.walkSegments specs (packages/dds/merge-tree/src/test/
client.getPostion.spec.ts, client.walkSegments.spec.ts), restated as sequenced observer logs.

Text a TestClient types before `startOrUpdateCollaboration` is universal (seq 0); each
`insertTextLocal` of one character is its own segment (getContainingSegment(4) is "o" at offset 0),
so the setup is a loaded SnapshotV1 header of one-character segments. A local remove the spec makes
and then sequences (`makeOpMessage`) is the same remove as a sequenced message here. The observer's
segment table stands in for the spec's segment object: a segment's getPosition is the visible length
of the table's rows before it, and a segment zamboni has detached is absent from the table.

Pins:
- getPosition "Existing Segment" (:29-32): "o" sits at 4;
- "Deleted Segment" (:34-39): removed but not yet collected, it is still in the tree at 4;
- "Detached Segment" (:41-57): the remove at seq 1, then eleven appends whose MSN reaches each
  previous seq: zamboni (mergeTree.ts:1422-1478, scourNode :1289-1365) drops the tombstone, so the
  segment is gone from the tree (getPosition -1) -- the one zamboni outcome a reference spec states;
- "Moved Segment" (:59-63): removing the "l" before it moves "o" to 3;
- walkSegments (:22-64): two universal segments walk as 2 segments of total length 10, over the whole
  document and over [3, 7); with splitRange the walk first splits at 3 and 7 (ensureIntervalBoundary)
  and visits "lo" and "wo", 2 segments of total length 4. An annotate of [3, 7) makes the same two
  boundaries on the observer (annotateRange splits like walkSegments' splitRange, mergeTree.ts:
  2565-2605), so the table holds exactly those two annotated segments.
Each case runs on the oracle here and on the GPU (test_client_specs_on_gpu), bit-exact against the
oracle there as well."""
import json

import pytest

from oracle import OracleDoc
from tests.oplog import ann, dumps, ins, msg, rem

OBS = "observer"
USER = "localUser"


def universal_segments(parts):
    """A SnapshotV1 header holding `parts` as separate settled segments at sequence number 0."""
    total = sum(len(p) for p in parts)
    header = {"version": "1", "segmentCount": len(parts), "length": total, "segments": list(parts),
              "startIndex": 0,
              "headerMetadata": {"minSequenceNumber": 0, "sequenceNumber": 0,
                                 "orderedChunkMetadata": [{"id": "header"}], "totalLength": total,
                                 "totalSegmentCount": len(parts)}}
    return json.dumps({"entries": [{"mode": "100644", "path": "header", "type": "Blob",
                                    "value": {"contents": json.dumps(header), "encoding": "utf-8"}}]})


HELLO = list("hello world")


def case_existing():
    return HELLO, [], {"o_pos": 4, "o_removed": False, "text": "hello world"}


def case_deleted():
    return HELLO, [msg(USER, 1, 0, rem(4, 5))], {"o_pos": 4, "o_removed": True, "text": "hell world"}


def case_detached():
    m = [msg(USER, 1, 0, rem(4, 5))]
    length = 10
    for c in "hello world":  # makeOpMessage(op, currentSeq + 1, currentSeq, undefined, currentSeq)
        seq = len(m) + 1
        m.append(msg(USER, seq, seq - 1, ins(length, c), seq - 1))
        length += 1
    return HELLO, m, {"o_pos": None, "text": "hell worldhello world"}


def case_moved():
    return HELLO, [msg(USER, 1, 0, rem(3, 4))], {"o_pos": 3, "o_removed": False, "text": "helo world"}


POSITION_CASES = {"existing (29)": case_existing, "deleted (34)": case_deleted, "detached (41)": case_detached,
                  "moved (59)": case_moved}


def first_o(segs):
    """The first table row whose text is "o" (the spec's segment: "hello world"[4]) and its position:
    the visible length of the rows before it, or (None, None) when no such row is left."""
    pos = 0
    for s in segs:
        if s.get("text") == "o":
            return s, pos
        if "removedSeq" not in s:
            pos += len(s.get("text", ""))
    return None, None


def check_position(segs, text, want):
    assert text == want["text"]
    seg, pos = first_o(segs)
    if want["o_pos"] is None:
        # detached: the removed "o" is gone (the only "o" rows left are the appended text's, live)
        assert all("removedSeq" not in s for s in segs), segs
        assert seg is None or pos > 4, segs
        return
    assert seg is not None and pos == want["o_pos"], (segs, pos)
    assert ("removedSeq" in seg) == want["o_removed"], seg


def run_oracle(parts, msgs):
    o = OracleDoc(OBS)
    assert o.load_summary(universal_segments(parts)) == 0, o.status()
    if msgs:
        assert o.apply_json(dumps(msgs)) == 0, o.status()
    return o


@pytest.mark.parametrize("case", sorted(POSITION_CASES))
def test_get_position_spec_on_oracle(case):
    parts, msgs, want = POSITION_CASES[case]()
    o = run_oracle(parts, msgs)
    check_position(json.loads(o.segments_json()), o.text(), want)


def test_detached_needs_the_msn():
    """The control of "Detached Segment": the same appends with the MSN held at 0 leave the
    tombstone in the tree (zamboni only collects at or below the MSN)."""
    parts, msgs, _ = case_detached()
    held = [dict(m, minimumSequenceNumber=0) for m in msgs]
    o = run_oracle(parts, held)
    seg, pos = first_o(json.loads(o.segments_json()))
    assert seg is not None and seg.get("removedSeq") == 1 and pos == 4


def walk_cases():
    """(parts, msgs, expected table rows as (text, annotated)) for the three walkSegments cases."""
    whole = (["hello", "world"], [], [("hello", False), ("world", False)])
    split = (["hello", "world"], [msg(USER, 1, 0, ann(3, 7, {"walk": 1}))],
             [("hel", False), ("lo", True), ("wo", True), ("rld", False)])
    return {"walk all segments (22)": whole, "walk segment range (35)": whole,
            "walk segment range with split (50)": split}


def check_walk(segs, rows):
    got = [(s["text"], bool(s.get("props"))) for s in segs]
    assert got == rows, segs
    visited = [s for s in segs if s.get("props")] if any(r[1] for r in rows) else segs
    assert len(visited) == 2
    assert sum(len(s["text"]) for s in visited) == (4 if any(r[1] for r in rows) else 10)


@pytest.mark.parametrize("case", sorted(walk_cases()))
def test_walk_segments_spec_on_oracle(case):
    parts, msgs, rows = walk_cases()[case]
    o = run_oracle(parts, msgs)
    check_walk(json.loads(o.segments_json()), rows)


@pytest.mark.gpu
def test_client_specs_on_gpu():
    """Every case above in one GPU batch: the pinned positions / walks from the device's segment
    table, and the table, text and SnapshotV1 equal to the oracle's."""
    from fluidframework_amd import mte

    cases = [POSITION_CASES[c]() for c in sorted(POSITION_CASES)]
    walks = [walk_cases()[c] for c in sorted(walk_cases())]
    b = mte.Builder()
    for parts, msgs, _ in cases + walks:
        b.add_doc_from_summary(universal_segments(parts), msgs or None, observer=OBS)
    e = mte.Engine(0)
    try:
        e.load(b.batch())
        assert e.replay()["failed_docs"] == 0
        for d, (parts, msgs, want) in enumerate(cases):
            segs = json.loads(e.segments_json(d))
            check_position(segs, e.text(d), want)
            o = run_oracle(parts, msgs)
            assert e.segments_json(d) == o.segments_json(), d
            assert e.snapshot_json(d) == o.snapshot_json(), d
        for i, (parts, msgs, rows) in enumerate(walks):
            d = len(cases) + i
            check_walk(json.loads(e.segments_json(d)), rows)
            o = run_oracle(parts, msgs)
            assert e.segments_json(d) == o.segments_json(), d
            assert e.snapshot_json(d) == o.snapshot_json(), d
    finally:
        e.close()
