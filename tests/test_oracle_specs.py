"""Restatements of the reference's merge-tree spec tests as observer replays on the oracle.

Expected values are the literal expectations of the reference tests (file:line cited per case)."""
import json

import pytest

from oracle import OracleDoc
from tests.oplog import TestString, ann, dumps, ins, msg, rem


def hello_world_log():
    # mergeTree.markRangeRemoved.spec.ts:13-22 — "local" types "hello world" one char at a time
    msgs = []
    for i, ch in enumerate("hello world"):
        msgs.append(msg("local", i + 1, i, ins(i, ch)))
    return msgs


def replay(msgs, observer="__observer__"):
    d = OracleDoc(observer)
    assert d.apply_json(dumps(msgs)) == 0, d.status()
    return d


def test_hello_world():
    assert replay(hello_world_log()).text() == "hello world"


def test_remote_remove_followed_by_remote_insert():
    # mergeTree.markRangeRemoved.spec.ts:67-85
    m = hello_world_log()
    c = 11
    m.append(msg("remote2", c + 1, c, rem(0, 11)))
    m.append(msg("remote", c + 2, c, ins(0, "text")))
    assert replay(m).text() == "text"


def test_remote_insert_followed_by_remote_remove():
    # mergeTree.markRangeRemoved.spec.ts:87-106
    m = hello_world_log()
    c = 11
    m.append(msg("remote", c + 1, c, ins(0, "text")))
    m.append(msg("remote2", c + 2, c, rem(0, 11)))
    assert replay(m).text() == "text"


def test_remote_remove_all_then_insert():
    # mergeTree.markRangeRemoved.spec.ts:41-50 (remote remove), then an insert that saw it
    m = hello_world_log()
    m.append(msg("remote", 12, 11, rem(0, 11)))
    m.append(msg("remote", 13, 12, ins(0, "text")))
    assert replay(m).text() == "text"


SNAPSHOT_CASES = {
    # snapshot.spec.ts:137-180
    "below_msn": ([("append", "0", True)], "0"),
    "above_msn": ([("append", "0", False)], "0"),
    "removal_above_msn": ([("append", "0x", False), ("remove", 1, 2, False)], "0"),
    "removal_above_msn_of_seg_below": ([("append", "0x", True), ("remove", 1, 2, False)], "0"),
    "insert_after_removed": ([("append", "0x", True), ("remove", 1, 2, False), ("append", "1", False)], "01"),
    "insert_relative_to_removed": ([("append", "0x", False), ("append", "2", False), ("remove", 1, 2, False),
                                    ("insert", 1, "1", False), ("append", "3", False)], "0123"),
}


@pytest.mark.parametrize("case", sorted(SNAPSHOT_CASES))
def test_snapshot_spec_texts(case):
    steps, expected = SNAPSHOT_CASES[case]
    s = TestString()
    for st in steps:
        if st[0] == "append":
            s.append(st[1], st[2])
        elif st[0] == "insert":
            s.insert(st[1], st[2], st[3])
        else:
            s.remove_range(st[1], st[2], st[3])
    d = replay(s.msgs)
    assert d.text() == expected
    tree = json.loads(d.snapshot_json())
    header = json.loads(tree["entries"][0]["value"]["contents"])
    assert header["headerMetadata"]["sequenceNumber"] == s.seq
    assert header["headerMetadata"]["minSequenceNumber"] == s.min_seq


@pytest.mark.parametrize("increase_msn", [True, False])
def test_snapshot_spec_body_chunks(increase_msn):
    # snapshot.spec.ts:182-203: chunkSize + 10 single-char appends, body chunk emitted
    s = TestString()
    for i in range(10000 + 10):
        s.append(str(i % 10), increase_msn)
    d = replay(s.msgs)
    assert d.text() == s.text
    tree = json.loads(d.snapshot_json())
    paths = [e["path"] for e in tree["entries"]]
    assert paths[0] == "header"
    if not increase_msn:  # merge-info segments cannot coalesce: the body chunk must exist
        assert len(paths) >= 2
    total = 0
    for e in tree["entries"]:
        total += json.loads(e["value"]["contents"])["length"]
    assert total == len(s.text)


def test_annotate_remote_only_and_split():
    # mergeTree.annotate.spec.ts:485-520 ("remote only", "split remote")
    m = [msg("w", 1, 0, ins(0, "hello world")),
         msg("remote", 2, 1, ann(0, 5, {"propertySource": "remote", "remoteProperty": 1})),
         msg("w", 3, 2, ins(2, "X"))]
    d = replay(m)
    segs = json.loads(d.segments_json())
    props = [json.loads(s["props"]) if s["props"] else None for s in segs]
    assert [s["text"] for s in segs] == ["he", "X", "llo", " world"]
    assert props[0] == {"propertySource": "remote", "remoteProperty": 1}
    assert props[2] == {"propertySource": "remote", "remoteProperty": 1}
    assert props[1] is None and props[3] is None


def test_annotate_null_deletes_and_key_order():
    # segmentPropertiesManager.ts:88-104: null deletes, re-add goes to the end; integer keys first
    m = [msg("w", 1, 0, ins(0, "abc")),
         msg("w", 2, 1, ann(0, 3, {"b": 1, "a": 2, "7": "x"})),
         msg("w", 3, 2, ann(0, 3, {"b": None})),
         msg("w", 4, 3, ann(0, 3, {"b": 3, "2": True}))]
    d = replay(m)
    segs = json.loads(d.segments_json())
    assert segs[0]["props"] == '{"2":true,"7":"x","a":2,"b":3}'


def test_insert_failed_beyond_length():
    # mergeTree.ts:2210-2216 "MergeTree insert failed"
    m = [msg("w", 1, 0, ins(0, "ab")), msg("w", 2, 1, ins(5, "x"))]
    d = OracleDoc()
    d.apply_json(dumps(m))
    code, err, seq = d.status()
    assert code == 1 and seq == 2 and "insert failed" in err


def test_concurrent_insert_tie_break_newer_first():
    # breakTie (mergeTree.ts:2248-2277): two concurrent inserts at the same position — the later-
    # sequenced one (which did not see the earlier) goes before it ("newer segments come first")
    m = [msg("a", 1, 0, ins(0, "xy")),
         msg("b", 2, 1, ins(1, "B")),
         msg("c", 3, 1, ins(1, "C"))]
    assert replay(m).text() == "xCBy"


def test_overlapping_remove_records_overlap_client():
    # markRangeRemoved (mergeTree.ts:2614-2660): first remover wins, later joins removedClientOverlap
    m = [msg("a", 1, 0, ins(0, "hello")),
         msg("b", 2, 1, rem(1, 3)),
         msg("c", 3, 1, rem(0, 4))]
    d = replay(m)
    assert d.text() == "o"
    segs = json.loads(d.segments_json())
    el = [s for s in segs if s.get("text") == "el"][0]
    assert el["removedSeq"] == 2 and el["removedClient"] == "b" and el["overlap"] == ["c"]


def test_c1_conflict_farm_replays_cleanly():
    # BASELINE.json configs[0]: 3 clients, 1k insert/remove ops; the oracle must replay it with no
    # sequencing / insert errors and converge to one text (its own replay is deterministic).
    from tests.workloads import c1_farm_log

    m = c1_farm_log(seed=5)
    assert len(m) == 1000
    a = replay(m, observer="0")
    b = replay(m, observer="0")
    assert a.text() == b.text() and a.snapshot_json() == b.snapshot_json()
