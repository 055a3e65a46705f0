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


# ---------------------------------------------------------------------------------------------
# mergeTree.annotate.spec.ts (:15-46 setup; the "collaborating" cases whose local ops end up sequenced)
# as observer replays: "hello world!" below the MSN, a Tile marker at 3 by "remote", then the case's
# annotates of [1, 5) in their sequenced order. Expected: the properties of the segment containing
# position 1 ("el"), literal values from the cited assertions.
def _annotate_base():
    return [msg("init", 1, 0, ins(0, "hello world!"), 1),
            msg("remote", 2, 1, ins(3, {"marker": {"refType": 1}}), 1)]


def _ann_case(steps):
    m = _annotate_base()
    for i, (client, props, rewrite) in enumerate(steps):
        c = ann(1, 5, props)
        if rewrite:
            c["combiningOp"] = {"name": "rewrite"}
        m.append(msg(client, 3 + i, 2 + i, c, 1))
    return m


ANNOTATE_CASES = {
    # :286-305 sequenced local
    "sequenced_local": ([("local", {"propertySource": "local"}, False)], {"propertySource": "local"}),
    # :307-341 sequenced local before remote
    "sequenced_local_before_remote": ([("local", {"propertySource": "local"}, False),
                                       ("remote", {"propertySource": "remote", "remoteProperty": 1}, False)],
                                      {"propertySource": "remote", "remoteProperty": 1}),
    # :343-434 three local changes, all acked in order
    "three_local_changes": ([("local", {"propertySource": "local"}, False),
                             ("local", {"propertySource": "local2", "secondSource": 1}, False),
                             ("local", {"thirdSource": 1}, False)],
                            {"propertySource": "local2", "secondSource": 1, "thirdSource": 1}),
    # :436-483 two local changes with an interleaved remote (the second local op is sequenced last)
    "two_local_interleaved_remote": ([("local", {"propertySource": "local"}, False),
                                      ("remote", {"propertySource": "remote", "remoteOnly": 1,
                                                  "secondSource": "remote"}, False),
                                      ("local", {"secondSource": "local2"}, False)],
                                     {"propertySource": "remote", "remoteOnly": 1, "secondSource": "local2"}),
    # :542-579 remote before sequenced local
    "remote_before_sequenced_local": ([("remote", {"propertySource": "remote", "remoteProperty": 1}, False),
                                       ("local", {"propertySource": "local"}, False)],
                                      {"propertySource": "local", "remoteProperty": 1}),
    # :644-679 rewrite: sequenced local before remote
    "rewrite_sequenced_local_before_remote": ([("local", {"propertySource": "local"}, True),
                                               ("remote", {"propertySource": "remote", "remoteProperty": 1}, False)],
                                              {"propertySource": "remote", "remoteProperty": 1}),
    # :681-729 rewrite: two local changes with an interleaved remote
    "rewrite_two_local_interleaved_remote": ([("local", {"propertySource": "local"}, True),
                                              ("remote", {"propertySource": "remote", "remoteOnly": 1,
                                                          "secondSource": "remote"}, False),
                                              ("local", {"secondSource": "local2"}, True)],
                                             {"secondSource": "local2"}),
}


def props_at(d, pos):
    """Properties of the live segment containing visible position `pos` (getContainingSegment)."""
    at = 0
    for s in json.loads(d.segments_json()):
        if "removedSeq" in s:
            continue
        if at <= pos < at + s["len"]:
            return s, (json.loads(s["props"]) if s["props"] else None)
        at += s["len"]
    raise AssertionError("position beyond the text")


@pytest.mark.parametrize("case", sorted(ANNOTATE_CASES))
def test_annotate_spec_cases(case):
    steps, expected = ANNOTATE_CASES[case]
    d = replay(_ann_case(steps))
    seg, props = props_at(d, 1)
    assert seg["text"] == "el"
    assert props == expected


# mergeTree.insertingWalk.spec.ts:24-174 trees, :179-256 inserts of "a" at the beginning, end and
# middle, with the expected strings. The trees are built by a sequenced writer ("w", MSN held at 0 so
# the 7-child layer stays 7 children, as reloaded/inserted in the reference) and the insert comes from
# another client that saw everything.
def _walk_tree(kind):
    m, seq, text = [], 0, ""

    def add(c, who="w"):
        nonlocal seq
        seq += 1
        m.append(msg(who, seq, seq - 1, c, 0))

    if kind == "single_segment":
        add(ins(0, "hello world"))
        text = "hello world"
        middle = round(len(text) / 2)
    elif kind == "full_single_layer":  # MaxNodesInBlock - 1 = 7 children "0".."6"
        for i in range(7):
            add(ins(len(text), str(i)))
            text += str(i)
        middle = round(8 / 2)
    else:  # "tree_with_removals": "0".."31", a quarter of the text removed from each end
        for i in range(32):
            add(ins(len(text), str(i)))
            text += str(i)
        r = round(len(text) / 4)
        add(rem(0, r))
        text = text[r:]
        add(rem(len(text) - r, len(text)))
        text = text[: len(text) - r]
        middle = round(len(text) / 2)
    return m, seq, text, middle


WALK_CASES = [(k, w) for k in ("single_segment", "full_single_layer", "tree_with_removals")
              for w in ("beginning", "end", "middle")]


def walk_case_log(kind, where):
    m, seq, text, middle = _walk_tree(kind)
    pos = {"beginning": 0, "end": len(text), "middle": middle}[where]
    m.append(msg("x", seq + 1, seq, ins(pos, "a"), 0))
    return m, text[:pos] + "a" + text[pos:]


@pytest.mark.parametrize("kind,where", WALK_CASES)
def test_inserting_walk_spec(kind, where):
    m, expected = walk_case_log(kind, where)
    d = replay(m)
    assert d.text() == expected
    assert d.length() == len(expected)


# properties.spec.ts:10-35 matchProperties cases, observed through zamboni and SnapshotV1 coalescing:
# two adjacent segments with the case's property sets fall below the MSN; they merge into one
# segment exactly when matchProperties holds (scourNode mergeTree.ts:1321-1336, snapshotV1.ts:196-202).
MATCH_CASES = [
    ({"a": "a"}, {"a": "a"}, True),
    ({"a": "a"}, {"a": "b"}, False),
    ({"a": "a", "1": 1}, {"a": "a", "1": 1}, True),
    ({"a": "a", "1": 1}, {"a": "b", "1": 2}, False),
    ({"a": "a"}, {"b": "a"}, False),
    ({"a": "a"}, {"a": "a", "b": "b"}, False),
    ({"c": {"a": "a"}}, {"c": {"a": "a"}}, True),
    ({"c": {"a": "a"}}, {"c": {"a": "b"}}, False),
]


def match_case_log(a, b):
    return [msg("w", 1, 0, ins(0, {"text": "x", "props": a}), 0),
            msg("w", 2, 1, ins(1, {"text": "y", "props": b}), 0),
            msg("v", 3, 2, ins(2, "z"), 2)]


@pytest.mark.parametrize("i", range(len(MATCH_CASES)))
def test_match_properties_spec(i):
    a, b, match = MATCH_CASES[i]
    d = replay(match_case_log(a, b))
    live = [s for s in json.loads(d.segments_json()) if "removedSeq" not in s]
    assert [s["text"] for s in live] == (["xy", "z"] if match else ["x", "y", "z"])
    header = json.loads(json.loads(d.snapshot_json())["entries"][0]["value"]["contents"])
    assert header["segmentCount"] == (2 if match else 3)
