"""relativePos1 / relativePos2 (ops.ts:66-94): positions given relative to a marker id, resolved by
Client.getValidOpRange -> MergeTree.posFromRelativePos -> getPosition (client.ts:493-510,
mergeTree.ts:1943-1966, 1586-1603) in the op's (refSeq, client) view.

The builder turns them into RELPOS records and marker tags (include/mte.h MTE_OP_RELPOS). CPU: the
oracle replays each log twice -- from the JSON (ids by string) and from the builder's records (ids by
tag) -- and both must agree; GPU: the engine against the oracle. The reference has no fixture for
relative positions (parity unpinned beyond the restatement of the functions cited above)."""
import ctypes
import json
import random

import pytest

from fluidframework_amd import mte
from oracle import OracleDoc
from tests.gpu_helpers import compare_doc
from tests.oplog import ann, dumps, ins, msg, rem
from tests.test_summary_load import OBS, fixture, oracle_catchup

UNSUPPORTED = 4


def view(segs, ref, client):
    """(start, visible length) of every segment in the (refSeq, client) view -- nodeLength
    (mergeTree.ts:1659-1699) -- and the view's length."""
    out, pos = [], 0
    for s in segs:
        seen = s["client"] == client or s["seq"] <= ref
        gone = "removedSeq" in s and (s["removedClient"] == client or s["removedSeq"] <= ref or client in s["overlap"])
        v = s["len"] if seen and not gone else 0
        out.append((pos, v))
        pos += v
    return out, pos


def marker_ids(segs):
    ids = []
    for i, s in enumerate(segs):
        if s["kind"] == "M" and s.get("props"):
            p = json.loads(s["props"])
            if isinstance(p, dict) and isinstance(p.get("markerId"), str):
                ids.append((i, p["markerId"]))
    return ids


def rel(mid, before=None, offset=None):
    r = {"id": mid}
    if before is not None:
        r["before"] = before
    if offset is not None:
        r["offset"] = offset
    return r


def relative_log(seed, n=300, clients=("a", "b", "c")):
    """A random valid log with relative inserts / removes / annotates against markers visible in the
    writer's view (positions computed here from the oracle's segment table)."""
    rng = random.Random(seed)
    d = OracleDoc(OBS)
    msgs, refs, seq, n_rel = [], {c: 0 for c in clients}, 0, 0
    for _ in range(n):
        c = rng.choice(clients)
        refs[c] = rng.randint(refs[c], seq)
        segs = json.loads(d.segments_json())
        vw, L = view(segs, refs[c], c)
        cands = [(vw[i][0], mid) for i, mid in marker_ids(segs) if vw[i][1] == 1]
        r = rng.random()
        contents = None
        if cands and r < 0.3:
            P, mid = rng.choice(cands)
            n_rel += 1
            if r < 0.12:  # insert relative to a marker
                seg = rng.choice(["xy", "q", {"marker": {"refType": 1}, "props": {"markerId": f"m{seq + 1}"}}])
                before = rng.random() < 0.5
                if before:
                    off = rng.randint(0, P)
                    contents = {"relativePos1": rel(mid, True, off if off or rng.random() < 0.5 else None), "seg": seg, "type": 0}
                else:
                    off = rng.randint(0, L - P - 1)
                    contents = {"relativePos1": rel(mid, rng.choice([False, None]), off if off or rng.random() < 0.5 else None),
                                "seg": seg, "type": 0}
            else:  # remove / annotate [marker - k, marker + 1 + j) with either end relative
                k, j = rng.randint(0, min(P, 3)), rng.randint(0, min(L - P - 1, 3))
                c2 = {"type": 1} if r < 0.22 else {"type": 2, "props": {"r": rng.randint(0, 2)}}
                mode = rng.randrange(3)
                if mode != 1:
                    c2["relativePos1"] = rel(mid, True, k)
                else:
                    c2["pos1"] = P - k
                if mode != 2:
                    c2["relativePos2"] = rel(mid, None, j)
                else:
                    c2["pos2"] = P + 1 + j
                contents = c2
        elif L == 0 or r < 0.6:
            if rng.random() < 0.15:
                seg = {"marker": {"refType": rng.choice([1, 2, 4])}, "props": {"markerId": f"m{seq + 1}"}}
            else:
                seg = "".join(rng.choice("abcdef") for _ in range(rng.randint(1, 6)))
            contents = ins(rng.randint(0, L), seg)
        elif r < 0.85:
            a = rng.randint(0, L - 1)
            contents = rem(a, min(L, a + rng.randint(1, 6)))
        else:
            a = rng.randint(0, L - 1)
            contents = ann(a, min(L, a + rng.randint(1, 6)), {rng.choice(["b", "i"]): rng.choice([True, None, 3])})
        seq += 1
        m = msg(c, seq, refs[c], contents, min(refs.values()))
        msgs.append(m)
        d.apply_json(dumps([m]))
        assert d.status()[0] == 0, (seed, seq, d.status(), contents)
    assert n_rel > 10
    return msgs


def _dropped():
    """'ZZhe[x]llo', the marker x removed (seq 4) and dropped by zamboni once the msn passes 4, then
    'kk' inserted in front: 'kkZZhello' with x unlinked."""
    return [msg("a", 1, 0, ins(0, "hello")),
            msg("a", 2, 1, ins(2, {"marker": {"refType": 1}, "props": {"markerId": "x"}})),
            msg("b", 3, 2, ins(0, "ZZ")), msg("a", 4, 3, rem(4, 5), 3), msg("b", 5, 4, ins(0, "k"), 5),
            msg("a", 6, 5, ins(0, "k"), 5)]


def edge_logs():
    """(name, log, expected status, failing seq): the cases the engine reports unsupported."""
    base = [msg("a", 1, 0, ins(0, "hello")),
            msg("a", 2, 1, ins(2, {"marker": {"refType": 1}, "props": {"markerId": "x"}})),
            msg("b", 3, 2, ins(0, "ZZ"))]
    cases = [("ok_after", base + [msg("b", 4, 3, {"relativePos1": rel("x"), "seg": "!", "type": 0})], 0, None),
             ("ok_before_offset", base + [msg("c", 4, 2, {"relativePos1": rel("x", True, 2), "seg": "!", "type": 0})], 0, None),
             ("ok_remove_both", base + [msg("b", 4, 3, {"relativePos1": rel("x", True, 1), "relativePos2": rel("x", False, 1),
                                                        "type": 1})], 0, None),
             ("pos1_wins", base + [msg("b", 4, 3, {"pos1": 0, "relativePos1": rel("x"), "seg": "!", "type": 0})], 0, None),
             ("unmapped", base + [msg("b", 4, 3, {"relativePos1": rel("nope"), "seg": "!", "type": 0})], UNSUPPORTED, 4),
             ("no_id", base + [msg("b", 4, 3, {"relativePos1": {"before": True}, "seg": "!", "type": 0})], UNSUPPORTED, 4),
             ("duplicate_id", base + [msg("a", 4, 3, ins(0, {"marker": {"refType": 1}, "props": {"markerId": "x"}})),
                                      msg("b", 5, 4, {"relativePos1": rel("x"), "seg": "!", "type": 0})], UNSUPPORTED, 5),
             ("annotated_id", base + [msg("a", 4, 3, ann(0, 1, {"markerId": "y"})),
                                      msg("b", 5, 4, {"relativePos1": rel("x"), "seg": "!", "type": 0})], UNSUPPORTED, 5),
             # removed but still in the tree (no msn advance): the position is still defined
             ("removed_marker", base + [msg("a", 4, 3, rem(4, 5)),
                                        msg("b", 5, 3, {"relativePos1": rel("x"), "seg": "!", "type": 0})], 0, None),
             # removed below the msn: zamboni unlinks it (scourNode: parent = undefined, mergeTree.ts:1317),
             # getPosition's parent walk is empty -> 0, and the position is 0 + 1 + offset (after) or
             # 0 - offset (before); a position below 0 is not modelled
             ("dropped_marker", _dropped() + [msg("b", 7, 6, {"relativePos1": rel("x"), "seg": "!", "type": 0}, 6)], 0, None),
             ("dropped_marker_before", _dropped() + [msg("b", 7, 6, {"relativePos1": rel("x", True), "seg": "!", "type": 0}, 6)],
              0, None),
             ("dropped_marker_offset", _dropped() + [msg("b", 7, 6, {"relativePos1": rel("x", False, 3),
                                                                     "relativePos2": rel("x", False, 5), "type": 1}, 6)], 0, None),
             ("dropped_marker_below_zero", _dropped() + [msg("b", 7, 6, {"relativePos1": rel("x", True, 1), "seg": "!",
                                                                         "type": 0}, 6)], UNSUPPORTED, 7),
             ("group_member", base + [msg("b", 4, 3, {"type": 3, "ops": [ins(0, "g"), {"relativePos1": rel("x"), "seg": "!", "type": 0}]})],
              0, None)]
    return cases


@pytest.mark.parametrize("seed", range(5))
def test_relative_log_records_match_json(seed):
    msgs = relative_log(seed)
    b = mte.Builder()
    b.add_doc(msgs)
    batch = b.batch()
    ops = mte.batch_ops(batch)
    assert (ops["type"] == 9).sum() > 10 and ((ops["flags"] & 0x100) != 0).sum() == (ops["type"] == 9).sum()
    a, z = OracleDoc(OBS), OracleDoc(OBS)
    a.apply_json(dumps(msgs))
    z.apply_batch(ctypes.addressof(batch), 0)
    assert a.status()[0] == z.status()[0] == 0, (a.status(), z.status())
    assert a.segments_json() == z.segments_json()
    assert a.snapshot_json() == z.snapshot_json()


@pytest.mark.parametrize("case", edge_logs(), ids=[c[0] for c in edge_logs()])
def test_relative_edge_cases(case):
    name, log, code, fseq = case
    b = mte.Builder()
    b.add_doc(log)
    batch = b.batch()
    a, z = OracleDoc(OBS), OracleDoc(OBS)
    a.apply_json(dumps(log))
    z.apply_batch(ctypes.addressof(batch), 0)
    assert a.status()[0] == z.status()[0] == code, (a.status(), z.status())
    if code:
        assert a.status()[2] == z.status()[2] == fseq
    else:
        assert a.snapshot_json() == z.snapshot_json()


def test_dropped_marker_positions():
    """A relative position naming a marker zamboni dropped resolves from 0 (the reference's getPosition
    of an unlinked segment): after it -> 1 + offset, before it -> 0 - offset."""
    texts = {}
    for name, log, code, _ in edge_logs():
        if name.startswith("dropped") and not code:
            o = OracleDoc(OBS)
            o.apply_json(dumps(log))
            assert o.status()[0] == 0, (name, o.status())
            texts[name] = o.text()
    assert texts == {"dropped_marker": "k!kZZhello", "dropped_marker_before": "!kkZZhello",
                     "dropped_marker_offset": "kkZZllo"}, texts


def test_relative_edge_positions():
    """The positions themselves, read back from the text."""
    log = [msg("a", 1, 0, ins(0, "hello")), msg("a", 2, 1, ins(2, {"marker": {"refType": 1}, "props": {"markerId": "x"}})),
           msg("a", 3, 2, {"relativePos1": rel("x"), "seg": "A", "type": 0}),
           msg("a", 4, 3, {"relativePos1": rel("x", True), "seg": "B", "type": 0}),
           msg("a", 5, 4, {"relativePos1": rel("x", False, 2), "seg": "C", "type": 0}),
           msg("a", 6, 5, {"relativePos1": rel("x", True, 3), "seg": "D", "type": 0})]
    o = OracleDoc(OBS)
    o.apply_json(dumps(log))
    assert o.status()[0] == 0
    # D h e B [x] A l C l o (the marker carries no text)
    assert o.text() == "DheBAlClo"


def summary_with_markers():
    """The reference's withMarkers summary (ids marker0, marker70, ...) then relative ops."""
    s = fixture("withMarkers")
    o = oracle_catchup(s, None)
    L = o.length()
    suffix = [msg("w", 1, 0, {"relativePos1": rel("marker70", True), "seg": "R", "type": 0}),
              msg("w", 2, 1, {"relativePos1": rel("marker140"), "relativePos2": rel("marker210", True), "type": 1}),
              msg("w", 3, 2, {"relativePos1": rel("marker0", False, 5), "relativePos2": rel("marker0", False, 9),
                              "props": {"k": 1}, "type": 2}),
              msg("w", 4, 3, {"relativePos1": rel("nothere"), "seg": "R", "type": 0})]
    assert L > 300
    return s, suffix


def test_relative_ops_after_summary_load():
    s, suffix = summary_with_markers()
    b = mte.Builder()
    b.add_doc_from_summary(s, suffix[:3], observer=OBS)
    b.add_doc_from_summary(s, suffix, observer=OBS)
    batch = b.batch()
    for d, suf in enumerate((suffix[:3], suffix)):
        ref = oracle_catchup(s, suf)
        rec = OracleDoc(OBS)
        rec.apply_batch(ctypes.addressof(batch), d)
        assert rec.status()[0] == ref.status()[0] == (0 if d == 0 else UNSUPPORTED)
        if d == 0:
            assert rec.snapshot_json() == ref.snapshot_json()
            assert "R" in ref.text()


def test_builder_still_rejects_registers():
    b = mte.Builder()
    with pytest.raises(mte.MteError):
        b.add_doc([msg("a", 1, 0, {"register": "r", "seg": "q", "type": 0})])


@pytest.fixture(scope="module")
def engine():
    e = mte.Engine(0)
    yield e
    e.close()


@pytest.mark.gpu
def test_gpu_relative_positions_match_oracle(engine):
    logs = [relative_log(s, n=400) for s in range(8)] + [c[1] for c in edge_logs()]
    b = mte.Builder()
    for m in logs:
        b.add_doc(m)
    s, suffix = summary_with_markers()
    b.add_doc_from_summary(s, suffix[:3])
    b.add_doc_from_summary(s, suffix)
    batch = b.batch()
    engine.load(batch)
    engine.replay()
    assert engine.run_info()["lean"] == 0
    for d in range(batch.n_docs):
        compare_doc(engine, batch, d)
    codes = [engine.status(d)[0] for d in range(batch.n_docs)]
    assert codes[:8] == [0] * 8
    assert codes[8:8 + len(edge_logs())] == [c[2] for c in edge_logs()]
    assert codes[-2:] == [0, UNSUPPORTED]


def marker_heavy_log(n_markers=150, n_ann=6):
    """Markers carry no payload: a relative annotate spanning them touches far more segments than
    the document has text characters."""
    msgs, seq, L = [msg("a", 1, 0, ins(0, "xy"))], 1, 2
    for i in range(n_markers):
        seq += 1
        msgs.append(msg("a", seq, seq - 1, ins(L, {"marker": {"refType": 1}, "props": {"markerId": f"m{i}"}})))
        L += 1
    for j in range(n_ann):
        seq += 1
        c = {"type": 2, "relativePos1": rel("m0", True), "relativePos2": rel(f"m{n_markers - 1}"), "props": {"k": j}}
        msgs.append(msg("b" if j % 2 else "a", seq, seq - 1, c))
    return msgs


@pytest.mark.gpu
def test_gpu_marker_heavy_relative_annotates_rerun(engine):
    """The host's re-run pass sizes a re-run document's property-map table from its ops; a relative
    annotate over many markers (length 1, no payload) must count them, or a valid document ends
    MTE_DOC_CAPACITY in the re-run (map_rerun). Forced through the re-run: HBM slots too small."""
    logs = [marker_heavy_log(), marker_heavy_log(60, 12)]
    engine.set_option("slot_blk_limit", 8)
    try:
        b = mte.Builder()
        for m in logs:
            b.add_doc(m)
        batch = b.batch()
        engine.load(batch)
        engine.set_option("force_hbm", 1)
        engine.replay()
        assert engine.run_info()["spilled"] == len(logs)
    finally:
        engine.set_option("force_hbm", 0)
        engine.set_option("slot_blk_limit", 0)
    for d in range(batch.n_docs):
        assert engine.status(d)[0] == 0
        compare_doc(engine, batch, d)
