"""Unbounded client ids (client.ts:644-668 getOrAddShortClientId never forgets a client; a container
log gets a new clientId on every reconnect): the builder maps clients to the engine's 128 slots and
reuses a slot once minSeq has passed every op of its client (mte_host.cpp DocBuild::short_id); a
window of more than 64 clients keeps removedClientOverlap of clients 64..127 in a second per-segment
mask (engine.hpp ovl2). CPU:
the oracle's record path (slot ids) against its JSON path (real ids, no cap); GPU: the engine against
the JSON path. Segment tables are not compared: a settled segment's client is immaterial (visibility
and SnapshotV1 name clients only above minSeq) and after a reuse the slot names its last owner."""
import ctypes
import json
import random

import pytest

from fluidframework_amd import mte
from oracle import OracleDoc
from tests.gpu_helpers import compare_doc
from tests.oplog import dumps, ins, msg, rem
from tests.test_container_log import EMPTY_CHUNK, SS, attributes, blob, tree

OBS = "readonly"
UNSUPPORTED = 4


def reconnect_log(n_msgs=1500, per_client=3, lag=6, seed=0):
    """Writers that reconnect under new ids: message i comes from c{i // per_client} (500 ids for
    1 500 messages); refSeq trails the head by at most `lag`, msn = seq - 2*lag."""
    rng = random.Random(seed)
    d = OracleDoc(OBS)
    msgs, order, last_ref = [], [], {}
    for i in range(n_msgs):
        seq = i + 1
        c = f"c{i // per_client}"
        if c not in order:
            order.append(c)
        ref = max(seq - 1 - rng.randint(0, lag - 1), last_ref.get(c, 0), 0)
        last_ref[c] = ref
        L = d.length_at(ref, order.index(c) + 1)
        if L > 4 and rng.random() < 0.4:
            a = rng.randint(0, L - 1)
            contents = rem(a, min(L, a + rng.randint(1, 4)))
        else:
            contents = ins(rng.randint(0, L), "".join(rng.choice("abcxyz") for _ in range(rng.randint(1, 5))))
        m = msg(c, seq, ref, contents, max(0, seq - 2 * lag))
        msgs.append(m)
        d.apply_json(dumps([m]))
        assert d.status()[0] == 0, d.status()
    return msgs


def concurrent_log(n_writers=70, n=200):
    """n_writers all inside the collaboration window (msn stays 0): more than 64 slots at once."""
    out, L = [], 0
    for s in range(1, n + 1):
        w = f"w{(s - 1) % n_writers}"
        out.append(msg(w, s, s - 1, ins(s % (L + 1), f"{s % 10}"), 0))
        L += 1
    return out


def overlap_log(n_writers=100):
    """Removes that overlap across the whole window: w0 inserts the alphabet; w1..w{n-1}, all at
    refSeq 1, remove [2, 10) (w1 first, every later one joins removedClientOverlap, ids up to
    n_writers - 1); then each of them inserts at a position of its own view (the range is gone for
    it, hidden by its overlap bit) and removes a character next to it; msn stays 0."""
    out, seq = [], 0

    def m(w, ref, contents):
        nonlocal seq
        seq += 1
        out.append(msg(f"w{w}", seq, ref, contents, 0))

    m(0, 0, ins(0, "abcdefghijklmnopqrstuvwxyz"))
    for w in range(1, n_writers):
        m(w, 1, rem(2, 10))
    for w in range(1, n_writers):
        m(w, 1, ins(2 + w % 7, f"<{w}>"))
    for w in range(1, n_writers, 3):
        m(w, 1, rem(2 + w % 5, 3 + w % 5))
    return out


def json_oracle(msgs, summary=None):
    o = OracleDoc(OBS)
    if summary is not None:
        assert o.load_summary(json.dumps(summary)) == 0
    o.apply_json(dumps(msgs))
    return o


@pytest.mark.parametrize("seed", range(3))
def test_reconnecting_clients_use_windowed_slots(seed):
    msgs = reconnect_log(seed=seed)
    b = mte.Builder()
    b.add_doc(msgs, observer=OBS)
    batch = b.batch()
    ops = mte.batch_ops(batch)
    assert int(ops["client"].max()) < 128
    assert batch.doc_client_offsets[1] - batch.doc_client_offsets[0] <= 128
    rec = OracleDoc(OBS)
    rec.apply_batch(ctypes.addressof(batch), 0)
    ref = json_oracle(msgs)
    assert rec.status()[0] == ref.status()[0] == 0, (rec.status(), ref.status())
    assert rec.text() == ref.text()
    assert rec.snapshot_json() == ref.snapshot_json()


@pytest.mark.parametrize("log", ["concurrent", "overlap"])
def test_more_than_64_concurrent_clients(log):
    """70 writers at once, and 99 removers overlapping on one range: slots up to 99, the record
    path (slot ids) equals the JSON path (real ids), overlap sets included."""
    msgs = concurrent_log() if log == "concurrent" else overlap_log()
    b = mte.Builder()
    b.add_doc(msgs, observer=OBS)
    batch = b.batch()
    assert int(mte.batch_ops(batch)["client"].max()) >= 64
    rec = OracleDoc(OBS)
    rec.apply_batch(ctypes.addressof(batch), 0)
    ref = json_oracle(msgs)
    assert rec.status()[0] == ref.status()[0] == 0, (rec.status(), ref.status())
    assert rec.text() == ref.text()
    assert rec.snapshot_json() == ref.snapshot_json()
    assert rec.segments_json() == ref.segments_json()


def test_more_than_127_concurrent_clients_is_unsupported():
    b = mte.Builder()
    b.add_doc(concurrent_log(130, 260), observer=OBS)
    rec = OracleDoc(OBS)
    rec.apply_batch(ctypes.addressof(b.batch()), 0)
    assert rec.status()[0] == UNSUPPORTED and rec.status()[2] == 128  # w127 (slot 128 does not exist)


def test_ref_seq_below_min_seq_after_reuse_is_unsupported():
    msgs = reconnect_log(n_msgs=600)  # 200 client ids: slots are reused past the 128th
    bad = dict(msgs[-1])
    bad.update(sequenceNumber=601, referenceSequenceNumber=100, clientId="late", minimumSequenceNumber=590)
    b = mte.Builder()
    b.add_doc(msgs + [bad], observer=OBS)
    rec = OracleDoc(OBS)
    rec.apply_batch(ctypes.addressof(b.batch()), 0)
    assert rec.status()[0] == UNSUPPORTED and rec.status()[2] == 601


def container_log_500():
    """A container log: a SharedString attached by a legacy attach envelope, then 1 500 edits from
    500 client ids (address envelopes)."""
    snap = {"entries": [attributes(SS), blob("header", "{}"), tree("content", [blob("header", EMPTY_CHUNK)])]}
    edits = reconnect_log(seed=7)
    out = [msg("c0", 1, 0, {"address": "ds1", "contents": {"type": "attach", "content": {
        "id": "text", "type": SS, "snapshot": snap}}}, 0)]
    for m in edits:
        w = dict(m)
        w["sequenceNumber"] = m["sequenceNumber"] + 1
        w["referenceSequenceNumber"] = m["referenceSequenceNumber"] + 1
        w["minimumSequenceNumber"] = m["minimumSequenceNumber"] + 1 if m["minimumSequenceNumber"] else 0
        w["contents"] = {"address": "ds1", "contents": {"content": {"address": "text", "contents": m["contents"]},
                                                        "type": "op"}}
        out.append(w)
    expect = [dict(w, contents=m["contents"]) for w, m in zip(out[1:], edits)]
    return out, snap, expect


def test_container_log_with_500_clients():
    log, snap, expect = container_log_500()
    b = mte.Builder()
    assert b.add_container_log(log, observer=OBS) == ["ds1/text"]
    batch = b.batch()
    rec = OracleDoc(OBS)
    rec.apply_batch(ctypes.addressof(batch), 0)
    ref = json_oracle(expect, snap)
    assert rec.status()[0] == ref.status()[0] == 0, (rec.status(), ref.status())
    assert rec.snapshot_json() == ref.snapshot_json()


@pytest.fixture(scope="module")
def engine():
    e = mte.Engine(0)
    yield e
    e.close()


@pytest.mark.gpu
def test_gpu_windowed_clients_match_json_oracle(engine):
    logs = [reconnect_log(seed=s) for s in range(3)]
    b = mte.Builder()
    for m in logs:
        b.add_doc(m, observer=OBS)
    b.add_doc(concurrent_log(130, 260), observer=OBS)
    b.add_doc(concurrent_log(), observer=OBS)
    b.add_doc(overlap_log(), observer=OBS)
    log, snap, expect = container_log_500()
    b.add_container_log(log, observer=OBS)
    batch = b.batch()
    engine.load(batch)
    engine.replay()
    refs = [json_oracle(m) for m in logs] + [None, json_oracle(concurrent_log()), json_oracle(overlap_log()),
                                             json_oracle(expect, snap)]
    for d, ref in enumerate(refs):
        if ref is None:
            assert engine.status(d) == (UNSUPPORTED, 128)
            continue
        assert engine.status(d)[0] == 0
        assert engine.text(d) == ref.text(), d
        assert engine.snapshot_json(d) == ref.snapshot_json(), d
    # overlap sets of clients 64..127 (the second mask word) against the record-path oracle
    for d in (len(logs) + 1, len(logs) + 2):
        compare_doc(engine, batch, d, observer=OBS)


@pytest.mark.gpu
def test_gpu_wide_window_on_the_solo_route(engine):
    """The overlap log alone (a one-document batch takes k_solo): the FULL row engine replays it until
    the first op of a client above 63, then hands the document to the LDS engine, whose second
    overlap word takes clients 64..99; segment table (overlap sets) and snapshot against the oracle."""
    engine.set_option("solo_min_ops", 1)
    try:
        b = mte.Builder()
        b.add_doc(overlap_log(), observer=OBS)
        batch = b.batch()
        engine.load(batch)
        engine.replay()
        assert engine.run_info()["solo"] == 1
        assert engine.doc_result(0)["mode"] == 3, engine.doc_result(0)
        compare_doc(engine, batch, 0, observer=OBS)
    finally:
        engine.set_option("solo_min_ops", 20000)
