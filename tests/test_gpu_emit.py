"""GPU: SnapshotV1 emission on the device (emit.hip) -- JSON escaping (quotes, backslashes, control
characters, non-ASCII, surrogate pairs split across segments, lone surrogates), coalesced runs across
elided segments, property objects in JS key order, merge-info entries with client names, chunking --
byte-identical to the oracle's SnapshotV1 (snapshotV1.ts:57-247 restated)."""
import ctypes
import json

import pytest

from fluidframework_amd import mte
from oracle import OracleDoc
from tests.oplog import ann, ins, msg, rem

TEXTS = ['a"b\\c', "\u0001\t\n\b\f\r", "é漢字", "\ud83d", "\ude00", "x\ud800y", "\udfff", "ok", "\U0001F600z"]


def escape_log(collab):
    out, seq, L = [], 0, 0
    for i, t in enumerate(TEXTS * 3):
        seq += 1
        w = f"w{i % 3}" if collab else "local"
        out.append(msg(w, seq, seq - 1, ins(L, t), max(0, seq - 4) if collab else 0))
        L += len(t.encode("utf-16-le", "surrogatepass")) // 2
    seq += 1
    out.append(msg("w0" if collab else "local", seq, seq - 1, ann(0, 6, {"b": 1, "7": True, "2": "s", "a": None}),
                   max(0, seq - 4) if collab else 0))
    seq += 1
    out.append(msg("w1" if collab else "local", seq, seq - 1, rem(3, 9), max(0, seq - 4) if collab else 0))
    return out


def test_escape_logs_records_match_json():
    """CPU: the builder carries lone surrogates and escapes through (oracle record path = JSON path)."""
    log = escape_log(True)
    b = mte.Builder()
    b.add_doc(json.dumps(log))
    batch = b.batch()
    obs = "__observer__"
    a, z = OracleDoc(obs), OracleDoc(obs)
    a.apply_json(json.dumps(log))
    z.apply_batch(ctypes.addressof(batch), 0)
    assert a.status()[0] == z.status()[0] == 0
    assert a.snapshot_json() == z.snapshot_json()
    snap = a.snapshot_json()
    assert "\\\\ud800" in snap and "\U0001F600" in snap  # a lone surrogate stays escaped, a split pair joins


@pytest.mark.gpu
def test_emission_escapes_and_runs():
    """(Local, non-collaborative emission is pinned byte-for-byte by the reference's v1 fixtures,
    test_gpu_parity.py::test_v1_golden_fixtures_on_gpu.)"""
    b = mte.Builder()
    b.add_doc(json.dumps(escape_log(True)))  # ensure_ascii: lone surrogates travel as \\uXXXX
    b.add_doc(json.dumps(escape_log(True)[:-1]))
    batch = b.batch()
    e = mte.Engine(0)
    try:
        e.load(batch)
        e.replay()
        for d in range(2):  # text() is not compared: lone surrogates have no UTF-8 form to compare by
            o = OracleDoc()
            o.apply_batch(ctypes.addressof(batch), d)
            assert e.status(d)[0] == o.status()[0] == 0
            assert e.segments_json(d) == o.segments_json()
            assert e.snapshot_json(d) == o.snapshot_json(), d
        e.set_option("emit", 0)
        e.replay()
        with pytest.raises(mte.MteError):
            e.snapshot_json(0)
        e.set_option("emit", 1)
        e.replay()
        o = OracleDoc()
        o.apply_batch(ctypes.addressof(batch), 1)
        assert e.snapshot_json(1) == o.snapshot_json()
        assert e.get_info("emit_us") >= 0
    finally:
        e.close()


def emptied_log(n, collab=True):
    """n inserts, then one remove of everything; the MSN reaches the remove's seq, so zamboni
    detaches every segment and the final table is empty."""
    out, seq, L = [], 0, 0
    for i in range(n):
        seq += 1
        out.append(msg(f"w{i % 2}" if collab else "local", seq, seq - 1, ins(L, "ab"), seq - 1))
        L += 2
    seq += 1
    out.append(msg("w0" if collab else "local", seq, seq - 1, rem(0, L), seq - 1))
    for _ in range(2):  # the MSN catches up to the remove (empty removes carry it)
        seq += 1
        out.append(msg("w1" if collab else "local", seq, seq - 1, rem(0, 0), seq - 1))
    return out


@pytest.mark.gpu
def test_empty_documents_beside_full_ones():
    """a document with no final segments owns no output rows, so its SnapshotV1
    chunk record must not land on the next document's first row. Empty logs, logs whose every
    segment zamboni detached, and ordinary documents interleaved; every snapshot byte-equal to the
    oracle's."""
    from tests.gpu_helpers import compare_doc

    b = mte.Builder()
    kinds = []
    for i in range(48):
        k = i % 4
        if k == 0:
            b.add_doc(json.dumps([]))
        elif k == 1:
            b.add_doc(json.dumps(emptied_log(5 + i)))
        else:
            b.add_doc(json.dumps(escape_log(True)[: 5 + i % 20]))
        kinds.append(k)
    batch = b.batch()
    e = mte.Engine(0)
    try:
        e.load(batch)
        e.replay()
        for d in range(len(kinds)):
            compare_doc(e, batch, d)
            if kinds[d] < 2:
                assert json.loads(e.snapshot_json(d)) is not None
    finally:
        e.close()
