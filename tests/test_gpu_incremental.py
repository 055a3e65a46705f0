"""GPU: incremental replay (mte_retain; reg_engine.hpp ckpt_save / ckpt_resume). Client.applyMsg is
incremental (client.ts:805-836) and readers interleave getText with messages; the engine keeps each
document's row-engine state after a pass and continues it over the new ops of the next. Every read
is checked against the oracle fed the same messages, and the resumed-op counters show the pass did
not replay the old ops again."""
import ctypes
import random

import numpy as np
import pytest

from fluidframework_amd import mte
from oracle import OracleDoc
from tests import regcpu
from tests.catchup import OBS, c5_json_log
from tests.gpu_helpers import compare_batch_checksums, compare_doc
from tests.oplog import dumps

pytestmark = pytest.mark.gpu


def _text(engine_text):
    # (the oracle's Python text is UTF-8: lone surrogates compare in the same form, gpu_helpers.py)
    return engine_text.encode("utf-16-le", "surrogatepass").decode("utf-16-le", "replace")


@pytest.mark.parametrize("seed,reads", [(1, 24), (2, 60)])
def test_client_interleaved_reads_match_oracle(seed, reads):
    """MergeTreeClient over a 10^4-message log (8 writers, lagging refSeqs, minSeq 64 behind): reads
    at random points; at each, getText and getLength equal the oracle client's after the same
    messages, and the pass replayed only the ops since the previous read."""
    msgs = c5_json_log(seed, 10_000)
    rng = random.Random(seed)
    cuts = sorted(rng.sample(range(1, len(msgs)), reads - 1)) + [len(msgs)]
    c = mte.MergeTreeClient(OBS)
    o = OracleDoc(OBS)
    at = 0
    for k, cut in enumerate(cuts):
        for m in msgs[at:cut]:
            c.applyMsg(m)
        assert o.apply_json(dumps(msgs[at:cut])) == 0
        assert _text(c.getText()) == o.text(), f"read {k} after {cut} messages"
        assert c.getLength() == o.length_at(cut, 0)
        # one op record per message in this log: the pass went on from the previous read's state
        assert c.resumed_ops() == (at if k else 0), (k, cut, c.resumed_ops())
        at = cut
    assert c.replays == len(cuts)
    assert c._engine.snapshot_json(0) == o.snapshot_json()


def test_client_reads_without_new_messages_reuse_the_pass():
    msgs = c5_json_log(7, 500)
    c = mte.MergeTreeClient(OBS)
    for m in msgs:
        c.applyMsg(m)
    t = c.getText()
    assert c.getText() == t and c.getLength() == len(t) and c.replays == 1


@pytest.mark.parametrize("seed", range(3))
def test_client_with_properties_and_many_writers(seed):
    """Random JSON logs with properties (the PROPS row engine), markers, group ops and up to 40 writers
    (WIDE): reads every few hundred messages match the oracle's full segment table and snapshot."""
    from tests.test_gpu_fuzz import random_json_log
    msgs = random_json_log(9000 + seed, 2500, n_writers=[8, 20, 40][seed], newline=False, emoji=seed == 1)
    c = mte.MergeTreeClient("obs")
    o = OracleDoc("obs")
    at = 0
    resumed = 0
    for cut in list(range(300, len(msgs), 350)) + [len(msgs)]:
        for m in msgs[at:cut]:
            c.applyMsg(m)
        o.apply_json(dumps(msgs[at:cut]))
        assert _text(c.getText()) == o.text()
        assert c._engine.segments_json(0) == o.segments_json()
        resumed += c.resumed_ops() > 0
        at = cut
    assert c._engine.snapshot_json(0) == o.snapshot_json()
    if seed < 2:  # (40 writers: the WIDE document may outgrow the rows and continue HBM-resident)
        assert resumed > 0, "no read continued from the previous pass"


def _cut_batch(ops, pay, names, cut):
    return regcpu.OneDocBatch(ops[:cut] if cut else ops, pay, names)


def test_solo_document_continues_from_its_checkpoint():
    """A document long enough for k_solo (> solo_min_ops): 25 000 ops, then 40 000 of the same log;
    the second pass continues the solo wave's row engine from op 25 000 and matches the oracle."""
    ops, pay = regcpu.generated(2, 77, 40_000, n_clients=8, seed=1000)
    names = ["__observer__"] + [f"w{i}" for i in range(1, 9)]
    e = mte.Engine(0)
    e.retain(True)
    b1 = _cut_batch(ops, pay, names, 25_000)
    e.load(b1.batch)
    e.replay()
    assert e.get_info("solo") == 1
    b2 = _cut_batch(ops, pay, names, 0)
    e.load(b2.batch)
    e.replay()
    assert e.get_info("resumed_docs") == 1 and e.get_info("resumed_ops") == 25_000
    compare_doc(e, b2.batch, 0)
    e.close()


def test_batch_of_extended_logs_resumes_every_row_document():
    """A batch of 64 documents replayed at a cut of each log, then with the whole logs: every document
    the row engines finished continues (resumed_docs), and every checksum equals the oracle's full
    replay -- also for a document whose log did NOT extend the old one (changed history)."""
    rng = random.Random(3)
    logs = [c5_json_log(500 + i, rng.choice([200, 900, 2000])) for i in range(64)]
    cuts = [rng.randint(1, len(l) - 1) for l in logs]
    e = mte.Engine(0)
    e.retain(True)
    b1 = mte.Builder()
    for l, c in zip(logs, cuts):
        b1.add_doc(l[:c], observer=OBS)
    e.load(b1.batch())
    e.replay()
    b2 = mte.Builder()
    changed = 5  # document 5's history is different: it must replay from its first op
    for i, l in enumerate(logs):
        b2.add_doc(c5_json_log(999, len(l)) if i == changed else l, observer=OBS)
    bt = b2.batch()
    e.load(bt)
    assert e.get_info("resumed_docs") == 0  # (counters of the last pass, before this one)
    e.replay()
    offered = e.get_info("ck_offered")
    assert offered == 63, offered
    # (a document the shared row pool could not hold in the first pass was re-run HBM-resident and
    # left no checkpoint: it replays from op 0)
    resumed, total = e.get_info("resumed_docs"), sum(c for i, c in enumerate(cuts) if i != changed)
    assert 60 <= resumed <= 63, resumed
    assert 0.9 * total <= e.get_info("resumed_ops") <= total
    bad, _, _ = compare_batch_checksums(e, bt)
    assert not bad, bad
    compare_doc(e, bt, changed, observer=OBS)
    # the same batch again continues every document from its end: the same results
    s1 = e.summaries()
    e.replay()
    assert e.get_info("resumed_docs") >= 60
    s2 = e.summaries()
    assert np.array_equal(s1["checksum"], s2["checksum"])
    e.close()


def test_retain_off_replays_from_the_start():
    logs = [c5_json_log(40 + i, 300) for i in range(4)]
    e = mte.Engine(0)
    b = mte.Builder()
    for l in logs:
        b.add_doc(l, observer=OBS)
    bt = b.batch()
    e.load(bt)
    e.replay()
    e.replay()
    assert e.get_info("resumed_docs") == 0
    e.retain(True)
    e.replay()  # (nothing kept yet: the first retained pass starts from op 0)
    assert e.get_info("resumed_docs") == 0
    e.replay()
    assert e.get_info("resumed_docs") == 4
    e.retain(False)
    e.replay()
    assert e.get_info("resumed_docs") == 0
    bad, _, _ = compare_batch_checksums(e, bt)
    assert not bad
    e.close()


def test_mixed_batch_extended_three_times():
    """Retain over a batch that mixes routes: short documents, a document with relative positions
    (FULL kernels; the row engines hand it over at op 0, so it never checkpoints), and one long enough
    for k_solo in every pass. Each of three passes loads longer logs; every checksum equals the oracle's
    full replay of the logs of that pass."""
    from tests.test_relative_pos import relative_log

    rng = random.Random(11)
    logs = [c5_json_log(700 + i, rng.choice([300, 1500])) for i in range(10)]
    rel = relative_log(3, n=600)
    ops, pay = regcpu.generated(2, 91, 60_000, n_clients=8, seed=1000)
    from bench import ops_to_messages
    long_log = ops_to_messages(ops, pay, 0, len(ops))
    e = mte.Engine(0)
    e.retain(True)
    resumed = []
    for frac in (0.4, 0.7, 1.0):
        b = mte.Builder()
        for l in logs:
            b.add_doc(l[:max(1, int(len(l) * frac))], observer=OBS)
        b.add_doc(rel[:max(1, int(len(rel) * frac))], observer=OBS)
        b.add_doc(long_log[:int(len(long_log) * frac)], observer="__observer__")
        bt = b.batch()
        e.load(bt)
        e.replay()
        bad, _, _ = compare_batch_checksums(e, bt)
        assert not bad, (frac, bad)
        resumed.append(e.get_info("resumed_docs"))
    # the bulk stays on k_rows (rows_mixed): the ten short documents and the long one (24 000+ ops in
    # every pass, k_solo's row engine) continue in passes 2 and 3; the relative-position document
    # hands over at op 0 each pass and replays from its start
    assert resumed == [0, 11, 11], resumed
    e.close()
