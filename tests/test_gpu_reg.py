"""GPU: the row-vectorised solo engine (fluidframework_amd/csrc/reg_engine.hpp) that replays lean
critical-path documents on k_solo, and its handoff to the LDS engine (reg_handoff.hpp). Every case is
bit-exact against the oracle: checksums (text + SnapshotV1 blobs) and, for a document that differs,
the full segment table."""
import ctypes

import numpy as np
import pytest

from fluidframework_amd import mte
from tests.gpu_helpers import compare_batch_checksums, compare_doc

pytestmark = pytest.mark.gpu

MODE_ROWS = 4  # DocRes.mode: solo, replayed start to end by the row engine
MODE_SOLO_LDS = 3  # solo, LDS engine (from the start, or after a handoff)


@pytest.fixture(scope="module")
def engine():
    e = mte.Engine(0)
    e.set_option("solo_min_ops", 1)  # one-document batches take the solo route
    yield e
    e.set_option("reg_lb_limit", 0)
    e.close()


def _check(engine, batch, n_docs=1):
    bad, _, _ = compare_batch_checksums(engine, batch, threads=min(16, n_docs))
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad


@pytest.mark.parametrize("kind,n_ops,clients", [(2, 1, 2), (2, 60, 3), (2, 3000, 8), (5, 3000, 8),
                                                (2, 40_000, 8), (5, 40_000, 16), (2, 8000, 31)])
def test_row_engine_lone_documents(engine, kind, n_ops, clients):
    engine.set_option("reg_lb_limit", 0)
    engine.generate(kind, 1, n_ops, n_clients=clients, seed=17)
    batch = engine.export_batch()
    st = engine.replay()
    assert engine.run_info()["solo"] == 1 and engine.run_info()["lean"] == 1
    r = engine.doc_result(0)
    assert r["status"] == 0 and st["ops"] == n_ops, r
    # a 31-writer document outgrows the row plan (more than 240 leaf blocks) and finishes on the LDS
    # engine; every other one stays on the rows
    assert r["mode"] == (MODE_SOLO_LDS if clients == 31 else MODE_ROWS), r
    _check(engine, batch)


@pytest.mark.parametrize("limit", [1, 20, 40])
def test_row_engine_hands_off_mid_document(engine, limit):
    """reg_lb_limit shrinks the row plan: the document moves to the LDS engine at op 0 (limit 1) or
    part-way (its leaf blocks pass limit - 16) and the result is unchanged."""
    engine.set_option("reg_lb_limit", limit)
    try:
        engine.generate(2, 1, 6000, n_clients=8, seed=23)
        batch = engine.export_batch()
        engine.replay()
        r = engine.doc_result(0)
        assert r["status"] == 0 and r["mode"] == MODE_SOLO_LDS, r
        _check(engine, batch)
    finally:
        engine.set_option("reg_lb_limit", 0)


@pytest.mark.parametrize("n_ops,clients,limit", [(3000, 8, 0), (40_000, 8, 0), (8000, 16, 0), (6000, 8, 20),
                                                (6000, 8, 40)])
def test_props_row_engine_lone_documents(engine, n_ops, clients, limit):
    """A property-carrying (kind 3) critical-path document on k_solo's PROPS row engine (mode 4) from
    start to end, or handed to the LDS engine part-way with its property map ids and map table
    (reg_lb_limit 20 / 40: mode 3); checksums with the SnapshotV1 property blobs against the oracle."""
    engine.set_option("reg_lb_limit", limit)
    try:
        engine.generate(3, 1, n_ops, n_clients=clients, seed=17)
        batch = engine.export_batch()
        st = engine.replay()
        assert engine.run_info()["solo"] == 1 and engine.run_info()["lean"] == 0
        r = engine.doc_result(0)
        assert r["status"] == 0 and st["ops"] == n_ops, r
        assert r["mode"] == (MODE_SOLO_LDS if limit else MODE_ROWS), r
        _check(engine, batch)
    finally:
        engine.set_option("reg_lb_limit", 0)


@pytest.mark.parametrize("kind,gid,n_ops,clients,rows", [(3, 2, 1100, 40, True), (2, 3, 1200, 48, True),
                                                         (3, 4, 1100, 63, True), (2, 0, 6000, 48, False),
                                                         (3, 0, 5000, 40, False)])
def test_wide_row_engine_lone_documents(engine, kind, gid, n_ops, clients, rows):
    """Documents with writers 32..63 (FULL batches) on k_solo's PROPS + WIDE row engine: the second
    removers word per slot (mode 4 to the end: the documents the CPU suite checks the same way); the
    longer ones outgrow the row plan and hand over to the LDS engine (mode 3, or 2 when they outgrow
    its plan too) with their high overlap bits in its HBM mask (F_OVLHI). Checksums against the
    oracle."""
    engine.set_option("reg_lb_limit", 0)
    engine.generate(kind, 1, n_ops, n_clients=clients, seed=1000, doc_ids=[gid])
    batch = engine.export_batch()
    st = engine.replay()
    assert engine.run_info()["solo"] == 1 and engine.run_info()["lean"] == 0
    r = engine.doc_result(0)
    assert r["status"] == 0 and st["ops"] == n_ops, r
    _check(engine, batch)
    assert r["mode"] == MODE_ROWS if rows else r["mode"] in (2, MODE_SOLO_LDS), r


def test_props_zipf_head_on_rows(engine):
    """The head of a Zipf kind-3 batch runs on k_solo's PROPS row engine (mode 4); the rest of the
    batch on k_rows' PROPS engine beside it; every checksum against the oracle."""
    from fluidframework_amd.shard import zipf_op_counts

    counts = zipf_op_counts(1024, seed=3, lo=100, hi=100_000)
    engine.generate(3, len(counts), 0, n_clients=8, seed=5, ops_per_doc=counts)
    batch = engine.export_batch()
    st = engine.replay()
    assert st["failed_docs"] == 0 and engine.run_info()["solo"] >= 1
    head = int(np.argmax(counts))
    assert engine.doc_result(head)["mode"] == MODE_ROWS, engine.doc_result(head)
    _check(engine, batch, n_docs=len(counts))


def test_row_engine_off_equals_on(engine):
    """The same documents with the row engine disabled (LDS solo engine) give the same checksums."""
    engine.generate(5, 1, 20_000, n_clients=8, seed=29)
    engine.replay()
    assert engine.doc_result(0)["mode"] == MODE_ROWS
    a = engine.summaries()["checksum"].copy()
    engine.set_option("reg_solo", 0)
    try:
        engine.replay()
        assert engine.doc_result(0)["mode"] == MODE_SOLO_LDS
        b = engine.summaries()["checksum"].copy()
    finally:
        engine.set_option("reg_solo", 1)
    assert a.tolist() == b.tolist()


def test_row_engine_markers_and_builder_logs(engine):
    """Marker inserts (no properties: still a lean batch) through the JSON builder, concurrent
    writers; the row engine replays them and the segment tables equal the oracle's."""
    import random

    from tests.oplog import dumps, ins, msg, rem
    from oracle import OracleDoc

    rng = random.Random(5)
    d = OracleDoc()
    msgs, refs, seq = [], {c: 0 for c in "abcd"}, 0
    order = []
    for _ in range(3000):
        c = rng.choice("abcd")
        refs[c] = rng.randint(refs[c], seq)
        if c not in order:
            order.append(c)
        short = order.index(c) + 1
        L = d.length_at(refs[c], short)
        if L == 0 or rng.random() < 0.55:
            seg = {"marker": {"refType": rng.choice([0, 1, 2])}} if rng.random() < 0.15 else \
                "".join(rng.choice("xyz") for _ in range(rng.randint(1, 6)))
            contents = ins(rng.randint(0, L), seg)
        else:
            a = rng.randint(0, L - 1)
            contents = rem(a, min(L, a + rng.randint(1, 9)))
        seq += 1
        m = msg(c, seq, refs[c], contents, min(refs.values()))
        msgs.append(m)
        d.apply_json(dumps([m]))
    b = mte.Builder()
    b.add_doc(dumps(msgs))
    batch = b.batch()
    engine.load(batch)
    engine.replay()
    assert engine.run_info()["lean"] == 1
    assert engine.doc_result(0)["mode"] == MODE_ROWS
    compare_doc(engine, batch, 0)


MODE_BULK_ROWS = 5  # DocRes.mode: k_rows (bulk documents on the row engine)
MODE_ROWS_CONTINUED = 6  # k_rows, then HBM-resident in the same pass (outgrew the row plan)


@pytest.mark.parametrize("waves", [4, 8, 12])
@pytest.mark.parametrize("kind", [2, 5])
def test_bulk_rows_kernel_matches_oracle(engine, kind, waves):
    """Lean bulk documents on k_rows (4 single-document waves per CU on fixed 20-row LDS quarters, or
    8 / 12 taking slot rows from one 79-row LDS pool per CU): a Zipf mix whose longest document stays on k_solo, every other one on
    the rows, checksums against the oracle; then documents held to 24 leaf blocks (reg_lb_limit) that
    are re-run HBM-resident."""
    from fluidframework_amd.shard import zipf_op_counts

    engine.set_option("reg_lb_limit", 0)
    engine.set_option("rows_bulk", waves)
    try:
        counts = zipf_op_counts(3000, seed=kind + waves, lo=50, hi=60_000)
        engine.generate(kind, len(counts), 0, n_clients=8, seed=29, ops_per_doc=counts)
        batch = engine.export_batch()
        st = engine.replay()
        assert st["failed_docs"] == 0 and engine.get_info("rows") == waves
        modes = [engine.doc_result(d)["mode"] for d in range(len(counts))]
        # the longest documents may take k_solo (4); a document the pool cannot grow is re-run
        # HBM-resident (1)
        # (at most 16 solo documents: every other document stays on the rows)
        assert set(modes) <= {MODE_BULK_ROWS, MODE_ROWS, 1}, sorted(set(modes))
        assert modes.count(MODE_BULK_ROWS) >= len(counts) - 16, (modes.count(1), engine.run_info())
        assert modes.count(1) == engine.run_info()["spilled"]
        _check(engine, batch, n_docs=len(counts))
        # documents that outgrow the rows between two ops (reg_lb_limit shrinks them): on fixed rows
        # (4 waves) they continue HBM-resident in the same pass (mode 6, k_rows_cont), none goes
        # back to the host; on the shared pool the host re-runs them from their first op
        engine.set_option("reg_lb_limit", 24)
        engine.generate(kind, 64, 6000, n_clients=8, seed=31)
        batch = engine.export_batch()
        st = engine.replay()
        info = engine.run_info()
        modes = [engine.doc_result(d)["mode"] for d in range(64)]
        if waves == 4:
            assert st["failed_docs"] == 0 and info["spilled"] == 0 and info["rows_continued"] > 0, info
            assert set(modes) <= {MODE_BULK_ROWS, MODE_ROWS_CONTINUED, MODE_ROWS, MODE_SOLO_LDS}, sorted(set(modes))
            assert modes.count(MODE_ROWS_CONTINUED) == info["rows_continued"], (modes, info)
        else:
            assert st["failed_docs"] == 0 and info["spilled"] > 0 and info["rows_continued"] == 0, info
        _check(engine, batch, n_docs=64)
    finally:
        engine.set_option("rows_bulk", -1)
        engine.set_option("reg_lb_limit", 0)


@pytest.mark.parametrize("waves", [8, 12])
def test_bulk_rows_pool_shared_and_exhausted(engine, waves):
    """C2-shaped documents (kind 2, 10^4 ops, 8 writers, leaf blocks peaking near 100) on the shared
    row pool, bit-exact against the oracle; then 31-writer documents too large for twelve (or eight)
    at once in 79 rows: the waves that cannot grow spill mid-op and the host re-runs them."""
    engine.set_option("rows_bulk", waves)
    try:
        engine.generate(2, 2048, 10_000, n_clients=8, seed=1000)
        batch = engine.export_batch()
        st = engine.replay()
        assert st["failed_docs"] == 0 and engine.get_info("rows") == waves
        modes = [engine.doc_result(d)["mode"] for d in range(2048)]
        assert modes.count(MODE_BULK_ROWS) >= 2048 - 16, (modes.count(1), engine.run_info())
        _check(engine, batch, n_docs=2048)
        engine.generate(2, 1024, 4000, n_clients=31, seed=4)
        batch = engine.export_batch()
        st = engine.replay()
        assert st["failed_docs"] == 0 and engine.run_info()["spilled"] > 0
        _check(engine, batch, n_docs=1024)
    finally:
        engine.set_option("rows_bulk", -1)


@pytest.mark.parametrize("waves", [4, 8, 12])
def test_bulk_rows_props_matches_oracle(engine, waves):
    """Property-carrying batches on k_rows' PROPS engine (C3's mix: 45/35/20 insert / remove /
    annotate, property maps per segment, merges only between matching maps): a Zipf mix and a
    C3-shaped batch, every checksum (text + SnapshotV1 blobs with the properties) against the
    oracle."""
    from fluidframework_amd.shard import zipf_op_counts

    engine.set_option("rows_bulk", waves)
    try:
        counts = zipf_op_counts(2000, seed=waves, lo=50, hi=30_000)
        engine.generate(3, len(counts), 0, n_clients=8, seed=41, ops_per_doc=counts)
        batch = engine.export_batch()
        st = engine.replay()
        assert st["failed_docs"] == 0 and engine.get_info("rows") == waves and engine.run_info()["lean"] == 0
        modes = [engine.doc_result(d)["mode"] for d in range(len(counts))]
        assert modes.count(MODE_BULK_ROWS) >= len(counts) - 16, (modes.count(1), engine.run_info())
        _check(engine, batch, n_docs=len(counts))
        engine.generate(3, 1024, 10_000, n_clients=8, seed=1000)
        batch = engine.export_batch()
        st = engine.replay()
        assert st["failed_docs"] == 0
        modes = [engine.doc_result(d)["mode"] for d in range(1024)]
        assert modes.count(MODE_BULK_ROWS) >= 1024 - 16, (modes.count(1), engine.run_info())
        _check(engine, batch, n_docs=1024)
    finally:
        engine.set_option("rows_bulk", -1)


@pytest.mark.parametrize("pool", [40, 56])
def test_bulk_rows_restart_queue(engine, pool):
    """k_rows' in-pass restart queue, forced: C2-shaped documents (leaf blocks peaking near 100, i.e.
    up to 13 slot rows) at 12 waves per CU on a pool shrunk to `pool` rows (option rows_pool), so
    waves find it full at their documents' peaks, give a document up after the bounded wait and queue
    it to restart from its first op. Asserts that documents were pushed and restarted in the pass
    (run_info rows_restart_pushed / _popped), that restarts finished on the rows (fewer host re-runs
    than pushes, every document mode 5 or re-run), and every checksum against the oracle."""
    engine.set_option("rows_bulk", 12)
    engine.set_option("rows_pool", pool)
    try:
        engine.generate(2, 2048, 10_000, n_clients=8, seed=1000)
        batch = engine.export_batch()
        st = engine.replay()
        info = engine.run_info()
        print(f"pool {pool}: {info}")
        assert st["failed_docs"] == 0 and info["rows"] == 12, info
        pushed, popped = info["rows_restart_pushed"], info["rows_restart_popped"]
        assert pushed > 0 and popped > 0 and popped <= pushed, info
        modes = [engine.doc_result(d)["mode"] for d in range(2048)]
        assert set(modes) <= {MODE_BULK_ROWS, 1} and modes.count(1) == info["spilled"], sorted(set(modes))
        assert info["spilled"] < pushed, info  # at least one restarted document finished on the rows
        _check(engine, batch, n_docs=2048)
    finally:
        engine.set_option("rows_pool", 0)
        engine.set_option("rows_bulk", -1)


def test_local_documents_keep_the_lds_engine(engine):
    """A lean batch of local (non-collaborative) documents and no solo document: the row engine does
    not replay local edits, so the batch must not take k_rows (its waves would hand every document to
    the host's HBM re-run); it runs on k_lds / k_hbmq with no re-run. Local edits apply in order, so
    each document's text is checked against the same edits on a Python string (the oracle's record
    path replays sequenced logs only)."""
    from tests.oplog import ins, msg, rem

    logs, texts = [], []
    for d in range(96):
        ops, text = [], ""
        for i in range(300 + d):
            if len(text) > 20 and i % 5 == 4:
                a = (i * 7) % (len(text) - 5)
                ops.append(msg("local", 0, 0, rem(a, a + 3)))
                text = text[:a] + text[a + 3:]
            else:
                t, at = f"t{d}.{i} ", (i * 13) % (len(text) + 1)
                ops.append(msg("local", 0, 0, ins(at, t)))
                text = text[:at] + t + text[at:]
        logs.append(ops)
        texts.append(text)
    b = mte.Builder()
    for m in logs:
        b.add_doc(m, observer="")
    engine.load(b.batch())
    st = engine.replay()
    info = engine.run_info()
    assert st["failed_docs"] == 0 and info["lean"] == 1 and info["solo"] == 0, info
    assert engine.get_info("rows") == 0 and info["spilled"] == 0, info
    assert [engine.text(d) for d in range(96)] == texts


@pytest.mark.parametrize("kind,clients", [(2, 40), (3, 48), (2, 63), (3, 63)])
def test_bulk_rows_wide_batches(engine, kind, clients):
    """Batches with writers 32..63 (FULL) on k_rows' WIDE engine (a second removers word per slot),
    auto route: 4 waves per CU on fixed rows. 1 024 documents of 300 ops stay on the rows to the end
    (mode 5, no continuation, no host re-run); 256 documents of 600 ops outgrow the 16 rows (their
    leaf blocks pass ~110: minSeq trails 40+ writers, so zamboni settles little) and every one of
    them continues HBM-resident in the pass (mode 6), none re-run by the host. Every checksum
    against the oracle."""
    engine.set_option("rows_bulk", -1)
    engine.generate(kind, 1024, 300, n_clients=clients, seed=1000)
    batch = engine.export_batch()
    st = engine.replay()
    info = engine.run_info()
    assert st["failed_docs"] == 0 and info["rows"] == 4 and info["lean"] == 0, info
    assert info["spilled"] == 0 and info["rows_continued"] == 0, info
    modes = [engine.doc_result(d)["mode"] for d in range(1024)]
    assert modes.count(MODE_BULK_ROWS) == 1024, sorted(set(modes))
    _check(engine, batch, n_docs=1024)
    engine.generate(kind, 256, 600, n_clients=clients, seed=1000)
    batch = engine.export_batch()
    st = engine.replay()
    info = engine.run_info()
    assert st["failed_docs"] == 0 and info["rows"] == 4 and info["spilled"] == 0, info
    modes = [engine.doc_result(d)["mode"] for d in range(256)]
    assert set(modes) <= {MODE_BULK_ROWS, MODE_ROWS_CONTINUED}, sorted(set(modes))
    assert modes.count(MODE_ROWS_CONTINUED) == info["rows_continued"] > 0, info
    _check(engine, batch, n_docs=256)


def test_mixed_batch_bulk_stays_on_rows():
    """A FULL batch whose bulk is mostly row-engine documents plus a few the row engines cannot replay
    -- summaries with a catch-up suffix, relative positions, a property-carrying document with '\\n',
    a local (non-collaborative) one -- runs its bulk on k_rows' fixed rows (option rows_mixed); those
    few hand over at op 0 and continue HBM-resident (DocRes mode 6). Every document equals the oracle;
    with rows_mixed off the same batch takes k_lds / k_hbmq with the same results."""
    import random as _r

    from tests.catchup import OBS, c5_json_log, catchup_cases
    from tests.gpu_helpers import compare_batch_checksums, compare_doc
    from tests.oplog import ins, msg, rem
    from tests.test_relative_pos import relative_log
    from tests.test_summary_load import OBS as REL_OBS

    engine = mte.Engine(0)

    rng = _r.Random(5)
    b = mte.Builder()
    for i in range(80):
        b.add_doc(c5_json_log(900 + i, rng.choice([200, 800, 1600])), observer=OBS)
    special = []
    for summ, suffix, _ in catchup_cases(3, 800, seed=9):
        special.append(b.n_docs())
        b.add_doc_from_summary(summ, suffix, observer=OBS)
    for s in (1, 2):
        special.append(b.n_docs())
        b.add_doc(relative_log(s, n=300), observer=REL_OBS)
    special.append(b.n_docs())
    b.add_doc([msg("w1", 1, 0, ins(0, {"text": "a\nb", "props": {"k": 1}})), msg("w2", 2, 1, ins(1, "zz"))],
              observer=OBS)
    special.append(b.n_docs())  # local edits (observer "")
    b.add_doc([msg("local", 0, 0, ins(0, "hello world")), msg("local", 0, 0, rem(2, 5))], observer="")
    batch = b.batch()
    observers = [OBS] * 83 + [REL_OBS] * 2 + [OBS, ""]
    try:
        results = {}
        for mixed in (1, 0):
            engine.set_option("rows_mixed", 2 * mixed)  # (2: even for a bulk of short documents)
            engine.load(batch)
            st = engine.replay()
            info = engine.run_info()
            assert engine.get_info("rows_mixed") == mixed and engine.get_info("rows") == (4 if mixed else 0), info
            bad, _, s = compare_batch_checksums(engine, batch)
            local = len(observers) - 1  # (the oracle's record path replays sequenced logs only)
            bad = [d for d in bad if d != local]
            if bad:
                compare_doc(engine, batch, bad[0], observer=observers[bad[0]])
            assert not bad, bad
            assert engine.status(local)[0] == 0 and engine.text(local) == "he world"
            if mixed:
                modes = [engine.doc_result(d)["mode"] for d in special]
                assert all(m in (6, 1) for m in modes), modes  # continued in the pass (or the host's re-run)
                assert sum(engine.doc_result(d)["mode"] == 5 for d in range(80)) == 80
            results[mixed] = (st["failed_docs"], [int(x) for x in s["checksum"]])
        assert results[1] == results[0]
    finally:
        engine.close()


def test_lean_batch_with_local_documents_stays_on_rows():
    """A lean batch (no properties, no '\n') of row-engine documents plus two local (non-collaborative)
    ones: the bulk stays on k_rows (4 waves), the local documents hand over at op 0 to the lean HBM
    engine; every collaborative document equals the oracle, the local ones their edited strings."""
    from tests.catchup import OBS, c5_json_log
    from tests.gpu_helpers import compare_batch_checksums
    from tests.oplog import ins, msg, rem

    b = mte.Builder()
    for i in range(60):
        b.add_doc(c5_json_log(1200 + i, 600), observer=OBS)
    b.add_doc([msg("local", 0, 0, ins(0, "hello world")), msg("local", 0, 0, rem(0, 6))], observer="")
    b.add_doc([msg("local", 0, 0, ins(0, "abc")), msg("local", 0, 0, ins(1, "XY"))], observer="")
    batch = b.batch()
    e = mte.Engine(0)
    e.set_option("rows_mixed", 2)  # (2: even for a bulk of short documents)
    try:
        e.load(batch)
        st = e.replay()
        info = e.run_info()
        assert st["failed_docs"] == 0 and info["lean"] == 1 and e.get_info("rows") == 4, info
        assert e.get_info("rows_mixed") == 1
        bad, _, _ = compare_batch_checksums(e, batch)
        assert [d for d in bad if d < 60] == []
        assert e.text(60) == "world" and e.text(61) == "aXYbc"
        assert [e.doc_result(d)["mode"] for d in (60, 61)] == [6, 6]
    finally:
        e.close()
