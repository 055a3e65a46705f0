"""GPU parity at the configurations' own per-document lengths (BASELINE.json configs 3 and 5), against
the CPU oracle: C3's 10 000-op documents with annotates, property sets, forced ties and overlapping
removes, and a C5 long-history document (10^6 ops, every writer's refSeq within 64 of the current seq,
so zamboni runs on nearly every op) with its SnapshotV1 bytes."""
import pytest

from fluidframework_amd import mte
from tests.gpu_helpers import compare_batch_checksums, compare_doc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = mte.Engine(0)
    yield e
    e.close()


def test_c3_documents_at_full_length(engine):
    """128 kind-3 documents of C3's 10 000 ops each (the FULL kernels: property maps, rewrite-free
    annotates, 15 % forced ties and overlapping removes): checksum of text + SnapshotV1 blobs and
    status of every document, and the full segment table / snapshot of four of them."""
    engine.generate(3, 128, 10000, n_clients=8, seed=1000)
    gen_fail = [d for d in range(128) if engine.status(d)[0]]
    assert not gen_fail, f"generator hit errors: {gen_fail[:5]}"
    batch = engine.export_batch()
    engine.replay()
    bad, ops, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad and ops == 128 * 10000
    for d in (0, 41, 86, 127):
        compare_doc(engine, batch, d)


def test_c5_long_history_document(engine):
    """One C5 document of 10^6 ops (kind 5: MSN lag <= 64, continuous zamboni), replayed alone on the
    critical-path route (k_solo, the row engine): text, segment table and SnapshotV1 bytes."""
    engine.generate(5, 1, 1_000_000, n_clients=8, seed=1000)
    assert engine.status(0)[0] == 0
    batch = engine.export_batch()
    engine.replay()
    assert engine.doc_result(0)["mode"] == 4  # the row-vectorised solo engine replayed it
    bad, ops, _ = compare_batch_checksums(engine, batch, threads=1)
    assert not bad and ops == 1_000_000
    compare_doc(engine, batch, 0)


def test_c2_full_batch(engine):
    """C2 itself (BASELINE.json config 2): 4 096 documents x 10 000 insert/remove ops, 8 writers --
    every document's status and checksum (text + SnapshotV1 blobs) against the oracle, and the full
    segment table / snapshot of four documents."""
    engine.generate(2, 4096, 10000, n_clients=8, seed=1000)
    batch = engine.export_batch()
    st = engine.replay()
    assert st["failed_docs"] == 0
    bad, ops, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad and ops == 4096 * 10000
    for d in (0, 1365, 2730, 4095):
        compare_doc(engine, batch, d)
