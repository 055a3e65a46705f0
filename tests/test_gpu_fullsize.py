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


def test_c5_batch_on_the_bench_route(engine):
    """C5 on the route bench.py takes (BASELINE.json config 5), whole: all 1 024 documents of 10^6
    kind-5 ops (the bench's global ids, equal lengths, so no solo document), replayed by k_rows at 4
    waves per CU on fixed 20-row LDS quarters (mode 5). Every document's status and checksum (text +
    SnapshotV1 blobs) against the oracle (1.02 * 10^9 oracle ops on 16 threads, ~4 min), and the full
    segment table / snapshot of two."""
    from fluidframework_amd.shard import plan_shard

    ids, counts = plan_shard("C5", 1, 0, 1024, 1_000_000)
    assert len(ids) == 1024
    engine.generate(5, len(ids), 1_000_000, n_clients=8, seed=1000, ops_per_doc=counts, doc_ids=ids)
    batch = engine.export_batch()
    st = engine.replay()
    assert st["failed_docs"] == 0
    info = engine.run_info()
    assert engine.get_info("rows") == 4 and info["solo"] == 0 and info["spilled"] == 0, info
    modes = [engine.doc_result(d)["mode"] for d in range(len(ids))]
    assert modes == [5] * len(ids), sorted(set(modes))
    bad, ops, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad and ops == len(ids) * 1_000_000
    for d in (0, 1023):
        compare_doc(engine, batch, d)
    del batch


def test_c3_full_batch(engine):
    """C3 itself (BASELINE.json config 3): 65 536 documents x 10 000 ops with annotates, property
    sets, forced ties and overlapping removes, on the default route (k_rows' PROPS row engine at 12
    waves per CU on the shared row pool, with the in-pass restart queue): every document's status and
    checksum against the oracle; any document the pool could not hold was restarted in the pass or
    re-run by the host, and still matches."""
    engine.generate(3, 65536, 10000, n_clients=8, seed=1000)
    batch = engine.export_batch()
    st = engine.replay()
    assert st["failed_docs"] == 0
    info = engine.run_info()
    assert engine.get_info("rows") == 12 and info["lean"] == 0, info
    print(f"C3 full: spilled {info['spilled']}, restarts pushed {info['rows_restart_pushed']} "
          f"popped {info['rows_restart_popped']}")
    bad, ops, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad and ops == 65536 * 10000
    for d in (0, 32768, 65535):
        compare_doc(engine, batch, d)
