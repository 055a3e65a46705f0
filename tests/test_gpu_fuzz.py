"""GPU: randomised routing sweep. Each case draws a batch (kind 2 / 3 / 5, 2-63 writers, Zipf document
lengths) and engine options that push documents through every route the pass has -- k_solo's row
engine and its handoff to the LDS plan, k_rows at 4 / 8 / 12 waves (lean, PROPS, WIDE), the fixed-row
continuation (k_rows_cont, DocRes mode 6), the shared pool's restart queue (a shrunken pool), the
host's HBM re-run -- and checks every document's status and checksum (text + SnapshotV1 blobs)
against the oracle, then the full segment table and snapshot of the first document that differs."""
import random

import pytest

from fluidframework_amd import mte
from fluidframework_amd.shard import zipf_op_counts
from tests.gpu_helpers import compare_batch_checksums, compare_doc

pytestmark = pytest.mark.gpu

OPTIONS = ("rows_bulk", "reg_lb_limit", "rows_pool", "solo_min_ops")
DEFAULTS = {"rows_bulk": -1, "reg_lb_limit": 0, "rows_pool": 0, "solo_min_ops": 20000}


@pytest.fixture(scope="module")
def engine():
    e = mte.Engine(0)
    yield e
    for k, v in DEFAULTS.items():
        e.set_option(k, v)
    e.close()


def draw(seed):
    rng = random.Random(seed)
    kind = rng.choice([2, 3, 5])
    clients = rng.choice([2, 5, 8, 16, 31, rng.randint(32, 63)])
    n_docs = rng.choice([64, 200, 512])
    hi = rng.choice([800, 3000, 12000]) if clients < 32 else rng.choice([300, 600])
    opts = {"rows_bulk": rng.choice([-1, 4, 8, 12]),
            "reg_lb_limit": rng.choice([0, 0, 24, 48]),
            "rows_pool": rng.choice([0, 0, 48]),
            "solo_min_ops": rng.choice([20000, 1000])}
    return kind, clients, n_docs, hi, opts


@pytest.mark.parametrize("seed", range(16))
def test_random_routes_match_oracle(engine, seed):
    kind, clients, n_docs, hi, opts = draw(seed)
    for k, v in opts.items():
        engine.set_option(k, v)
    try:
        counts = zipf_op_counts(n_docs, seed=seed, lo=20, hi=hi)
        engine.generate(kind, n_docs, 0, n_clients=clients, seed=100 + seed, ops_per_doc=counts)
        batch = engine.export_batch()
        st = engine.replay()
        info = engine.run_info()
        modes = sorted({engine.doc_result(d)["mode"] for d in range(n_docs)})
        print(f"seed {seed}: kind {kind} clients {clients} docs {n_docs} hi {hi} {opts} -> modes {modes} "
              f"rows {info['rows']} spilled {info['spilled']} continued {info['rows_continued']} "
              f"restarts {info['rows_restart_popped']}")
        assert st["failed_docs"] == 0, (st, info)
        bad, _, _ = compare_batch_checksums(engine, batch, threads=16)
        if bad:
            compare_doc(engine, batch, bad[0])
        assert not bad, bad[:8]
    finally:
        for k, v in DEFAULTS.items():
            engine.set_option(k, v)
