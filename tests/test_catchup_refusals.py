"""How often a catch-up load is refused, on C5-shaped documents.

Each document is a C5-shaped log (tests/catchup.py: 8 writers a few ops behind, MSN lag <= 64), cut
at a random message; the prefix's SnapshotV1 summary (chunk size 10 000 characters, the reference's
default) is loaded and the rest of the log replayed. Three outcomes exist, and the engine must give the
reference's for every document:
- the document loads and catches up (status 0): every summary without body chunks;
- SnapshotLoader.loadBody's never-cleared `batch` (snapshotLoader.ts:196-199) re-appends segments
  already in the tree; when the walk to the append position then fails for a NEW segment, blockInsert
  throws "MergeTree insert failed" (mergeTree.ts:2209-2215) -- the reference's own error, reproduced
  (MTE_DOC_INSERT_FAILED);
- when the walk succeeds for a segment already in the tree, the reference links the same object a
  second time (an aliased tree with stale cached lengths): refused (MTE_DOC_UNSUPPORTED).
The fractions are printed and pinned loosely (the generator is seeded, so they are stable)."""
import collections
import ctypes
import json

import pytest

from fluidframework_amd import mte
from oracle import OracleDoc
from tests.catchup import OBS, body_chunks, catchup_cases
from tests.oplog import dumps

INSERT_FAILED, UNSUPPORTED = 1, 4
_CASES = {}


def cases():
    if not _CASES:
        _CASES["c"] = catchup_cases(8, 20000, seed=2) + catchup_cases(8, 3000, seed=3)
    return _CASES["c"]


def oracle_outcome(summ, suffix):
    o = OracleDoc(OBS)
    if o.load_summary(summ) == 0 and suffix:
        o.apply_json(dumps(suffix))
    return o


def tally(statuses, summaries):
    c = collections.Counter()
    for st, summ in zip(statuses, summaries):
        c[("body" if body_chunks(summ) else "header only", {0: "ok", INSERT_FAILED: "insert failed",
                                                            UNSUPPORTED: "refused"}.get(st, str(st)))] += 1
    return dict(c)


def test_catchup_outcomes_on_the_oracle():
    """The builder's load records replayed by the oracle give the oracle JSON loader's status for
    every document; the outcome fractions on this workload."""
    cs = cases()
    b = mte.Builder()
    for summ, suffix, _ in cs:
        b.add_doc_from_summary(summ, suffix, observer=OBS)
    batch = b.batch()
    statuses = []
    for d, (summ, suffix, log) in enumerate(cs):
        ref = oracle_outcome(summ, suffix)
        rec = OracleDoc(OBS)
        rec.apply_batch(ctypes.addressof(batch), d)
        assert rec.status()[0] == ref.status()[0], (d, rec.status(), ref.status())
        if ref.status()[0] == 0:
            full = OracleDoc(OBS)
            full.apply_json(dumps(log))
            assert ref.text() == full.text(), d  # a loaded catch-up ends where the full replay does
        statuses.append(ref.status()[0])
    t = tally(statuses, [c[0] for c in cs])
    print("catch-up outcomes (oracle):", json.dumps({f"{a} / {b}": v for (a, b), v in sorted(t.items())}))
    assert t.get(("header only", "ok"), 0) == 8, t
    body = {k[1]: v for k, v in t.items() if k[0] == "body"}
    assert sum(body.values()) == 8 and body.get("insert failed", 0) >= 1, t


@pytest.mark.gpu
def test_catchup_outcomes_on_gpu():
    """The same documents on the GPU: every status equal to the oracle's (refusals included), every
    loaded document bit-exact (segments, text, SnapshotV1); the refused fraction is printed."""
    from tests.gpu_helpers import compare_doc

    cs = cases()
    b = mte.Builder()
    for summ, suffix, _ in cs:
        b.add_doc_from_summary(summ, suffix, observer=OBS)
    batch = b.batch()
    e = mte.Engine(0)
    try:
        e.load(batch)
        e.replay()
        for d in range(len(cs)):
            compare_doc(e, batch, d, observer=OBS)
        t = tally([e.status(d)[0] for d in range(len(cs))], [c[0] for c in cs])
        print("catch-up outcomes (GPU):", json.dumps({f"{a} / {b}": v for (a, b), v in sorted(t.items())}))
    finally:
        e.close()
