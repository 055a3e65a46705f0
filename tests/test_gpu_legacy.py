"""SnapshotLegacy emission on the GPU (snapshotlegacy.ts:103-238; the reference's default summary format,
client.ts:930-941): header / body chunks written by the device (emit.hip, EmitParams::legacy), the
catch-up blob by the host from the builder's stashed messages and the delta ranges the engine records
for the rewritten ones (sequence.ts:597-634, createOpsFromDelta :58-100).

Pins: the ten reference legacy fixtures (packages/dds/sequence/src/test/snapshots/legacy{,WithCatchUp},
copied as data into tests/golden/) byte-for-byte. Catch-up messages have no reference fixture (parity
unpinned): the engine's whole legacy ITree must equal the oracle's (tests/test_summary_load.py round-trips
the oracle's)."""
import json
import random

import pytest

from fluidframework_amd import mte
from oracle import OracleDoc
from tests.gpu_helpers import dump, first_diff
from tests.oplog import ann, dumps, group, ins, msg, rem
from tests.test_gpu_parity import local_fixture_log
from tests.test_oracle_fixtures import LEGACY_CATCHUP, legacy_fixture_blobs
from tests.workloads import c1_farm_log

pytestmark = pytest.mark.gpu

NAMES = ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"]


@pytest.fixture(scope="module")
def engine():
    e = mte.Engine(0, snapshot_format=1)
    yield e
    e.close()


def test_legacy_golden_fixtures_on_gpu(engine):
    b = mte.Builder()
    for nm in NAMES:
        b.add_doc(local_fixture_log(nm), observer="")
    engine.load(b.batch())
    engine.replay()
    for d, nm in enumerate(NAMES):
        assert engine.status(d)[0] == 0
        for version, cname in sorted(LEGACY_CATCHUP.items()):
            tree = json.loads(engine.snapshot_legacy(d, cname))
            got = [(e["path"], e["value"]["contents"]) for e in tree["entries"]]
            assert got == legacy_fixture_blobs(version, nm), (version, nm)
        # the SharedString tree wraps the legacy merge-tree tree under "content"
        ss = json.loads(engine.snapshot_shared_string(d))
        assert [e["path"] for e in ss["entries"]] == ["header", "content"]
    with pytest.raises(mte.MteError):
        engine.snapshot_json(0)  # the batch was emitted in the legacy format


def rich_log(seed, total_ops=500, writers=("w1", "w2", "w3")):
    """Concurrent writers (rounds against the round-start refSeq, MSN = round start) with text / marker
    inserts carrying props, removes, annotates (some with combiningOp rewrite) and group ops."""
    rng = random.Random(seed)
    d = OracleDoc("obs")
    msgs, seq, short, per_round = [], 0, {}, 1
    while seq < total_ops:
        ref = seq
        for _ in range(min(per_round, total_ops - seq)):
            w = rng.choice(writers)
            short.setdefault(w, len(short) + 1)
            L = d.length_at(ref, short[w])
            r = rng.random()

            def one(L):
                q = rng.random()
                if L < 3 or q < 0.4:
                    t = "".join(rng.choice("abcdefgh") for _ in range(rng.randint(1, 5)))
                    k = rng.random()
                    seg = t if k < 0.6 else ({"text": t, "props": {"b": rng.randint(0, 2)}} if k < 0.85 else
                                             {"marker": {"refType": 1}, "props": {"t": "p"}})
                    return ins(rng.randint(0, L), seg)
                a = rng.randint(0, L - 1)
                e = rng.randint(a + 1, min(L, a + 12))
                if q < 0.75:
                    return rem(a, e)
                props = rng.choice([{"b": 1}, {"c": "x", "b": None}, {"7": True, "b": 2}, {"b": 0}])
                return ann(a, e, props, {"name": "rewrite"} if rng.random() < 0.3 else None)

            if r < 0.15:
                c = group(one(L), ins(0, "G"))  # the first member may shorten the view
            else:
                c = one(L)
            seq += 1
            m = msg(w, seq, ref, c, ref)
            msgs.append(m)
            d.apply_json(dumps([m]))
            assert d.status()[0] == 0, d.status()
        per_round += 1
    return msgs


def test_legacy_catch_up_matches_oracle(engine):
    cases = []
    for seed in range(3):
        log = c1_farm_log(seed=seed, total_ops=400)
        cases += [log[:k] for k in (57, 200, 400)]
    for seed in range(4):
        log = rich_log(seed)
        cases += [log[:k] for k in (90, 333, 500)]
    b = mte.Builder()
    for m in cases:
        b.add_doc(m, observer="obs")
    engine.load(b.batch())
    engine.replay()
    n_catch = 0
    for d, m in enumerate(cases):
        o = OracleDoc("obs")
        o.apply_json(dumps(m))
        assert o.status()[0] == 0 and engine.status(d)[0] == 0, (d, o.status(), engine.status(d))
        want, got = o.snapshot_legacy_json(), engine.snapshot_legacy(d)
        if got != want:
            dump(f"legacy_doc{d}", got, want)
            i, ga, oa = first_diff(got, want)
            raise AssertionError(f"doc {d}: legacy tree differs at {i}\n gpu: {ga}\n orc: {oa}")
        n_catch += len(json.loads(json.loads(got)["entries"][-1]["value"]["contents"]))
    assert n_catch > 60  # the rewrite path is exercised
