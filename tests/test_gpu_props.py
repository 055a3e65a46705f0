"""GPU: property maps wider than the narrow 7-key record (the batch's map width follows its documents'
distinct keys, up to MTE_MAX_PROPS = 63 per segment), against the oracle's unbounded maps
(properties.ts:95-170, segmentPropertiesManager.ts:35-111): annotates adding up to 20 keys to one
segment, null deletes, rewrite, concurrent annotates, splits and zamboni merges of wide maps
(matchProperties on wide maps), and the SnapshotV1 property objects in JS key order."""
import json
import random

import pytest

from fluidframework_amd import mte
from tests.gpu_helpers import compare_doc
from tests.oplog import ann, dumps, ins, msg, rem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = mte.Engine(0)
    yield e
    e.close()


def _wide_log(seed, n_keys, n_msgs=500):
    """Three concurrent writers; positions drawn from each writer's own view (the oracle's
    getLength(refSeq, client)), so every op is valid for the reference."""
    from oracle import OracleDoc

    rng = random.Random(seed)
    keys = [f"k{i}" for i in range(n_keys)] + ["7", "3", "12"]  # index-like keys sort first in JS order
    vals = [1, 2, "x", True, False, None, {"a": 1}, [1, 2]]
    d = OracleDoc()
    seq, refs, order, msgs = 0, {c: 0 for c in "abc"}, [], []
    for _ in range(n_msgs):
        c = rng.choice("abc")
        refs[c] = rng.randint(max(refs[c], seq - 4), seq)
        if c not in order:
            order.append(c)
        L = d.length_at(refs[c], order.index(c) + 1)
        r = rng.random()
        if L < 20 or r < 0.25:
            seg = "".join(rng.choice("uvw") for _ in range(rng.randint(1, 6)))
            if rng.random() < 0.3:
                seg = {"text": seg, "props": {rng.choice(keys): 1}}
            contents = ins(rng.randint(0, L), seg)
        elif r < 0.35:
            a = rng.randint(0, L - 1)
            contents = rem(a, min(L, a + rng.randint(1, 3)))
        else:
            a = rng.randint(0, L - 1)
            props = {rng.choice(keys): rng.choice(vals) for _ in range(rng.randint(1, 4))}
            contents = ann(a, min(L, a + rng.randint(1, 40)), props, {"name": "rewrite"} if rng.random() < 0.05 else None)
        seq += 1
        m = msg(c, seq, refs[c], contents, min(refs.values()))
        msgs.append(m)
        d.apply_json(dumps([m]))
    assert d.status()[0] == 0, d.status()
    return msgs


@pytest.mark.parametrize("seed,n_keys", [(1, 12), (2, 20), (3, 9)])
def test_wide_property_maps_match_oracle(engine, seed, n_keys):
    logs = [_wide_log(seed * 10 + i, n_keys) for i in range(4)]
    b = mte.Builder()
    for m in logs:
        b.add_doc(dumps(m))
    batch = b.batch()
    engine.load(batch)
    engine.replay()
    for d in range(len(logs)):
        compare_doc(engine, batch, d)
    # at least one segment of the batch carries more keys than the narrow record holds
    widest = max(len(json.loads(s["props"])) for d in range(len(logs)) for s in json.loads(engine.segments_json(d))
                 if s.get("props"))
    assert widest > 7, widest
