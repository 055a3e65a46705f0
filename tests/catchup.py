"""TEST INFRASTRUCTURE: C5-shaped catch-up documents (BASELINE.json config 5's shape: 8 writers, every
writer's refSeq a few ops behind, MSN lagging the current seq by <= 64, long enough that a SnapshotV1
summary has BODY chunks), summarized at a random seq by the oracle and resumed from that summary with
the rest of the log. What fraction of such documents a loader refuses (MTE_DOC_UNSUPPORTED: the
aliased re-link of snapshotLoader.ts:196-199) is measured on this workload.

Positions come from the oracle itself: each message's position range is drawn inside its writer's
view at its refSeq (Client.getLength of that view, mergeTree.ts getLength(refSeq, clientId)), so the
log is a valid sequenced stream with real concurrency."""
import random

from oracle import OracleDoc
from tests.oplog import dumps, ins, msg, rem

OBS = "obs"
LETTERS = "abcdefghijklmnopqrstuvwxyz"


def c5_json_log(seed, n_msgs, writers=8, lag=64, max_behind=3):
    rng = random.Random(seed)
    o = OracleDoc(OBS)
    msgs = []
    msn = 0
    for i in range(n_msgs):
        seq = i + 1
        w = i if i < writers else rng.randrange(writers)
        ref = max(msn, seq - 1 - rng.randint(0, max_behind))
        length = o.length_at(ref, w + 1)  # short ids: observer 0, writer w = w + 1 (first seen in order)
        new_msn = max(msn, seq - lag)
        if length > 0 and rng.random() < 0.3:
            a = rng.randrange(length)
            b = min(length, a + rng.randint(1, 20))
            contents = rem(a, b)
        else:
            t = "".join(rng.choice(LETTERS) for _ in range(rng.randint(1, 12)))
            contents = ins(rng.randint(0, length), t)
        m = msg(f"w{w}", seq, ref, contents, new_msn)
        assert o.apply_json(dumps([m])) == 0, o.status()
        msn = new_msn
        msgs.append(m)
    return msgs


def catchup_cases(n_docs, n_msgs, seed=0, chunk=10000):
    """(summary, suffix, full log) per document: the log cut at a random message, the prefix's
    SnapshotV1 summary (chunk size `chunk` characters) and the rest of the log."""
    rng = random.Random(9000 + seed)
    out = []
    for d in range(n_docs):
        log = c5_json_log(seed * 1000 + d, n_msgs)
        k = rng.randint(n_msgs // 2, n_msgs - 1)
        o = OracleDoc(OBS)
        assert o.apply_json(dumps(log[:k])) == 0
        out.append((o.snapshot_json(chunk), log[k:], log))
    return out


def body_chunks(summary):
    import json

    return len(json.loads(summary)["entries"]) - 1
