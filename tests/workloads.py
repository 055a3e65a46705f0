"""Config C1 (BASELINE.json configs[0]): the merge-tree conflict farm — 3 clients (observer + 2
writers), 1k random insert/remove ops. Mirrors mergeTreeOperationRunner.ts:95-145 with the farm's
debugOptions (client.conflictFarm.spec.ts:31-39): rounds of 1, 2, 3 ... ops, every op of a round issued
against the round-start refSeq, MSN = round-start seq, insertTextLocal when the view is shorter than
minLength 2. random-js (mt19937) is not vendored, so the op stream uses Python's PRNG; the positions are
drawn from each writer's own view length computed by the oracle."""
import random

from oracle import OracleDoc
from tests.oplog import dumps, ins, msg, rem


def c1_farm_log(seed=0, total_ops=1000, writers=("1", "2"), min_length=2):
    rng = random.Random(seed)
    d = OracleDoc("0")  # client 0 is the farm's observer
    msgs = []
    seq = 0
    short = {}
    ops_per_round = 1
    while seq < total_ops:
        round_ref = seq
        for _ in range(min(ops_per_round, total_ops - seq)):
            w = rng.choice(writers)
            if w not in short:
                short[w] = len(short) + 1
            L = d.length_at(round_ref, short[w])
            if L < min_length or rng.random() < 0.5:
                text = "".join(rng.choice("abcdefghij") for _ in range(rng.randint(1, 4)))
                c = ins(rng.randint(0, L), text)
            else:
                a = rng.randint(0, L - 1)
                c = rem(a, rng.randint(a + 1, L))
            seq += 1
            m = msg(w, seq, round_ref, c, round_ref)
            msgs.append(m)
            d.apply_json(dumps([m]))
            assert d.status()[0] == 0, d.status()
        ops_per_round += 1
    return msgs
