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


def random_json_log(seed, n_msgs, n_writers=None, newline=None, emoji=None, text_max=6, extra="", n_keys=3):
    """A random sequenced log through the JSON path: 2-100 writers with lagging refSeqs (minSeq
    trails), text with '\\n' and surrogate pairs now and then, markers with a refType, annotates
    (rewrite too) with property values incl. null, removes, group ops; every position valid in its
    writer's view (the oracle's length_at)."""
    from oracle import OracleDoc
    from tests.oplog import ann, dumps, group, ins, msg, rem

    rng = random.Random(seed)
    n_writers = n_writers or rng.choice([2, 3, 8, 20, 40, 70, 100])
    names = [f"w{i}" for i in range(n_writers)]
    d = OracleDoc("obs")
    order, refs, out, seq = [], {}, [], 0
    nl = rng.random() < 0.3 if newline is None else newline
    em = rng.random() < 0.3 if emoji is None else emoji
    alphabet = "abcdefxyz" + ("\n" if nl else "") + ("\U0001F600" if em else "") + extra
    keys = ["bold", "size", "color"] + [f"k{j}" for j in range(max(0, n_keys - 3))]
    for _ in range(n_msgs):
        c = rng.choice(names)
        if c not in order:
            order.append(c)
        short = order.index(c) + 1
        lag = rng.randint(0, 6)
        refs[c] = max(refs.get(c, 0), seq - lag, 0)
        ref = refs[c]
        L = d.length_at(ref, short)

        def one(L):
            r = rng.random()
            if L == 0 or r < (0.6 if L < 300 else 0.4):
                if rng.random() < 0.1:
                    seg = {"marker": {"refType": rng.choice([0, 1, 2])}}
                else:
                    seg = {"text": "".join(rng.choice(alphabet) for _ in range(rng.randint(1, text_max)))}
                    if rng.random() < 0.2:
                        seg["props"] = {"k": rng.choice([1, "v", None, True])}
                return ins(rng.randint(0, L), seg), 1
            a = rng.randint(0, L - 1)
            b = min(L, a + rng.randint(1, 8))
            if r < 0.8:
                return rem(a, b), -(b - a)
            props = {rng.choice(keys): rng.choice([True, 12, "red", None, {"n": [1, "x"]}, 0.5])
                     for _ in range(rng.randint(1, 3))}
            return ann(a, b, props, {"name": "rewrite"} if rng.random() < 0.2 else None), 0

        if L > 4 and rng.random() < 0.08:  # a group of two ops: the second sees the first (same client)
            o1, d1 = one(L)
            o2, _ = one(L + d1)
            contents = group(o1, o2)
        else:
            contents, _ = one(L)
        seq += 1
        msn = min(refs[x] for x in order) if len(order) == n_writers else 0
        m = msg(c, seq, ref, contents, msn)
        d.apply_json(dumps([m]))
        if d.status()[0] != 0:
            out.append(None)
            break
        out.append(m)
    return [m for m in out if m is not None]


@pytest.mark.parametrize("seed", range(16))
def test_random_json_logs_match_oracle(engine, seed):
    """Random JSON logs (many writers, markers, properties, rewrite annotates, group ops, '\\n' and
    surrogate pairs) through the builder: 24 documents per batch on whatever route the batch takes,
    every status and checksum against the oracle's record path."""
    rng = random.Random(1000 + seed)
    b = mte.Builder()
    for i in range(24):
        b.add_doc(random_json_log(seed * 100 + i, rng.choice([60, 300, 1200])), observer="obs")
    batch = b.batch()
    engine.load(batch)
    st = engine.replay()
    info = engine.run_info()
    print(f"seed {seed}: lean {info['lean']} rows {info['rows']} solo {info['solo']} "
          f"modes {sorted({engine.doc_result(d)['mode'] for d in range(24)})} failed {st['failed_docs']}")
    bad, _, _ = compare_batch_checksums(engine, batch, threads=16)
    if bad:
        compare_doc(engine, batch, bad[0], observer="obs")
    assert not bad, bad


@pytest.mark.parametrize("seed", range(6))
def test_random_json_logs_legacy_format(seed):
    """The same kind of random JSON logs emitted in the reference's default format (SnapshotLegacy:
    header, body and the catch-up messages above minSeq, rewritten from their delta records): every
    document's legacy tree equals the oracle's JSON-path tree byte for byte."""
    import json as _json

    from oracle import OracleDoc
    from tests.gpu_helpers import first_diff
    from tests.oplog import dumps

    rng = random.Random(2000 + seed)
    logs = [random_json_log(5000 + seed * 100 + i, rng.choice([40, 200, 700])) for i in range(16)]
    b = mte.Builder()
    for lg in logs:
        b.add_doc(lg, observer="obs")
    e = mte.Engine(0, snapshot_format=1)
    try:
        e.load(b.batch())
        e.replay()
        for d, lg in enumerate(logs):
            o = OracleDoc("obs")
            o.apply_json(dumps(lg))
            assert o.status()[0] == 0 and e.status(d)[0] == 0, (d, o.status(), e.status(d))
            want, got = o.snapshot_legacy_json(), e.snapshot_legacy(d)
            if got != want:
                i, ga, oa = first_diff(got, want)
                raise AssertionError(f"doc {d}: legacy tree differs at {i}\n gpu: {ga}\n orc: {oa}")
            _json.loads(got)
    finally:
        e.close()


@pytest.mark.parametrize("seed,writers,newline,emoji", [(0, 3, False, False), (1, 8, True, False),
                                                        (2, 40, False, True), (3, 100, True, True)])
def test_random_json_log_on_the_solo_route(engine, seed, writers, newline, emoji):
    """One long random JSON log alone (k_solo: the FULL row engine to the end, or handing over to the
    LDS plan -- '\n' in the payload at the start, a client above 63 at its first op): full segment
    table, text and snapshot against the oracle."""
    engine.set_option("solo_min_ops", 1)
    try:
        b = mte.Builder()
        b.add_doc(random_json_log(9000 + seed, 6000, writers, newline, emoji), observer="obs")
        batch = b.batch()
        engine.load(batch)
        engine.replay()
        assert engine.run_info()["solo"] == 1
        print(f"seed {seed}: mode {engine.doc_result(0)['mode']}")
        compare_doc(engine, batch, 0, observer="obs")
    finally:
        engine.set_option("solo_min_ops", 20000)


@pytest.mark.parametrize("seed", range(6))
def test_random_summary_catch_up(engine, seed):
    """Resume from a summary: random JSON logs cut at a random point, the oracle's SnapshotV1 summary of
    the prefix (merge info above minSeq, body chunks for long documents) loaded by the builder with the
    rest of the log as the catch-up suffix; the engine's final state against the oracle's record path
    (status, segment table, text, snapshot) and against the oracle loading the same summary."""
    import json as _json

    from oracle import OracleDoc
    from tests.oplog import dumps

    rng = random.Random(3000 + seed)
    cases = []
    for i in range(16):
        log = random_json_log(7000 + seed * 100 + i, rng.choice([80, 400, 1500]))
        k = rng.randint(1, len(log) - 1)
        o = OracleDoc("obs")
        o.apply_json(dumps(log[:k]))
        assert o.status()[0] == 0
        cases.append((o.snapshot_json(), log[k:]))
    b = mte.Builder()
    for summ, suffix in cases:
        b.add_doc_from_summary(summ, suffix, observer="obs")
    batch = b.batch()
    engine.load(batch)
    st = engine.replay()
    print(f"seed {seed}: failed {st['failed_docs']} statuses {sorted({engine.status(d)[0] for d in range(16)})}")
    for d, (summ, suffix) in enumerate(cases):
        compare_doc(engine, batch, d, observer="obs")
        if engine.status(d)[0]:
            continue  # (a summary the loader refuses: compare_doc matched the oracle's status)
        ref = OracleDoc("obs")
        assert ref.load_summary(summ) == 0
        ref.apply_json(dumps(suffix))
        gtext = engine.text(d).encode("utf-16-le", "surrogatepass").decode("utf-16-le", "replace")
        assert gtext == ref.text(), d
        assert _json.loads(engine.snapshot_json(d)) == _json.loads(ref.snapshot_json()), d
