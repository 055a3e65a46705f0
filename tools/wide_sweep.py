"""GPU probe: the suite's random generators over many more seeds than the suite runs -- SharedMatrix cell
logs (tests/test_matrix.py matrix_cell_log), relative-position logs (tests/test_relative_pos.py
relative_log) and random JSON logs (tests/test_gpu_fuzz.py random_json_log) -- each checked against the
oracle (segment tables, snapshots, checksums). Prints one line per family; exits 1 on the first
mismatch, naming it. Usage: python tools/wide_sweep.py [n_seeds]"""
import ctypes
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402
from tests.gpu_helpers import compare_batch_checksums, compare_doc  # noqa: E402
from tests.test_gpu_fuzz import random_json_log  # noqa: E402
from tests.test_matrix import matrix_cell_log, oracle_matrix  # noqa: E402
from tests.test_relative_pos import relative_log  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
e = mte.Engine(0)
bad = 0

# SharedMatrix: vectors' segment tables and snapshots, the matrix summary
logs = [matrix_cell_log(100 + s, total=random.Random(s).choice([300, 900, 2000])) for s in range(n)]
b = mte.Builder()
pairs = [b.add_matrix_log(m, observer="obs") for m in logs]
e.load(b.batch())
e.replay()
for s, (m, (ri, ci)) in enumerate(zip(logs, pairs)):
    o = oracle_matrix(m)
    ok = all(e.segments_json(d) == v.segments_json() and e.snapshot_json(d) == v.snapshot_json()
             for d, v in ((ri, o.rows), (ci, o.cols)))
    ok = ok and json.loads(e.snapshot_matrix(ri, ci)) == json.loads(o.snapshot_json())
    if not ok:
        print(f"matrix seed {100 + s}: MISMATCH", flush=True)
        bad += 1
print(f"matrix: {n} logs, {bad} mismatches", flush=True)

# relative positions
logs = [relative_log(200 + s, n=random.Random(s).choice([200, 600])) for s in range(n)]
b = mte.Builder()
for m in logs:
    b.add_doc(m)
batch = b.batch()
e.load(batch)
e.replay()
rb = 0
for d in range(batch.n_docs):
    try:
        compare_doc(e, batch, d)
    except AssertionError as x:
        print(f"relpos seed {200 + d}: {str(x)[:300]}", flush=True)
        rb += 1
print(f"relpos: {n} logs, {rb} mismatches", flush=True)
bad += rb

# random JSON logs, four batches
jb = 0
for k in range(4):
    rng = random.Random(5000 + k)
    b = mte.Builder()
    for i in range(n):
        b.add_doc(random_json_log(20000 + k * 1000 + i, rng.choice([60, 300, 1500])), observer="obs")
    batch = b.batch()
    e.load(batch)
    e.replay()
    bb, _, _ = compare_batch_checksums(e, batch, threads=16)
    for d in bb[:3]:
        try:
            compare_doc(e, batch, d, observer="obs")
        except AssertionError as x:
            print(f"json batch {k} doc {d}: {str(x)[:300]}", flush=True)
    jb += len(bb)
print(f"json: {4 * n} logs, {jb} mismatches", flush=True)
bad += jb

# generated batches under random engine options (tests/test_gpu_fuzz.py draw), seeds past the suite's
from fluidframework_amd.shard import zipf_op_counts  # noqa: E402
from tests.test_gpu_fuzz import DEFAULTS, draw  # noqa: E402

gb = 0
for seed in range(100, 100 + n):
    kind, clients, n_docs, hi, opts = draw(seed)
    for k, v in opts.items():
        e.set_option(k, v)
    counts = zipf_op_counts(n_docs, seed=seed, lo=20, hi=hi)
    e.generate(kind, n_docs, 0, n_clients=clients, seed=100 + seed, ops_per_doc=counts)
    batch = e.export_batch()
    st = e.replay()
    bb, _, _ = compare_batch_checksums(e, batch, threads=16)
    if bb or st["failed_docs"]:
        print(f"generated seed {seed} {kind} {clients} {n_docs} {hi} {opts}: {len(bb)} mismatches, "
              f"{st['failed_docs']} failed", flush=True)
        gb += 1
    for k, v in DEFAULTS.items():
        e.set_option(k, v)
print(f"generated: {n} batches, {gb} with mismatches", flush=True)
bad += gb

# resume from a summary of a random prefix (the oracle's SnapshotV1), the rest as catch-up
from oracle import OracleDoc  # noqa: E402
from tests.oplog import dumps  # noqa: E402

sb = 0
rng = random.Random(77)
cases = []
for i in range(n):
    log = random_json_log(40000 + i, rng.choice([80, 400, 1500]))
    k = rng.randint(1, len(log) - 1)
    o = OracleDoc("obs")
    o.apply_json(dumps(log[:k]))
    cases.append((o.snapshot_json(), log[k:]))
b = mte.Builder()
for summ, suffix in cases:
    b.add_doc_from_summary(summ, suffix, observer="obs")
batch = b.batch()
e.load(batch)
e.replay()
for d, (summ, suffix) in enumerate(cases):
    try:
        compare_doc(e, batch, d, observer="obs")
        if not e.status(d)[0]:
            ref = OracleDoc("obs")
            ref.load_summary(summ)
            ref.apply_json(dumps(suffix))
            assert json.loads(e.snapshot_json(d)) == json.loads(ref.snapshot_json()), "snapshot vs JSON-path load"
    except AssertionError as x:
        print(f"summary case {d}: {str(x)[:300]}", flush=True)
        sb += 1
print(f"summary: {n} resumed logs, {sb} mismatches", flush=True)
bad += sb
e.close()

# stress: long texts (runs past the 256-unit granularity), quotes, backslashes, control characters,
# non-BMP and combining characters, up to 12 property keys (wide map records), object values
xb = 0
for k in range(2):
    rng = random.Random(6000 + k)
    b = mte.Builder()
    for i in range(n):
        b.add_doc(random_json_log(60000 + k * 1000 + i, rng.choice([100, 500]), text_max=rng.choice([20, 400]),
                                  extra='"\\\x01\t\u00e9\u0301\U0001F680', n_keys=rng.choice([3, 12])), observer="obs")
    batch = b.batch()
    e = mte.Engine(0)
    e.load(batch)
    e.replay()
    bb, _, _ = compare_batch_checksums(e, batch, threads=16)
    for d in bb[:3]:
        try:
            compare_doc(e, batch, d, observer="obs")
        except AssertionError as x:
            print(f"stress batch {k} doc {d}: {str(x)[:300]}", flush=True)
    xb += len(bb)
    e.close()
print(f"stress: {2 * n} logs, {xb} mismatches", flush=True)
bad += xb

# JSON logs without '\n' and with at most 63 writers, so the batches take k_rows (PROPS, WIDE when a
# document has 32+ writers), at the auto route and at 4 / 12 waves
rb2 = 0
for k, waves in enumerate((-1, 4, 12, -1)):
    rng = random.Random(7000 + k)
    b = mte.Builder()
    for i in range(n):
        b.add_doc(random_json_log(70000 + k * 1000 + i, rng.choice([100, 600, 2000]),
                                  n_writers=rng.choice([3, 8, 20] if k < 3 else [40, 60]), newline=False), observer="obs")
    batch = b.batch()
    e = mte.Engine(0)
    e.set_option("rows_bulk", waves)
    e.load(batch)
    e.replay()
    info = e.run_info()
    bb, _, _ = compare_batch_checksums(e, batch, threads=16)
    for d in bb[:3]:
        try:
            compare_doc(e, batch, d, observer="obs")
        except AssertionError as x:
            print(f"json-rows batch {k} doc {d}: {str(x)[:300]}", flush=True)
    print(f"json-rows batch {k}: rows {info['rows']} lean {info['lean']} spilled {info['spilled']} "
          f"continued {info['rows_continued']} mismatches {len(bb)}", flush=True)
    rb2 += len(bb)
    e.close()
print(f"json-rows: {4 * n} logs, {rb2} mismatches", flush=True)
bad += rb2

# the legacy format (SnapshotLegacy with catch-up messages)
lb = 0
el = mte.Engine(0, snapshot_format=1)
rng = random.Random(88)
logs = [random_json_log(50000 + i, rng.choice([40, 200, 700])) for i in range(n)]
b = mte.Builder()
for lg in logs:
    b.add_doc(lg, observer="obs")
el.load(b.batch())
el.replay()
for d, lg in enumerate(logs):
    o = OracleDoc("obs")
    o.apply_json(dumps(lg))
    if o.status()[0] != el.status(d)[0] or (not o.status()[0] and o.snapshot_legacy_json() != el.snapshot_legacy(d)):
        print(f"legacy doc {d}: MISMATCH", flush=True)
        lb += 1
print(f"legacy: {n} logs, {lb} mismatches", flush=True)
bad += lb
el.close()
sys.exit(1 if bad else 0)
