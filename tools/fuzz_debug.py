"""GPU debug of tests/test_gpu_fuzz.py::test_random_json_logs_match_oracle[seed] document d: dumps the
engine's and the oracle's text, segment table and snapshot into gpurun_out/fuzzdbg/."""
import ctypes
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402
from oracle import OracleDoc  # noqa: E402
from tests.test_gpu_fuzz import random_json_log  # noqa: E402

seed, doc = int(sys.argv[1]), int(sys.argv[2])
rng = random.Random(1000 + seed)
b = mte.Builder()
logs = []
for i in range(24):
    logs.append(random_json_log(seed * 100 + i, rng.choice([60, 300, 1200])))
    b.add_doc(logs[-1], observer="obs")
batch = b.batch()
e = mte.Engine(0)
e.load(batch)
e.replay()
o = OracleDoc("obs")
o.apply_batch(ctypes.addressof(batch), doc)
def first_diff(a, b):
    n = min(len(a), len(b))
    i = next((k for k in range(n) if a[k] != b[k]), n)
    return i, a[max(0, i - 150): i + 150], b[max(0, i - 150): i + 150]


print("doc_result", e.doc_result(doc))
print("status", e.status(doc), o.status())
for name, g, r in (("segments", e.segments_json(doc), o.segments_json()),
                   ("snapshot", e.snapshot_json(doc), o.snapshot_json())):
    if g == r:
        print(name, "equal", len(g))
    else:
        i, ga, ra = first_diff(g, r)
        print(name, "differ at", i, "of", len(g), len(r))
        print(" gpu:", ga.encode("unicode_escape").decode())
        print(" orc:", ra.encode("unicode_escape").decode())
s = e.summaries()
print("checksum gpu", int(s["checksum"][doc]))
e.close()
