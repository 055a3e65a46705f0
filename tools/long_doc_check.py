"""Parity probe for long documents: generate, replay, compare every document's checksum with the
oracle; print the engine's per-document record of the first mismatches and a full diff of one."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402
from tests.gpu_helpers import compare_batch_checksums, compare_doc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", type=int, default=2)
ap.add_argument("--docs", type=int, default=64)
ap.add_argument("--ops", type=int, default=50000)
ap.add_argument("--force-hbm", type=int, default=0)
ap.add_argument("--hw", type=int, default=8)
a = ap.parse_args()
e = mte.Engine(0)
e.generate(a.kind, a.docs, a.ops, n_clients=8, seed=1000)
batch = e.export_batch()
e.set_option("force_hbm", a.force_hbm)
e.set_option("hbm_waves_per_cu", a.hw)
st = e.replay()
print(json.dumps({**st, **e.run_info()}), flush=True)
bad, _, _ = compare_batch_checksums(e, batch)
print("bad", len(bad), bad[:20], flush=True)
for d in bad[:5]:
    print(d, e.doc_result(d), flush=True)
good = [d for d in range(a.docs) if d not in bad][:3]
for d in good:
    print("good", d, e.doc_result(d), flush=True)
if bad:
    try:
        compare_doc(e, batch, bad[0])
    except AssertionError as ex:
        print(str(ex)[:3000])
