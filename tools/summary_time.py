"""Replay a generated batch and time the host summary path (download of the final state + SnapshotV1
blobs + checksums, mte_summaries). Usage (GPU box): python tools/summary_time.py [--kind 3 --docs 8192]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", type=int, default=3)
ap.add_argument("--docs", type=int, default=8192)
ap.add_argument("--ops", type=int, default=10000)
a = ap.parse_args()
e = mte.Engine(0)
e.generate(a.kind, a.docs, a.ops, n_clients=8, seed=3)
st = e.replay()
t0 = time.perf_counter()
e.text(0)  # final-state download
t1 = time.perf_counter()
s = e.summaries()
t2 = time.perf_counter()
print(json.dumps({"kind": a.kind, "docs": a.docs, "kernel_ms": st["kernel_ms"], "download_s": t1 - t0,
                  "summaries_s": t2 - t1, "snapshot_bytes": int(s["snapshot_bytes"].sum()),
                  "failed": st["failed_docs"]}))
