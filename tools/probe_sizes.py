"""Probe per-document state sizes after replay (leaf blocks, heap, segments, maps, arena) for the
synthetic workloads; used to size the LDS-resident engine. Run on a GPU box."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402


def probe(kind, docs, ops, clients=8):
    e = mte.Engine(0)
    e.generate(kind, docs, ops, n_clients=clients, seed=7)
    st = e.replay()
    rows = [e.doc_result(d) for d in range(0, docs, max(1, docs // 256))]
    out = {"kind": kind, "docs": docs, "ops": ops, "kernel_ms": st["kernel_ms"], "failed": st["failed_docs"]}
    for k in ("n_lb", "heap_size", "seg_next", "map_next", "height", "arena_top", "n_gc", "min_seq", "cur_seq"):
        v = np.array([r[k] for r in rows], dtype=np.int64)
        out[k] = {"mean": float(v.mean()), "p99": float(np.percentile(v, 99)), "max": int(v.max())}
    e.close()
    return out


if __name__ == "__main__":
    res = []
    for kind, docs, ops in ((2, 1024, 10000), (3, 1024, 10000), (5, 256, 50000), (2, 256, 50000)):
        r = probe(kind, docs, ops)
        print(json.dumps(r), flush=True)
        res.append(r)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_sizes.json", "w") as f:
        json.dump(res, f, indent=1)
