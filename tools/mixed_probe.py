"""Mixed batches (rows_mixed): a C2-mix batch of generated documents turned into JSON logs, plus a few
documents the row engines cannot replay (relative positions, a summary load), replayed with the bulk on
k_rows (rows_mixed 1) and on k_lds / k_hbmq (rows_mixed 0). Prints pass times and routing; every status
must be 0 in both. Usage (GPU box): python tools/mixed_probe.py [docs] [ops]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import ops_to_messages  # noqa: E402
from fluidframework_amd import mte  # noqa: E402


def main():
    n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n_ops = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    from tests.test_relative_pos import relative_log
    from tests.test_summary_load import OBS as REL_OBS
    g = mte.Engine(0)
    g.generate(2, n_docs, n_ops, n_clients=8, seed=1000)
    b0 = g.export_batch()
    ops = mte.batch_ops(b0).copy()
    npay = b0.doc_payload_offsets[b0.n_docs]
    pay = np.frombuffer(bytes((ctypes.c_uint16 * npay).from_address(ctypes.addressof(b0.payload.contents))), dtype=np.uint16)
    b = mte.Builder()
    t0 = time.time()
    for d in range(n_docs):
        lo, hi, p0 = b0.doc_op_offsets[d], b0.doc_op_offsets[d + 1], b0.doc_payload_offsets[d]
        b.add_doc(ops_to_messages(ops, pay[p0:], lo, hi), observer="__observer__")
    for s in range(4):
        b.add_doc(relative_log(s, n=400), observer=REL_OBS)
    build_s = time.time() - t0
    g.close()
    out = {"docs": n_docs, "ops_per_doc": n_ops, "special_docs": 4, "build_s": round(build_s, 1)}
    if os.environ.get("LEGACY"):  # SnapshotLegacy (the reference's default format): catch-up records
        e = mte.Engine(0, snapshot_format=1)
        e.load(b.batch())
        ms, infos = [], []
        for _ in range(int(os.environ.get("REPS", "3"))):
            ms.append(round(e.replay()["kernel_ms"], 2))
            ri = e.run_info()
            infos.append({k: ri[k] for k in ("spilled", "continued", "lds_ms", "hbm_ms", "hbm_docs", "lds_groups", "hbm_waves")})
        out["legacy"] = {"kernel_ms": ms, "rows": e.get_info("rows"), "per_pass": infos}
        e.close()
    e = mte.Engine(0)
    for mixed in (1, 0):
        e.set_option("rows_mixed", 2 * mixed)  # (2: the rows route even for short documents)
        e.load(b.batch())
        ms, infos = [], []
        for _ in range(int(os.environ.get("REPS", "3"))):
            st = e.replay()
            ms.append(round(st["kernel_ms"], 2))
            ri = e.run_info()
            infos.append({k: ri[k] for k in ("spilled", "continued", "lds_ms", "hbm_ms", "hbm_docs")})
        out[f"mixed{mixed}"] = {"kernel_ms": ms, "failed": st["failed_docs"], "rows": e.get_info("rows"),
                                "rows_mixed": e.get_info("rows_mixed"), "per_pass": infos}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
