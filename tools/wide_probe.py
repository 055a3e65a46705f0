"""GPU probe: batches with writers 32..63 on k_rows' WIDE engine at 4 / 8 / 12 waves per CU against the
LDS / HBM kernels (rows_bulk 0): pass time (median of 3), host re-runs, in-pass restarts, and every
checksum against the oracle once per configuration. One JSON line per configuration to stdout.
Usage: python tools/wide_probe.py [n_docs] [n_ops,...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402
from tests.gpu_helpers import compare_batch_checksums  # noqa: E402

n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
op_list = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "300,600").split(",")]
e = mte.Engine(0)
for kind in (2, 3):
    for clients in (40, 63):
        for n_ops in op_list:
            for waves in (0, 4, 8, 12):
                e.set_option("rows_bulk", waves)
                e.generate(kind, n_docs, n_ops, n_clients=clients, seed=1000)
                batch = e.export_batch()
                ms = []
                for _ in range(3):
                    t = time.perf_counter()
                    st = e.replay()
                    ms.append((time.perf_counter() - t) * 1e3)
                info = e.run_info()
                bad, _, _ = compare_batch_checksums(e, batch, threads=16)
                why = {}
                modes = {}
                for d in range(n_docs):
                    r = e.doc_result(d)
                    modes[r["mode"]] = modes.get(r["mode"], 0) + 1
                    if r["mode"] == 1:
                        k = r["spill_why"] & 0xFF
                        why[k] = why.get(k, 0) + 1
                rec = {"kind": kind, "clients": clients, "n_ops": n_ops, "waves": waves, "rows": info["rows"],
                       "ms": sorted(ms)[1], "kernel_ms": st["kernel_ms"], "failed": st["failed_docs"],
                       "spilled": info["spilled"], "pushed": info["rows_restart_pushed"],
                       "popped": info["rows_restart_popped"], "lean": info["lean"], "solo": info["solo"],
                       "bad": len(bad), "continued": info["rows_continued"], "modes": modes, "why": why}
                print(json.dumps(rec), flush=True)
e.set_option("rows_bulk", -1)
e.close()
