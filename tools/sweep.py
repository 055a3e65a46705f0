"""Throughput sweep: LDS-resident pass vs HBM-resident pass over growing batch sizes (concurrency).
Usage (GPU box): python tools/sweep.py [--kind 2 --ops 10000 --docs 2048,4096,8192]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", type=int, default=2)
ap.add_argument("--ops", type=int, default=10000)
ap.add_argument("--docs", default="2048,4096,8192")
ap.add_argument("--modes", default="lds,hbm")
ap.add_argument("--hw", default="12", help="hbm_waves_per_cu values tried in lds mode")
a = ap.parse_args()
for nd in [int(x) for x in a.docs.split(",")]:
    e = mte.Engine(0)
    e.generate(a.kind, nd, a.ops, n_clients=8, seed=3)
    runs = []
    for mode in a.modes.split(","):
        runs += [(mode, int(h)) for h in a.hw.split(",")] if mode == "lds" else [(mode, 0)]
    for mode, hw in runs:
        e.set_option("force_hbm", 1 if mode == "hbm" else 0)
        e.set_option("hbm_waves_per_cu", hw)
        e.replay()
        t = time.perf_counter()
        st = e.replay()
        dt = time.perf_counter() - t
        info = e.run_info()
        if st["failed_docs"]:
            info["fail_codes"] = sorted({(e.doc_result(d)["status"], e.doc_result(d)["mode"]) for d in range(nd)
                                         if e.doc_result(d)["status"]})
        print(json.dumps({"docs": nd, "mode": mode, "hw": hw, "ops": st["ops"], "wall_ms": dt * 1e3,
                          "kernel_ms": st["kernel_ms"], "mops": st["ops"] / st["kernel_ms"] / 1e3,
                          "failed": st["failed_docs"], **info}), flush=True)
    del e
