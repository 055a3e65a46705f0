"""Critical-path probe: replay ONE long document alone (a lone wave) and report its per-op latency,
its residency mode and peak state sizes; with MTE_LIB=prof also the per-phase cycles per op.

Usage (GPU box): python tools/lone_doc.py --ops 200000 [--kind 2] [--docs 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", type=int, default=2)
    ap.add_argument("--docs", type=int, default=1)
    ap.add_argument("--ops", type=int, default=200000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--force-hbm", type=int, default=0)
    ap.add_argument("--verify", type=int, default=1)
    ap.add_argument("--opt", action="append", default=[], help="engine option key=value (repeatable)")
    a = ap.parse_args()
    e = mte.Engine(0)
    t0 = time.time()
    e.generate(a.kind, a.docs, a.ops, n_clients=8, seed=1000)
    gen_s = time.time() - t0
    if a.force_hbm:
        e.set_option("force_hbm", 1)
    for kv in a.opt:
        k, v = kv.split("=")
        e.set_option(k, int(v))
    res = {"kind": a.kind, "docs": a.docs, "ops": a.ops, "gen_s": round(gen_s, 2), "lib": os.environ.get("MTE_LIB", "")}
    for r in range(a.reps):
        st = e.replay()
        res[f"kernel_ms_{r}"] = st["kernel_ms"]
    res["us_per_op"] = res[f"kernel_ms_{a.reps - 1}"] * 1e3 / a.ops
    try:  # the critical wave's clock stamps (libraries from before them lack the keys)
        cyc, ref = e.get_info("solo_cycles"), e.get_info("solo_ref_ticks")
        res["solo_cycles_per_op"] = cyc / a.ops
        res["solo_clock_ghz"] = cyc / (ref / 100e6) / 1e9 if ref else None
    except mte.MteError:
        pass
    res["run_info"] = e.run_info()
    res["doc0"] = e.doc_result(0)
    if os.environ.get("MTE_LIB", "").startswith(("prof", "po_", "rp_")):
        prof = e.profile().astype(np.float64)
        ops = prof[:, mte.PROF_NAMES.index("ops")].sum()
        res["cycles_per_op"] = {n: round(float(prof[:, i].sum() / max(ops, 1)), 2)
                                for i, n in enumerate(mte.PROF_NAMES) if n != "ops"}
    if a.verify:
        import ctypes

        from oracle import replay_batch
        batch = e.export_batch()
        t1 = time.time()
        o_ops, cks, sts = replay_batch(ctypes.addressof(batch), 0, a.docs, threads=min(16, a.docs))
        res["oracle_s"] = round(time.time() - t1, 2)
        res["oracle_us_per_op_thread"] = (time.time() - t1) * 1e6 / max(o_ops, 1) * min(16, a.docs)
        s = e.summaries()
        res["verified"] = all(int(s["checksum"][d]) == cks[d] for d in range(a.docs))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
