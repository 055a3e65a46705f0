"""Per-phase cycle breakdown of the replay engine (MTE_LIB=prof build, engine.hpp MTE_PROFILE).

Usage (GPU box): MTE_LIB=prof python tools/phase_profile.py [--kind 2 --docs 4096 --ops 10000]
Prints cycles per applied op for every phase (inclusive; nested phases overlap), separately for the
documents that stayed LDS-resident and those replayed by HBM-resident waves. s_memtime reads perturb timing (~10 %)."""
import argparse
import json
import os
import sys

import numpy as np

os.environ.setdefault("MTE_LIB", "prof")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", type=int, default=2)
    ap.add_argument("--docs", type=int, default=4096)
    ap.add_argument("--ops", type=int, default=10000)
    ap.add_argument("--out", default="gpurun_out/phase_profile.json")
    ap.add_argument("--hw", type=int, default=8, help="hbm_waves_per_cu")
    a = ap.parse_args()
    e = mte.Engine(0)
    e.generate(a.kind, a.docs, a.ops, n_clients=8, seed=3)
    e.set_option("hbm_waves_per_cu", a.hw)
    st = e.replay()
    info = e.run_info()
    prof = e.profile().astype(np.float64)
    modes = np.array([e.doc_result(d)["mode"] for d in range(a.docs)])
    res = {"kind": a.kind, "docs": a.docs, "ops": a.ops, "kernel_ms": st["kernel_ms"], **info}
    for mode, name in ((0, "lds"), (1, "hbm")):
        sel = prof[modes == mode]
        ops = sel[:, mte.PROF_NAMES.index("ops")].sum()
        res[name + "_docs"] = int((modes == mode).sum())
        res["cycles_per_op_" + name] = {n: round(float(sel[:, i].sum() / max(ops, 1)), 2)
                                        for i, n in enumerate(mte.PROF_NAMES) if n != "ops"}
    print(json.dumps(res, indent=1))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
