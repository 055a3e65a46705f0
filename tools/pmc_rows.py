"""SQ counters of k_rows (tools/pmc_rows.sh): per op of the C2 batch and per wave-cycle.
Usage: python tools/pmc_rows.py [gpurun_out/pmc_rows] -> profiles/r04/pmc_rows_c2.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(d=os.path.join(ROOT, "gpurun_out", "pmc_rows")):
    tot = defaultdict(float)
    launches = defaultdict(set)  # per pass: k_rows dispatches (each replays the whole batch)
    vgpr = None
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_rows" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                launches[f].add(r["Dispatch_Id"])
                vgpr = r.get("VGPR_Count")
    n = max((len(v) for v in launches.values()), default=1)
    ops = 4096 * 10_000 * n
    per_op = {k: round(v / ops, 2) for k, v in sorted(tot.items())}
    wc = tot.get("SQ_WAVE_CYCLES", 0.0)
    derived = {}
    if wc:
        derived = {"issue_fraction_per_wave": round(tot.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
                   "wait_fraction_per_wave": round(tot.get("SQ_WAIT_ANY", 0) / wc, 3),
                   "instructions_per_op": round(sum(tot.get(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM")) / ops, 1)}
    out = {"config": "C2 (4 096 docs x 10^4 ops), k_rows at 8 waves per CU (two per SIMD)", "source": "tools/pmc_rows.sh",
           "k_rows_launches_per_pass": n, "vgpr_count": vgpr, "raw": tot, "per_op": per_op, "derived": derived}
    json.dump(out, open(os.path.join(ROOT, "profiles", "r04", "pmc_rows_c2.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
