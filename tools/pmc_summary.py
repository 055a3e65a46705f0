"""Summarise tools/pmc_passes.sh output for one kernel: counters per wave and per applied op."""
import csv
import glob
import json
import sys
from collections import defaultdict

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kernel = sys.argv[2] if len(sys.argv) > 2 else "k_lds<false>"
ops = float(sys.argv[3]) if len(sys.argv) > 3 else 0
tot = defaultdict(float)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if kernel in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
res = {k: v for k, v in sorted(tot.items())}
if ops:
    res["per_op"] = {k: v / ops for k, v in sorted(tot.items())}
print(json.dumps(res, indent=1))
