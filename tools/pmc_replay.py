"""Per-pass HBM traffic of the replay for bench.py's roofline (`traffic`), from tools/profile.sh's
FETCH_SIZE and WRITE_SIZE passes, corrected with the gfx950 calibration of profiles/fetch_calib_r04.json
(FETCH_SIZE x 2 for the engine's coalesced dword / 16-B reads, WRITE_SIZE x 1).

rocprofv3 serialises dispatches while it collects counters, so in these passes k_lds takes every
non-solo document and k_hbmq finds the queue drained: the per-kernel split is that of the serialised
pass, the total is the pass's. Usage: python tools/pmc_replay.py <tag> [config] -> profiles/pmc_replay_<config>.json (C2 / C3 / C5 run
their bulk on k_rows: its launches count the passes there)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = ("k_solo<false", "k_lds<false", "k_hbmq<false", "k_rows<", "k_emit_count", "k_emit_write")


def main(tag, config="C4"):
    sys.path.insert(0, ROOT)
    import bench
    from fluidframework_amd.shard import plan_shard

    cal = json.load(open(os.path.join(ROOT, "profiles", "fetch_calib_r04.json")))
    c = bench.CONFIGS[config]
    ids, counts = plan_shard(config, 1, 0, c["docs"], c["ops"])
    per = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for ctr, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        for f in glob.glob(f"{ROOT}/gpurun_out/prof_{tag}/{sub}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = next((x for x in REPLAY if x in r["Kernel_Name"]), None)
                if k and r["Counter_Name"] == ctr:
                    per[k][ctr] += float(r["Counter_Value"]) * 1024.0
                    calls[k][ctr] += 1
    # replay passes: the bulk kernel's launches (k_lds, or k_rows for the row-engine configs)
    steps = max(list(calls["k_lds<false"].values()) + list(calls["k_rows<"].values()) or [1])
    kernels = {}
    total = 0.0
    for k, v in per.items():
        fb, wb = v.get("FETCH_SIZE", 0.0) / steps, v.get("WRITE_SIZE", 0.0) / steps
        corr = fb * cal["fetch_factor"] + wb * cal["write_factor"]
        kernels[k] = {"fetch_raw": fb, "write_raw": wb, "hbm_bytes_corrected": corr}
        total += corr
    out = {"docs": len(ids), "ops": int(counts.sum()), "kind": c["kind"], "tag": tag, "passes": steps,
           "hbm_bytes_per_launch": total, "kernels": kernels,
           "correction": "FETCH_SIZE x %.1f, WRITE_SIZE x %.1f (profiles/fetch_calib_r04.json)" % (cal["fetch_factor"], cal["write_factor"]),
           "note": "rocprofv3 serialises dispatches while collecting: per-kernel split of the serialised pass"}
    path = os.path.join(ROOT, "profiles", f"pmc_replay_{config}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
