"""Summarise rocprofv3 CSV output (kernel stats + FETCH_SIZE/WRITE_SIZE passes) into profiles/."""
import csv
import glob
import json
import os
import sys

# the replay pass: LDS workgroups and HBM-resident waves, launched together on two streams
KERNELS = ("k_lds<false>", "k_hbmq<false>")


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main(tag, docs=4096, ops=10000, kind=2):
    base = f"gpurun_out/prof_{tag}"
    stats = rows(f"{base}/trace/**/*kernel_stats.csv")
    trace = rows(f"{base}/trace/**/*kernel_trace.csv")
    summary = {"tag": tag, "docs": docs, "ops": ops, "kind": kind, "kernels": {}}
    for r in stats:
        summary["kernels"][r["Name"]] = {k: r[k] for k in ("Calls", "TotalDurationNs", "AverageNs", "Percentage")}
    for k in KERNELS:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace if k in r["Kernel_Name"]]
        if durs:
            summary[f"{k}_avg_ms_trace"] = sum(durs) / len(durs) / 1e6
    # pass time: first start to last end of each (k_lds, k_hbmq) pair, in dispatch order
    lds = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in trace if KERNELS[0] in r["Kernel_Name"])
    hbq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in trace if KERNELS[1] in r["Kernel_Name"])
    if lds and len(lds) == len(hbq):
        passes = [max(a[1], b[1]) - min(a[0], b[0]) for a, b in zip(lds, hbq)]
        summary["replay_pass_avg_ms_trace"] = sum(passes) / len(passes) / 1e6
    for cname in ("FETCH_SIZE", "WRITE_SIZE"):
        pm = rows(f"{base}/pmc_{'fetch' if cname == 'FETCH_SIZE' else 'write'}/**/*counter_collection.csv")
        # per pass: the counters of one k_lds dispatch plus one k_hbmq dispatch (rocprofv3 serialises
        # dispatches while it collects counters)
        tot = 0.0
        for k in KERNELS:
            vals = [float(r["Counter_Value"]) for r in pm if k in r["Kernel_Name"] and r["Counter_Name"] == cname]
            if vals:
                summary[f"{cname}_kib_{k}"] = sum(vals) / len(vals)
                tot += sum(vals) / len(vals)
        if tot:
            summary[cname + "_kib_per_launch"] = tot
    if "FETCH_SIZE_kib_per_launch" in summary and "WRITE_SIZE_kib_per_launch" in summary:
        summary["hbm_bytes_per_launch"] = (summary["FETCH_SIZE_kib_per_launch"] + summary["WRITE_SIZE_kib_per_launch"]) * 1024
    os.makedirs("profiles", exist_ok=True)
    with open(f"profiles/{tag}_summary.json", "w") as f:
        json.dump(summary, f, indent=1)
    for p in glob.glob(f"{base}/trace/**/*kernel_stats.csv", recursive=True):
        with open(p) as f, open(f"profiles/{tag}_kernel_stats.csv", "w") as g:
            g.write(f.read())
    if "hbm_bytes_per_launch" in summary:
        with open("profiles/pmc_replay.json", "w") as f:
            json.dump({"docs": docs, "ops": ops, "kind": kind, "source": f"profiles/{tag}_summary.json",
                       "hbm_bytes_per_launch": summary["hbm_bytes_per_launch"],
                       "note": "raw (FETCH_SIZE+WRITE_SIZE)*1024; gfx950 FETCH_SIZE calibration (x2) applies only to "
                               "wide coalesced streams and is NOT applied to this narrow-access kernel"}, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
