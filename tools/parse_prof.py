"""Summarise rocprofv3 CSV output (kernel stats + FETCH_SIZE/WRITE_SIZE passes) into profiles/."""
import csv
import glob
import json
import os
import sys

# the replay pass: solo workgroups, LDS workgroups and HBM-resident waves, launched together on three
# streams
KERNELS = ("k_solo<false", "k_lds<false", "k_hbmq<false", "k_emit_count", "k_emit_write")


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main(tag, config="C4"):
    sys.path.insert(0, os.getcwd())
    import bench
    from fluidframework_amd.shard import plan_shard

    c = bench.CONFIGS[config]
    ids, counts = plan_shard(config, 1, 0, c["docs"], c["ops"])
    docs, ops, kind = len(ids), int(counts.sum()), c["kind"]
    base = f"gpurun_out/prof_{tag}"
    stats = rows(f"{base}/trace/**/*kernel_stats.csv")
    trace = rows(f"{base}/trace/**/*kernel_trace.csv")
    summary = {"tag": tag, "config": config, "docs": docs, "ops": ops, "kind": kind, "kernels": {}}
    for r in stats:
        summary["kernels"][r["Name"]] = {k: r[k] for k in ("Calls", "TotalDurationNs", "AverageNs", "Percentage")}
    for k in KERNELS:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace if k in r["Kernel_Name"]]
        if durs:
            summary[f"{k}_avg_ms_trace"] = sum(durs) / len(durs) / 1e6
    # pass time: from the pass's first kernel start to its last kernel end; passes are told apart by
    # the dispatches of their first kernel (k_solo when the batch has critical-path documents)
    evts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in trace
                  if any(k in r["Kernel_Name"] for k in KERNELS))
    anchor = "k_solo<false" if any("k_solo<false" in e[2] for e in evts) else "k_lds<false"
    starts = [e[0] for e in evts if anchor in e[2]]
    passes = []
    for i, a in enumerate(starts):
        lo = a - 50_000_000  # the other streams' first kernels start within 50 ms of the anchor
        hi = starts[i + 1] - 50_000_000 if i + 1 < len(starts) else float("inf")
        win = [e for e in evts if lo <= e[0] < hi]
        passes.append(max(e[1] for e in win) - min(e[0] for e in win))
    if passes:
        summary["replay_pass_avg_ms_trace"] = sum(passes) / len(passes) / 1e6
    for cname in ("FETCH_SIZE", "WRITE_SIZE"):
        pm = rows(f"{base}/pmc_{'fetch' if cname == 'FETCH_SIZE' else 'write'}/**/*counter_collection.csv")
        # per pass: every dispatch of the pass kernels / the number of passes (rocprofv3 serialises
        # dispatches while it collects counters, so k_lds then takes every document k_solo does not;
        # the emission kernels run twice per pass)
        n_pass = len({r["Dispatch_Id"] for r in pm if anchor in r["Kernel_Name"] and r["Counter_Name"] == cname})
        tot = 0.0
        for k in KERNELS:
            vals = [float(r["Counter_Value"]) for r in pm if k in r["Kernel_Name"] and r["Counter_Name"] == cname]
            if vals and n_pass:
                summary[f"{cname}_kib_{k}"] = sum(vals) / n_pass
                tot += sum(vals) / n_pass
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
    # (profiles/pmc_replay_<config>.json, the bench's calibrated traffic, is tools/pmc_replay.py's)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02", sys.argv[2] if len(sys.argv) > 2 else "C4")
