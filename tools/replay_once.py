"""Generate a synthetic batch and replay it once (target for rocprofv3 counter / trace passes).
Usage: python tools/replay_once.py [--config C4] | [--kind 2 --docs 2048 --ops 10000]
--config takes bench.py's workload (plan_shard, global ids, generator seed) at N=1."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default=None)
ap.add_argument("--kind", type=int, default=2)
ap.add_argument("--docs", type=int, default=2048)
ap.add_argument("--ops", type=int, default=10000)
ap.add_argument("--replays", type=int, default=1)
ap.add_argument("--opt", action="append", default=[], help="engine option key=value (repeatable)")
a = ap.parse_args()
e = mte.Engine(0)
for kv in a.opt:
    k, v = kv.split("=")
    e.set_option(k, int(v))
if a.config:
    import bench
    from fluidframework_amd.shard import plan_shard

    c = bench.CONFIGS[a.config]
    ids, counts = plan_shard(a.config, 1, 0, c["docs"], c["ops"])
    e.generate(c["kind"], len(ids), c["ops"], n_clients=8, seed=bench.GEN_SEED, ops_per_doc=counts, doc_ids=ids)
    meta = {"config": a.config, "docs": len(ids), "ops": int(counts.sum()), "kind": c["kind"]}
else:
    e.generate(a.kind, a.docs, a.ops, n_clients=8, seed=3)
    meta = {"docs": a.docs, "ops": a.docs * a.ops, "kind": a.kind}
times = []
for _ in range(a.replays):
    st = e.replay()
    times.append(round(st["kernel_ms"], 2))
meta["kernel_ms_all"] = times
print(json.dumps({**meta, **st, **e.run_info()}))
