"""Generate a synthetic batch and replay it once (target for rocprofv3 counter passes).
Usage: python tools/replay_once.py [--kind 2 --docs 2048 --ops 10000]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", type=int, default=2)
ap.add_argument("--docs", type=int, default=2048)
ap.add_argument("--ops", type=int, default=10000)
ap.add_argument("--replays", type=int, default=1)
a = ap.parse_args()
e = mte.Engine(0)
e.generate(a.kind, a.docs, a.ops, n_clients=8, seed=3)
for _ in range(a.replays):
    st = e.replay()
print(json.dumps({**st, **e.run_info()}))
