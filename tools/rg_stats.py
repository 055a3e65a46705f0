"""What the critical document's ops do, from the CPU build of the row engine with event statistics
(tests/native MTE_CPU_STATS): per op, resolves and the rows they scan, heap pops and the heap size at
a pop, scour outcomes, packs, block splits and slots moved. Sizes the device code paths (which path a
pop takes, how many rows a resolve sees). Usage: python tools/rg_stats.py [ops] [gid]"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import regcpu  # noqa: E402

NAMES = ["ops", "resolve", "res_rows", "res_nrows", "pop", "pop_big", "pop_heap", "find_rows", "scour", "scour_nop",
         "scour_serial", "scour_copy", "pack", "split_blk", "move_slots", "split_at", "zam_calls", "zam_pops", "lru_push",
         "range_rows"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    gid = int(sys.argv[2]) if len(sys.argv) > 2 else 111877
    nat = os.path.join(ROOT, "tests", "native")
    subprocess.run(["make", "-s", "-C", nat, "stats"], check=True)
    L = ctypes.CDLL(os.path.join(nat, "_build", "libregcpu_stats.so"))
    regcpu._lib = None
    base = regcpu.lib()
    # the stats build exports the same entry points: route regcpu.replay through it
    L.regcpu_replay.restype = ctypes.c_uint64
    L.regcpu_replay.argtypes = base.regcpu_replay.argtypes
    L.regcpu_docres_size.restype = ctypes.c_uint32
    L.regcpu_heap.restype = ctypes.c_uint32
    L.regcpu_stats.restype = ctypes.c_uint32
    regcpu._lib = L
    ops, pay = regcpu.generated(2, gid, n, n_clients=8, seed=1000)
    at, res, rows, text = regcpu.replay(ops, pay)
    out = (ctypes.c_uint64 * 64)()
    L.regcpu_stats(out, len(NAMES) + 2)
    st = {k: int(out[i]) for i, k in enumerate(NAMES)}
    o = max(st["ops"], 1)
    per = {k: round(v / o, 4) for k, v in st.items() if k != "ops"}
    heap_max, lb_max = int(out[len(NAMES)]), int(out[len(NAMES) + 1])
    derived = {
        "rows_per_resolve": round(st["res_rows"] / max(st["resolve"], 1), 3),
        "nrows_at_resolve": round(st["res_nrows"] / max(st["resolve"], 1), 3),
        "heap_at_pop": round(st["pop_heap"] / max(st["pop"], 1), 1),
        "pops_on_serial_sift": round(st["pop_big"] / max(st["pop"], 1), 4),
        "slots_moved_per_split": round(st["move_slots"] / max(st["split_blk"] + st["pack"], 1), 1),
        "heap_max_at_pop": heap_max,
        "n_lb_max_at_pop": lb_max,
    }
    print(json.dumps({"doc": f"kind 2 gid {gid}, first {n} ops (CPU build of reg_engine.hpp)", "stop": int(at),
                      "max_lb": int(res["max_lb"]), "n_lb": int(res["n_lb"]), "height": int(res["height"]),
                      "heap_size_end": int(res["heap_size"]), "per_op": per, "derived": derived}, indent=1))


if __name__ == "__main__":
    main()
