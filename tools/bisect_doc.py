"""Find the first op at which the GPU replay of one document diverges from the oracle: replay
prefixes of the document's log (a one-document view of the exported batch) and bisect on the
checksum. Usage (GPU box): python tools/bisect_doc.py --kind 2 --docs 64 --ops 50000 --doc 7"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import mte  # noqa: E402
from oracle import OracleDoc, replay_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", type=int, default=2)
ap.add_argument("--docs", type=int, default=64)
ap.add_argument("--ops", type=int, default=50000)
ap.add_argument("--seed", type=int, default=1000)
ap.add_argument("--doc", type=int, default=7)
ap.add_argument("--force-hbm", type=int, default=0)
a = ap.parse_args()

gen = mte.Engine(0)
gen.generate(a.kind, a.docs, a.ops, n_clients=8, seed=a.seed)
full = gen.export_batch()
d = a.doc
ob, oe = full.doc_op_offsets[d], full.doc_op_offsets[d + 1]
keep = []


def prefix(n):
    """One-document batch: document d's first n ops (same op/payload/client arrays)."""
    b = mte.mte_batch()
    ctypes.pointer(b)[0] = full
    b.n_docs = 1
    opo = (ctypes.c_uint64 * 2)(ob, ob + n)
    pyo = (ctypes.c_uint64 * 2)(full.doc_payload_offsets[d], full.doc_payload_offsets[d + 1])
    cli = (ctypes.c_uint32 * 2)(full.doc_client_offsets[d], full.doc_client_offsets[d + 1])
    keep.extend([opo, pyo, cli])
    b.doc_op_offsets = ctypes.cast(opo, ctypes.POINTER(ctypes.c_uint64))
    b.doc_payload_offsets = ctypes.cast(pyo, ctypes.POINTER(ctypes.c_uint64))
    b.doc_client_offsets = ctypes.cast(cli, ctypes.POINTER(ctypes.c_uint32))
    return b


eng = mte.Engine(0)
eng.set_option("force_hbm", a.force_hbm)


def same(n):
    b = prefix(n)
    eng.load(b)
    eng.replay()
    s = eng.summaries()
    _, cks, sts = replay_batch(ctypes.addressof(b), 0, 1, threads=1)
    return int(s["status"][0]) == sts[0] and (sts[0] != 0 or int(s["checksum"][0]) == cks[0]), b


lo, hi = 0, int(oe - ob)  # same(lo) holds, same(hi) fails
ok, _ = same(hi)
print("full doc matches:", ok, flush=True)
if not ok:
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if same(mid)[0]:
            lo = mid
        else:
            hi = mid
    print("first diverging prefix:", hi, "(op index", hi - 1, ")", flush=True)
    ops = mte.batch_ops(full)[ob:oe]
    for i in range(max(0, hi - 4), hi):
        print("op", i, ops[i], flush=True)
    _, b = same(hi)
    print(eng.doc_result(0), flush=True)
    o = OracleDoc("__observer__")
    o.apply_batch(ctypes.addressof(b), 0)
    gs, rs = json.loads(eng.segments_json(0)), json.loads(o.segments_json())
    gl = gs if isinstance(gs, list) else gs.get("segments", gs)
    rl = rs if isinstance(rs, list) else rs.get("segments", rs)
    for i, (x, y) in enumerate(zip(gl, rl)):
        if x != y:
            print("segment", i, "\n gpu", x, "\n orc", y)
            for j in range(max(0, i - 3), min(len(gl), i + 4)):
                print("  gpu", j, gl[j])
            for j in range(max(0, i - 3), min(len(rl), i + 4)):
                print("  orc", j, rl[j])
            break
