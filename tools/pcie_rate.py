"""PCIe-inclusive replay rate (GPU box): the drop-in boundary hands the engine HOST buffers (mte_load of
an mte_batch built by the builder), so a caller's end-to-end rate includes the host-to-device upload.
The bench's `value` starts with the inputs resident in HBM; this tool times the other case on the same
workload: the config's batch is generated on one engine, exported to host memory, then a second
engine times mte_load (upload + per-document setup) and one replay.

Usage (GPU box): python tools/pcie_rate.py --config C4 [--reps 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fluidframework_amd import mte  # noqa: E402
from fluidframework_amd.shard import plan_shard  # noqa: E402


def clone_batch(b):
    """A deep copy of an mte_batch view (the generator engine's host batch), so that engine -- and its
    device memory -- can be released before the timed engine loads the copy."""
    import ctypes

    import numpy as np

    keep = []

    def cp(ptr, nbytes):
        buf = np.empty(max(1, int(nbytes)), np.uint8)
        if ptr and nbytes:
            ctypes.memmove(buf.ctypes.data, ptr, int(nbytes))
        keep.append(buf)
        return buf.ctypes.data

    def u64s(ptr, n):
        return np.ctypeslib.as_array(ptr, (n,)).copy() if ptr else None

    n = b.n_docs
    out = mte.mte_batch()
    out.n_docs = n
    op_off = u64s(b.doc_op_offsets, n + 1)
    pay_off = u64s(b.doc_payload_offsets, n + 1)
    P64 = ctypes.POINTER(ctypes.c_uint64)
    P32 = ctypes.POINTER(ctypes.c_uint32)
    out.doc_op_offsets = ctypes.cast(cp(ctypes.addressof(b.doc_op_offsets.contents), 8 * (n + 1)), P64)
    out.ops = cp(b.ops, 32 * int(op_off[n]))
    out.doc_payload_offsets = ctypes.cast(cp(ctypes.addressof(b.doc_payload_offsets.contents), 8 * (n + 1)), P64)
    out.payload = ctypes.cast(cp(ctypes.cast(b.payload, ctypes.c_void_p).value, 2 * int(pay_off[n])),
                              ctypes.POINTER(ctypes.c_uint16))
    out.n_propsets = b.n_propsets
    ps = np.frombuffer(ctypes.string_at(b.propsets, 8 * b.n_propsets), np.uint32).reshape(-1, 2) \
        if b.n_propsets else np.zeros((0, 2), np.uint32)
    nkv = int((ps[:, 0] + ps[:, 1]).max()) if len(ps) else 0
    out.propsets = cp(b.propsets, 8 * b.n_propsets)
    addr = lambda p: ctypes.cast(p, ctypes.c_void_p).value  # noqa: E731
    out.prop_keys = ctypes.cast(cp(addr(b.prop_keys), 4 * nkv), P32)
    out.prop_vals = ctypes.cast(cp(addr(b.prop_vals), 4 * nkv), P32)
    out.n_keys = b.n_keys
    ko = u64s(b.key_offsets, b.n_keys + 1)
    out.key_offsets = ctypes.cast(cp(addr(b.key_offsets), 8 * (b.n_keys + 1)), P64)
    out.key_text = cp(b.key_text, int(ko[-1]))
    out.n_vals = b.n_vals
    vo = u64s(b.val_offsets, b.n_vals + 1)
    out.val_offsets = ctypes.cast(cp(addr(b.val_offsets), 8 * (b.n_vals + 1)), P64)
    out.val_text = cp(b.val_text, int(vo[-1]))
    dco = np.ctypeslib.as_array(b.doc_client_offsets, (n + 1,)).copy()
    nn = int(dco[n])
    out.doc_client_offsets = ctypes.cast(cp(addr(b.doc_client_offsets), 4 * (n + 1)), P32)
    cno = u64s(b.client_name_offsets, nn + 1)
    out.client_name_offsets = ctypes.cast(cp(addr(b.client_name_offsets), 8 * (nn + 1)), P64)
    out.client_names = cp(b.client_names, int(cno[-1]))
    if b.doc_msg_offsets and b.msg_first_op and b.msg_text_offsets and b.msg_text:
        mo = u64s(b.doc_msg_offsets, n + 1)
        nm = int(mo[n])
        mto = u64s(b.msg_text_offsets, nm + 1)
        out.doc_msg_offsets = ctypes.cast(cp(addr(b.doc_msg_offsets), 8 * (n + 1)), P64)
        out.msg_first_op = ctypes.cast(cp(addr(b.msg_first_op), 8 * nm), P64)
        out.msg_text_offsets = ctypes.cast(cp(addr(b.msg_text_offsets), 8 * (nm + 1)), P64)
        out.msg_text = cp(b.msg_text, int(mto[-1]))
    out._keep = keep
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    args = bench.parse(["--config", a.config])
    gen = mte.Engine(0)
    ids, counts = plan_shard(args.config, 1, 0, args.docs, args.ops)
    gen.generate(args.kind, len(ids), args.ops, n_clients=args.clients, seed=bench.GEN_SEED, ops_per_doc=counts,
                 doc_ids=ids)
    batch = clone_batch(gen.export_batch())
    gen.close()  # one engine on the device at a time (C4's worst-case buffers are large)
    ops = int(len(mte.batch_ops(batch)))
    host_bytes = ops * 32 + int(batch.doc_payload_offsets[batch.n_docs]) * 2  # op records + UTF-16 payload
    res = {"config": a.config, "ops": ops, "host_batch_bytes": host_bytes, "reps": []}
    eng = mte.Engine(0)
    try:
        for _ in range(a.reps):
            t0 = time.perf_counter()
            eng.load(batch)
            t1 = time.perf_counter()
            st = eng.replay()
            t2 = time.perf_counter()
            assert st["failed_docs"] == 0, st
            res["reps"].append({"load_ms": round((t1 - t0) * 1e3, 1), "replay_wall_ms": round((t2 - t1) * 1e3, 1),
                                "kernel_ms": round(st["kernel_ms"], 1), "h2d_ms": round(st["h2d_ms"], 1),
                                "alloc_ms": round(eng.get_info("load_alloc_us") / 1000.0, 1),
                                "stage_copy_ms": round(eng.get_info("load_stage_copy_us") / 1000.0, 1),
                                "stage_wait_ms": round(eng.get_info("load_stage_wait_us") / 1000.0, 1),
                                "ops_per_s_pcie_inclusive": ops / (t2 - t0),
                                "upload_GBps": host_bytes / (t1 - t0) / 1e9})
    finally:
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
