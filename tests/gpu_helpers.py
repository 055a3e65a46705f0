"""Shared parity helpers for the GPU tests (compare the HIP engine with the CPU oracle)."""
import ctypes
import json
import os

import numpy as np

from oracle import OracleDoc, replay_batch

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i] != b[i]:
            return i, a[max(0, i - 120): i + 120], b[max(0, i - 120): i + 120]
    return n, a[n - 60:], b[n - 60:]


def compare_doc(engine, batch, d, observer="__observer__"):
    """Full comparison of one document: status, text, segment table, SnapshotV1 ITree."""
    o = OracleDoc(observer)
    o.apply_batch(ctypes.addressof(batch), d)
    ocode, oerr, oseq = o.status()
    gcode, gseq = engine.status(d)
    assert gcode == ocode, f"doc {d}: status gpu={gcode}@{gseq} oracle={ocode}@{oseq} ({oerr})"
    if ocode:
        assert gseq == oseq, f"doc {d}: failing seq gpu={gseq} oracle={oseq}"
        return
    gs, os_ = engine.segments_json(d), o.segments_json()
    if gs != os_:
        dump(f"doc{d}_segments", gs, os_)
        i, ga, oa = first_diff(gs, os_)
        raise AssertionError(f"doc {d}: segment tables differ at {i}\n gpu: {ga}\n orc: {oa}")
    # (the oracle's Python text is UTF-8: a lone surrogate -- a remove can split a pair -- arrives as
    # U+FFFD; the engine's keeps the UTF-16 units, so it is compared in the same form)
    gtext = engine.text(d).encode("utf-16-le", "surrogatepass").decode("utf-16-le", "replace")
    assert gtext == o.text(), f"doc {d}: text differs"
    gsnap, osnap = engine.snapshot_json(d), o.snapshot_json()
    if gsnap != osnap:
        dump(f"doc{d}_snapshot", gsnap, osnap)
        i, ga, oa = first_diff(gsnap, osnap)
        raise AssertionError(f"doc {d}: snapshot differs at {i}\n gpu: {ga}\n orc: {oa}")


def dump(name, gpu, orc):
    try:
        os.makedirs(OUT, exist_ok=True)
        with open(os.path.join(OUT, name + ".gpu.json"), "w") as f:
            f.write(gpu)
        with open(os.path.join(OUT, name + ".oracle.json"), "w") as f:
            f.write(orc)
    except OSError:
        pass


def compare_batch_checksums(engine, batch, threads=16):
    """Checksum (text + SnapshotV1 blobs) and status for every doc; returns mismatching doc ids."""
    n = batch.n_docs
    s = engine.summaries()
    ops, cks, st = replay_batch(ctypes.addressof(batch), 0, n, threads=threads)
    bad = [d for d in range(n) if int(s["status"][d]) != st[d] or (st[d] == 0 and int(s["checksum"][d]) != cks[d])]
    return bad, ops, s
