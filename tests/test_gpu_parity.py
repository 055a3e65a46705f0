"""GPU parity: the HIP replay engine (through the C ABI) against the CPU oracle and the reference's
golden vectors. Integer/byte work: every comparison is bit-exact."""
import json
import os

import numpy as np
import pytest

from fluidframework_amd import mte
from tests.gpu_helpers import compare_batch_checksums, compare_doc
from tests.oplog import TestString, ann, ins, msg, rem
from tests.test_builder_cpu import random_log
from tests.test_oracle_fixtures import GOLDEN, fixture_blobs
from tests.test_oracle_specs import SNAPSHOT_CASES, hello_world_log

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    # this file tests the LDS / HBM-resident engine (engine.hpp) and its routing: lean batches without
    # solo documents would otherwise take k_rows (tests/test_gpu_reg.py covers that route)
    e = mte.Engine(0)
    e.set_option("rows_bulk", 0)
    yield e
    e.close()


def test_wave_primitives(engine):
    rng = np.random.default_rng(1)
    vals = rng.integers(0, 1 << 20, size=64 * 8, dtype=np.uint32)
    out = engine.wave_selftest(vals)
    for w in range(8):
        v = vals[w * 64:(w + 1) * 64]
        assert np.array_equal(out[w, 0], np.cumsum(v, dtype=np.uint64).astype(np.uint32))
        assert np.array_equal(out[w, 1], v[::-1])
        bits = (v & 1).astype(np.uint64)
        mask = int(sum(int(b) << i for i, b in enumerate(bits)))
        assert int(out[w, 2][0]) == mask & 0xFFFFFFFF and int(out[w, 2][32]) == mask >> 32
        g = v.reshape(8, 8)
        assert np.array_equal(out[w, 3], np.cumsum(g, axis=1, dtype=np.uint64).astype(np.uint32).ravel())
        assert np.array_equal(out[w, 4], np.maximum.accumulate(g.astype(np.int64), axis=1).astype(np.uint32).ravel())


def spec_logs():
    logs = [hello_world_log()]
    m = hello_world_log()
    m += [msg("remote2", 12, 11, rem(0, 11)), msg("remote", 13, 11, ins(0, "text"))]
    logs.append(m)
    m = hello_world_log()
    m += [msg("remote", 12, 11, ins(0, "text")), msg("remote2", 13, 11, rem(0, 11))]
    logs.append(m)
    for case in sorted(SNAPSHOT_CASES):
        steps, _ = SNAPSHOT_CASES[case]
        s = TestString()
        for st in steps:
            if st[0] == "append":
                s.append(st[1], st[2])
            elif st[0] == "insert":
                s.insert(st[1], st[2], st[3])
            else:
                s.remove_range(st[1], st[2], st[3])
        logs.append(s.msgs)
    for inc in (True, False):
        s = TestString()
        for i in range(10010):
            s.append(str(i % 10), inc)
        logs.append(s.msgs)
    logs.append([msg("a", 1, 0, ins(0, "xy")), msg("b", 2, 1, ins(1, "B")), msg("c", 3, 1, ins(1, "C"))])
    logs.append([msg("a", 1, 0, ins(0, "hello")), msg("b", 2, 1, rem(1, 3)), msg("c", 3, 1, rem(0, 4))])
    logs.append([msg("w", 1, 0, ins(0, "abc")), msg("w", 2, 1, ann(0, 3, {"b": 1, "a": 2, "7": "x"})),
                 msg("w", 3, 2, ann(0, 3, {"b": None})), msg("w", 4, 3, ann(0, 3, {"b": 3, "2": True}))])
    logs.append([msg("w", 1, 0, ins(0, "ab")), msg("w", 2, 1, ins(5, "x"))])  # insert failed
    return logs


def test_spec_logs_match_oracle(engine):
    logs = spec_logs()
    b = mte.Builder()
    for m in logs:
        b.add_doc(m)
    batch = b.batch()
    engine.load(batch)
    engine.replay()
    for d in range(len(logs)):
        compare_doc(engine, batch, d)
    assert engine.text(1) == "text" and engine.text(2) == "text"
    assert engine.status(len(logs) - 1)[0] == 1  # MergeTree insert failed


def local_fixture_log(name):
    """generateSharedStrings.ts:24-98 as local (non-collaborative) ops; lengths tracked here."""
    ops = []
    length = 0

    def add(c):
        ops.append(msg("local", 0, 0, c))

    n = {"headerOnly": 1250, "headerAndBody": 5000, "withMarkers": 5000, "withAnnotations": 5000}.get(name)
    if name == "largeBody":
        for i in range(10000):
            t = f"text-{i}"
            add(ins(0, t))
            length += len(t)
    else:
        for i in range(n):
            t = f"text{i}"
            add(ins(0, t))
            length += len(t)
    if name == "withMarkers":
        i = 0
        while i < length:
            add(ins(i, {"marker": {"refType": 1}, "props": {"ItemType": "Paragraph", "Properties": {"Bold": False},
                                                            "markerId": f"marker{i}", "referenceTileLabels": ["Eop"]}}))
            length += 1
            i += 70
    if name == "withAnnotations":
        i = 0
        while i < length:
            add(ann(i, i + 10, {"bold": True}))
            i += 70
    return ops


def test_v1_golden_fixtures_on_gpu(engine):
    names = ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"]
    b = mte.Builder()
    for nm in names:
        b.add_doc(local_fixture_log(nm), observer="")
    engine.load(b.batch())
    engine.replay()
    for d, nm in enumerate(names):
        assert engine.status(d)[0] == 0
        tree = json.loads(engine.snapshot_json(d))
        got = [(e["path"], e["value"]["contents"]) for e in tree["entries"]]
        assert got == fixture_blobs(nm), nm


def test_random_logs_match_oracle(engine):
    logs = [random_log(s, n=400) for s in range(24)]
    b = mte.Builder()
    for m in logs:
        b.add_doc(m)
    batch = b.batch()
    engine.load(batch)
    engine.replay()
    for d in range(len(logs)):
        compare_doc(engine, batch, d)


@pytest.mark.parametrize("kind,docs,ops", [(2, 96, 3000), (3, 96, 3000), (5, 32, 6000)])
def test_generated_workloads_match_oracle(engine, kind, docs, ops):
    engine.generate(kind, docs, ops, n_clients=8, seed=7)
    gen_fail = [d for d in range(docs) if engine.status(d)[0]]
    assert not gen_fail, f"generator hit errors: {[(d, engine.status(d)) for d in gen_fail[:5]]}"
    batch = engine.export_batch()
    engine.replay()  # a fresh replay of the recorded log
    bad, _, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])  # raises with a precise diff
    assert not bad


def test_c1_conflict_farm_on_gpu(engine):
    from tests.workloads import c1_farm_log

    logs = [c1_farm_log(seed=s) for s in range(4)]
    b = mte.Builder()
    for m in logs:
        b.add_doc(m, observer="0")
    batch = b.batch()
    engine.load(batch)
    engine.replay()
    for d in range(len(logs)):
        compare_doc(engine, batch, d, observer="0")


def _summary_key(s):
    return [(int(x["checksum"]), int(x["status"]), int(x["segments"])) for x in s]


def test_hbm_resident_pass_matches_lds_pass(engine):
    """The HBM-resident engine (second pass for documents that outgrow LDS) is the same code over
    HBM; both passes must give bit-identical results, and both match the oracle."""
    engine.generate(3, 64, 2500, n_clients=8, seed=11)
    batch = engine.export_batch()
    engine.replay()
    lds = engine.summaries()
    info = engine.run_info()
    assert info["spilled"] == 0, (info, [engine.doc_result(d) for d in range(64) if engine.doc_result(d)["mode"] == 1][:3])
    engine.set_option("force_hbm", 1)
    try:
        engine.replay()
        hbm = engine.summaries()
    finally:
        engine.set_option("force_hbm", 0)
    assert _summary_key(lds) == _summary_key(hbm)
    bad, _, _ = compare_batch_checksums(engine, batch)
    assert not bad


def test_lds_pool_exhaustion_spills_and_matches_oracle(engine):
    """A tiny LDS block pool forces documents out of the LDS plan mid-replay: between ops they move
    to HBM and continue in the same wave, mid-op failures are re-run by the host; every document
    still matches the oracle."""
    engine.generate(2, 128, 3000, n_clients=8, seed=5)
    batch = engine.export_batch()
    engine.set_option("pool_limit", 48)
    try:
        engine.replay()
        info = engine.run_info()
    finally:
        engine.set_option("pool_limit", 0)
    assert info["spilled"] + info["continued"] > 0, info
    bad, _, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad


def test_many_clients_overlap_masks_match_oracle(engine):
    """48 writers: overlapping removes by clients >= 32 take the HBM half of the overlap mask."""
    engine.generate(3, 48, 2500, n_clients=48, seed=21)
    batch = engine.export_batch()
    engine.replay()
    bad, _, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad
    for d in range(0, 48, 12):
        compare_doc(engine, batch, d)


def test_generator_continues_hbm_resident(engine):
    """Generation under a tiny LDS pool hands documents to HBM mid-log; the log recorded must be
    the same as the one generated entirely in LDS (the generator is deterministic)."""
    engine.generate(2, 64, 2000, n_clients=8, seed=4)
    ref = mte.batch_ops(engine.export_batch()).copy()
    engine.set_option("pool_limit", 40)
    try:
        engine.generate(2, 64, 2000, n_clients=8, seed=4)
        info = engine.run_info()
    finally:
        engine.set_option("pool_limit", 0)
    assert info["continued"] + info["spilled"] > 0, info
    got = mte.batch_ops(engine.export_batch())
    assert np.array_equal(ref, got)


def test_hybrid_pass_lds_and_hbm_waves_agree(engine):
    """The hybrid pass (LDS workgroup + HBM-resident waves sharing one queue) routes documents to
    both kinds of wave; results are identical to an LDS-only pass and to HBM waves waiting on a
    handful of slots, and match the oracle."""
    nd = 3072
    engine.generate(3, nd, 300, n_clients=8, seed=17)
    batch = engine.export_batch()
    engine.replay()
    info = engine.run_info()
    modes = np.array([engine.doc_result(d)["mode"] for d in range(nd)])
    assert info["hbm_waves"] > 0 and (modes == 1).sum() > 0 and (modes == 0).sum() > 0, info
    hybrid = _summary_key(engine.summaries())
    bad, _, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad
    try:
        engine.set_option("hbm_waves_per_cu", 0)
        engine.replay()
        assert engine.run_info()["hbm_waves"] == 0
        assert _summary_key(engine.summaries()) == hybrid
        engine.set_option("hbm_waves_per_cu", 8)
        slot = engine.get_info("slot_bytes")
        engine.set_option("slot_budget_mb", ((2048 + 24) * slot >> 20) + 1)  # ~24 HBM slots
        engine.replay()
        info = engine.run_info()
        assert 0 < info["hbm_waves"] < 64, info
        assert _summary_key(engine.summaries()) == hybrid
    finally:
        engine.set_option("hbm_waves_per_cu", 8)
        engine.set_option("slot_budget_mb", 48 << 10)


def test_slot_overflow_reruns_with_worst_case_capacity(engine):
    """HBM slots are sized for typical documents; one that outgrows its slot is marked for the
    host's re-run with worst-case capacities and still matches the oracle."""
    engine.set_option("slot_blk_limit", 24)
    try:
        engine.generate(2, 48, 3000, n_clients=8, seed=23)
        batch = engine.export_batch()
        engine.set_option("force_hbm", 1)
        engine.replay()
        info = engine.run_info()
    finally:
        engine.set_option("force_hbm", 0)
        engine.set_option("slot_blk_limit", 0)
    assert info["spilled"] > 0 and info["hbm_ms"] > 0, info
    bad, _, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad


def test_long_documents_match_oracle(engine):
    """50k-op documents: merge chains that append in place and then outgrow their chunk within one
    scour (the copy of the head must not read bytes the same batch has yet to write), arena GC,
    LDS-to-HBM continuation (a 40-block LDS pool per CU: the 255-entry heap keeps these documents in
    a full pool to the end)."""
    engine.generate(2, 16, 50000, n_clients=8, seed=1000)
    batch = engine.export_batch()
    engine.set_option("pool_limit", 40)
    try:
        engine.replay()
    finally:
        engine.set_option("pool_limit", 0)
    assert engine.run_info()["continued"] > 0
    bad, _, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad


def test_one_document_view_of_a_batch(engine):
    """mte_batch offsets are absolute: a batch whose only document starts mid-array (a prefix of
    document 5's log here) replays exactly that document."""
    import ctypes

    from oracle import replay_batch

    engine.generate(2, 8, 3000, n_clients=8, seed=31)
    full = engine.export_batch()
    d, n = 5, 2000
    ob = full.doc_op_offsets[d]
    b = mte.mte_batch()
    ctypes.pointer(b)[0] = full
    b.n_docs = 1
    opo = (ctypes.c_uint64 * 2)(ob, ob + n)
    pyo = (ctypes.c_uint64 * 2)(full.doc_payload_offsets[d], full.doc_payload_offsets[d + 1])
    cli = (ctypes.c_uint32 * 2)(full.doc_client_offsets[d], full.doc_client_offsets[d + 1])
    b.doc_op_offsets = ctypes.cast(opo, ctypes.POINTER(ctypes.c_uint64))
    b.doc_payload_offsets = ctypes.cast(pyo, ctypes.POINTER(ctypes.c_uint64))
    b.doc_client_offsets = ctypes.cast(cli, ctypes.POINTER(ctypes.c_uint32))
    e2 = mte.Engine(0)
    try:
        e2.load(b)
        st = e2.replay()
        assert st["ops"] == n
        _, cks, sts = replay_batch(ctypes.addressof(b), 0, 1, threads=1)
        s = e2.summaries()
        assert int(s["status"][0]) == sts[0] == 0 and int(s["checksum"][0]) == cks[0]
    finally:
        e2.close()


def test_reference_spec_pins_on_gpu(engine):
    """The restated reference spec cases (mergeTree.annotate.spec.ts, mergeTree.insertingWalk.spec.ts,
    properties.spec.ts; tests/test_oracle_specs.py) on the GPU: bit-exact vs the oracle and the
    reference tests' literal expectations."""
    from tests.test_oracle_specs import (ANNOTATE_CASES, MATCH_CASES, WALK_CASES, _ann_case, match_case_log,
                                         walk_case_log)

    logs, checks = [], []
    for case in sorted(ANNOTATE_CASES):
        steps, expected = ANNOTATE_CASES[case]
        logs.append(_ann_case(steps))
        checks.append(("props", expected))
    for kind, where in WALK_CASES:
        m, expected = walk_case_log(kind, where)
        logs.append(m)
        checks.append(("text", expected))
    for a, b, match in MATCH_CASES:
        logs.append(match_case_log(a, b))
        checks.append(("live", ["xy", "z"] if match else ["x", "y", "z"]))
    bld = mte.Builder()
    for m in logs:
        bld.add_doc(m)
    batch = bld.batch()
    engine.load(batch)
    st = engine.replay()
    assert st["failed_docs"] == 0
    for d, (what, expected) in enumerate(checks):
        compare_doc(engine, batch, d)
        segs = json.loads(engine.segments_json(d))
        live = [s for s in segs if "removedSeq" not in s]
        if what == "text":
            assert engine.text(d) == expected and engine.length(d) == len(expected)
        elif what == "live":
            assert [s.get("text") for s in live] == expected
        else:
            at = 0
            for s in live:
                if at <= 1 < at + s["len"]:
                    assert s["text"] == "el" and json.loads(s["props"]) == expected
                    break
                at += s["len"]


def test_hbm_slot_exhaustion_completes(engine):
    """Far fewer HBM slots than resident k_hbmq waves (force_hbm: one wave per document, all launched
    at once; a slot budget of ~3 slots): waves without a slot spin in acquire_hslot until a holder --
    a resident wave of the same kernel, which always progresses -- releases one. The pass completes
    and every document matches the oracle (no spin-wait depends on another stream's
    kernel being co-resident)."""
    engine.generate(2, 384, 1500, n_clients=8, seed=29)
    batch = engine.export_batch()
    engine.set_option("force_hbm", 1)
    try:
        engine.replay()
        slot = engine.run_info()["slot_bytes"]
        engine.set_option("slot_budget_mb", max(1, (3 * slot) >> 20))
        engine.replay()
        info = engine.run_info()
    finally:
        engine.set_option("force_hbm", 0)
        engine.set_option("slot_budget_mb", 48 << 10)
    assert 1 <= info["hbm_waves"] <= 8 and info["lds_groups"] == 0, info  # hbm_waves = the slot count
    bad, _, _ = compare_batch_checksums(engine, batch)
    if bad:
        compare_doc(engine, batch, bad[0])
    assert not bad


def test_reloads_reuse_device_tables(engine):
    """mte_load keeps device tables that are large enough (DevBuf::fit): a small batch after a large
    one replays in the larger buffers, then the large one again, each matching the oracle."""
    big = mte.Builder()
    for s in range(40):
        big.add_doc(random_log(100 + s, n=600))
    small = mte.Builder()
    for s in range(5):
        small.add_doc(random_log(200 + s, n=150))
    for b in (big, small, big):
        batch = b.batch()
        engine.load(batch)
        engine.replay()
        for d in range(batch.n_docs):
            compare_doc(engine, batch, d)
