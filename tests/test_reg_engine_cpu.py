"""CPU: the row-vectorised solo engine (fluidframework_amd/csrc/reg_engine.hpp) built with the emulated
wave backend (tests/native/reg_cpu.cpp) against the oracle on the same op records: segment table
(text, boundaries, seq / client / removal info, overlap sets) and observer text, bit-exact. The device
build of the same source runs on k_solo (tests/test_gpu_reg.py)."""
import ctypes
import json
import random

import numpy as np
import pytest

from fluidframework_amd import mte
from tests import regcpu
from tests.oplog import dumps, ins, msg, rem


@pytest.mark.parametrize("kind", [2, 5])
@pytest.mark.parametrize("clients", [2, 3, 8, 16])
def test_generated_documents(kind, clients):
    for gid in range(4):
        n = [1, 40, 900, 6000][gid]
        ops, pay = regcpu.generated(kind, 1000 + gid, n, n_clients=clients, seed=clients)
        regcpu.compare(ops, pay)


def test_critical_path_document_prefix():
    """The first 200k ops of C4's longest document (global id 111877, SURVEY §8d's Zipf head)."""
    ops, pay = regcpu.generated(2, 111877, 200_000, n_clients=8, seed=1000)
    r = regcpu.compare(ops, pay)
    assert int(r["max_lb"]) <= 200 and int(r["height"]) >= 3


@pytest.mark.parametrize("arena_cap", [1200, 3000])
def test_arena_compaction(arena_cap):
    """A small merge arena forces the semispace compaction (arena_gc) many times."""
    ops, pay = regcpu.generated(2, 77, 15_000, n_clients=8, seed=3)
    r = regcpu.compare(ops, pay, arena_cap=arena_cap)
    assert int(r["n_gc"]) > 10


@pytest.mark.parametrize("kind", [2, 5])
def test_paged_rows_match_oracle(kind):
    """k_rows' PAGED engine: logical rows in pool rows taken in a scattered order as the document
    grows and given back as it shrinks (block moves and splits cross pool rows), bit-exact with the
    oracle; C2-shaped documents whose leaf blocks peak near 100."""
    for gid in (256, 1792, 3584):
        ops, pay = regcpu.generated(kind, gid, 10_000, n_clients=8, seed=1000)
        r = regcpu.compare(ops, pay, pool_rows=32)
        assert int(r["max_lb"]) > 16


def test_paged_pool_exhausted_spills():
    """A pool too small for the document stops it with REG_HANDOFF (k_rows marks it for the host's
    re-run) instead of failing it."""
    ops, pay = regcpu.generated(2, 256, 10_000, n_clients=8, seed=1000)
    at, res, _, _ = regcpu.replay(ops, pay, pool_rows=4)
    assert int(res["status"]) == regcpu.REG_HANDOFF and 0 < at < len(ops)


def test_outgrows_the_rows_and_hands_off():
    """31 concurrent writers keep hundreds of tombstones and heap entries in the collaboration window:
    the document outgrows the row plan's margins (leaf blocks, level-1 nodes or heap) and would hand
    off to the LDS engine between two ops (GPU only: tests/test_gpu_reg.py)."""
    ops, pay = regcpu.generated(2, 4, 3000, n_clients=31, seed=4)
    at, res, _, _ = regcpu.replay(ops, pay)
    assert int(res["status"]) == regcpu.REG_HANDOFF and 0 < at < len(ops)
    assert int(res["n_lb"]) > 100


def _builder_ops(msgs):
    b = mte.Builder()
    b.add_doc(dumps(msgs))
    batch = b.batch()
    ops = mte.batch_ops(batch).copy()
    n_pay = batch.doc_payload_offsets[1]
    pay = np.ctypeslib.as_array(batch.payload, shape=(max(n_pay, 1),))[:n_pay].copy()
    cno = batch.client_name_offsets
    names = [ctypes.string_at(batch.client_names + cno[i], cno[i + 1] - cno[i]).decode()
             for i in range(batch.doc_client_offsets[1])]
    return ops, pay, names


@pytest.mark.parametrize("seed", range(4))
def test_markers_and_concurrent_writers_from_json(seed):
    """Marker inserts (no properties), overlapping removes and ties from concurrent writers, through
    the JSON builder: the engine's records path against the oracle's."""
    from oracle import OracleDoc

    rng = random.Random(seed)
    d = OracleDoc()
    msgs, refs, seq, order = [], {c: 0 for c in "abcde"}, 0, []
    for _ in range(1500):
        c = rng.choice("abcde")
        refs[c] = rng.randint(max(refs[c], seq - 12), seq)
        if c not in order:
            order.append(c)
        L = d.length_at(refs[c], order.index(c) + 1)
        if L == 0 or rng.random() < 0.5:
            seg = {"marker": {"refType": rng.choice([0, 1, 2])}} if rng.random() < 0.15 else \
                "".join(rng.choice("pq") for _ in range(rng.randint(1, 5)))
            contents = ins(rng.randint(0, L), seg)
        else:
            a = rng.randint(0, L - 1)
            contents = rem(a, min(L, a + rng.randint(1, 7)))
        seq += 1
        m = msg(c, seq, refs[c], contents, min(refs.values()))
        msgs.append(m)
        d.apply_json(dumps([m]))
    ops, pay, names = _builder_ops(msgs)
    assert (ops["type"] == mte.MTE_OP_INSERT_MARKER).sum() > 50
    res = regcpu.compare(ops, pay, names=names)
    assert int(res["n_segs"]) == len(json.loads(d.segments_json()))


@pytest.mark.parametrize("seed", range(3))
def test_long_segments_granularity(seed):
    """Inserts of 1..600 characters: zamboni's merge runs meet TextSegment.canAppend's granularity
    test (textSegment.ts:63-85, either side <= 256 by the run's accumulated length), which the
    lane-parallel scour hands to the serial walk; short runs merge lane-parallel, contiguous or not."""
    from oracle import OracleDoc

    rng = random.Random(100 + seed)
    d = OracleDoc()
    msgs, refs, seq, order = [], {c: 0 for c in "abc"}, 0, []
    for _ in range(1200):
        c = rng.choice("abc")
        refs[c] = rng.randint(max(refs[c], seq - 6), seq)
        if c not in order:
            order.append(c)
        L = d.length_at(refs[c], order.index(c) + 1)
        if L == 0 or rng.random() < 0.6:
            n = rng.choice([1, 2, 5, 40, 120, 250, 257, 300, 600])
            contents = ins(rng.randint(0, L), "".join(rng.choice("xyz") for _ in range(n)))
        else:
            a = rng.randint(0, L - 1)
            contents = rem(a, min(L, a + rng.randint(1, 30)))
        seq += 1
        m = msg(c, seq, refs[c], contents, min(refs.values()))
        msgs.append(m)
        d.apply_json(dumps([m]))
    ops, pay, names = _builder_ops(msgs)
    res = regcpu.compare(ops, pay, names=names)
    assert int(res["n_segs"]) == len(json.loads(d.segments_json()))


def _heap_pops(ops):
    """collections.ts:213-265 restated: push appends then sifts up while the parent is strictly
    larger; pop moves the last entry to the root and sifts down to the smaller child (left on
    ties) while that child is strictly smaller."""
    h, out = [None], []
    for i, k in enumerate(ops):
        if k > 0:
            h.append((k, i + 1))
            j = len(h) - 1
            while j > 1 and h[j // 2][0] > h[j][0]:
                h[j // 2], h[j] = h[j], h[j // 2]
                j //= 2
        elif len(h) > 1:
            out.append(h[1][1])
            last = h.pop()
            if len(h) > 1:
                h[1] = last
                k2, m = 1, len(h) - 1
                while 2 * k2 <= m:
                    j = 2 * k2
                    if j < m and h[j][0] > h[j + 1][0]:
                        j += 1
                    if last[0] <= h[j][0]:
                        break
                    h[k2] = h[j]
                    k2 = j
                h[k2] = last
    return out


@pytest.mark.parametrize("seed", range(6))
def test_lru_heap_pop_order(seed):
    """The engine's heap (lane-parallel pop up to 127 entries, serial beyond) pops in exactly the
    reference heap's order, ties included (keys are op seqs: non-decreasing pushes, runs of equal
    keys from one op)."""
    rng = random.Random(seed)
    ops, key, size = [], 1, 0
    target = [20, 100, 126, 127, 128, 300][seed]
    for _ in range(6000):
        if size < target and (size == 0 or rng.random() < 0.55):
            key += rng.choice([0, 0, 1, 1, 2])
            ops.append(key)
            size += 1
        else:
            ops.append(0)
            size -= 1
    arr = np.array(ops, dtype=np.int32)
    out = np.zeros(len(ops), dtype=np.uint32)
    n = regcpu.lib().regcpu_heap(arr.ctypes.data, len(ops), out.ctypes.data)
    assert list(out[:n]) == _heap_pops(ops)


@pytest.mark.parametrize("gid,n_ops,clients,pool", [(1, 3000, 8, 0), (2, 10_000, 8, 0), (3, 10_000, 8, 32),
                                                    (4, 6000, 16, 0), (7, 20_000, 8, 24), (9, 2000, 31, 0)])
def test_props_engine_matches_oracle(gid, n_ops, clients, pool):
    """The PROPS row engine (k_rows for property-carrying batches): C3-mix logs (45/35/20 insert /
    remove / annotate, 15 % forced ties), property maps built on insert and annotate, merges only
    between segments whose maps match (deep, not by id), paged rows when pool > 0; segment table
    with every segment's properties and the text against the oracle."""
    ops, pay = regcpu.generated(3, gid, n_ops, n_clients=clients, seed=1000)
    assert (ops["type"] == 2).sum() > n_ops // 10
    r = regcpu.compare_props(ops, pay, pool_rows=pool)
    assert int(r["map_next"]) > n_ops // 4


def test_props_engine_rewrite_annotates():
    """annotate with combiningOp rewrite (MTE_F_REWRITE: keys whose new value is falsy or absent are
    dropped, segmentPropertiesManager.ts:65-78) on every third annotate of a C3-mix log."""
    ops, pay = regcpu.generated(3, 11, 8000, n_clients=8, seed=1000)
    ann = np.nonzero(ops["type"] == 2)[0][::3]
    ops = ops.copy()
    ops["flags"][ann] |= 0x2
    regcpu.compare_props(ops, pay)


@pytest.mark.parametrize("kind,gid,n_ops,clients", [(3, 2, 1100, 40), (2, 3, 1200, 48), (3, 4, 1100, 63),
                                                    (3, 7, 1100, 50), (5, 5, 8000, 36), (3, 1, 4000, 8)])
def test_wide_engine_matches_oracle(kind, gid, n_ops, clients):
    """k_solo's FULL instantiation (PROPS + WIDE): removers 32..63 in a second mask word per slot
    (removedClient and removedClientOverlap of clients up to 63), with and without properties;
    segment table incl. overlap sets and text against the oracle."""
    ops, pay = regcpu.generated(kind, gid, n_ops, n_clients=clients, seed=1000)
    assert clients < 32 or (ops["client"] >= 32).sum() > 0
    regcpu.compare_props(ops, pay, wide=True)


@pytest.mark.parametrize("kind,gid,n_ops,clients,pool", [(3, 2, 1100, 40, 32), (2, 3, 1100, 48, 32),
                                                         (3, 4, 1100, 63, 30), (5, 5, 4000, 36, 24)])
def test_wide_paged_engine_matches_oracle(kind, gid, n_ops, clients, pool):
    """k_rows' WIDE instantiation (PAGED + PROPS + WIDE: batches with writers 32..63 on the shared
    row pool; rows taken in a scattered order from a pool of `pool` rows): the second removers word
    moves with its slots through the pool-row table; segment table and text against the oracle."""
    ops, pay = regcpu.generated(kind, gid, n_ops, n_clients=clients, seed=1000)
    assert (ops["client"] >= 32).sum() > 0
    regcpu.compare_props(ops, pay, pool_rows=pool, wide=True)


@pytest.mark.parametrize("seed", range(12))
def test_row_engine_variants_random_logs(seed):
    """Randomised logs (kind, writers 2-63, length) through every row-engine instantiation the
    product builds -- lean, lean paged, PROPS, PROPS paged, PROPS + WIDE, paged PROPS + WIDE -- each
    against the oracle."""
    rng = random.Random(seed)
    kind = rng.choice([2, 3, 5])
    clients = rng.choice([2, 3, 8, 16, 31]) if seed % 3 else rng.randint(32, 63)
    n = rng.randint(200, 2500) if clients < 32 else rng.randint(200, 900)
    ops, pay = regcpu.generated(kind, 500 + seed, n, n_clients=clients, seed=seed)
    regcpu.compare_props(ops, pay, wide=True)
    regcpu.compare_props(ops, pay, pool_rows=32, wide=True)
    if clients >= 32:
        return
    regcpu.compare_props(ops, pay, pool_rows=rng.randint(12, 32))
    regcpu.compare_props(ops, pay)
    if kind != 3:
        regcpu.compare(ops, pay)
        regcpu.compare(ops, pay, pool_rows=rng.randint(12, 32))
