"""Incremental replay (option retain; reg_engine.hpp ckpt_save / ckpt_resume) on the CPU build of the row
engine: a log replayed in two passes -- ops [0, cut) checkpointed, then a fresh engine with a fresh
merge arena and map table continuing from the checkpoint -- ends in exactly the state of the one-pass
replay (Client.applyMsg is incremental, client.ts:805-836: the continued client is the same client).
Every product instantiation (lean, paged, PROPS, PROPS paged, PROPS + WIDE), cuts anywhere a message
ends, and the oracle as the anchor of the one-pass replay."""
import random

import numpy as np
import pytest

from tests import regcpu

END_OF_MSG = 0x1


def _cuts(ops, rng, k):
    ends = np.nonzero(ops["flags"] & END_OF_MSG)[0] + 1
    ends = ends[ends < len(ops)]
    return sorted(rng.sample(list(ends), min(k, len(ends))))


def _same(a, b):
    """Two replays' (stop, DocRes, rows, text, maps) agree on everything the outputs are made of."""
    at1, r1, rows1, t1, m1 = a
    at2, r2, rows2, t2, m2 = b
    assert at1 == at2
    for f in ("status", "ops", "msgs", "min_seq", "cur_seq", "height", "n_lb", "seg_next", "heap_size",
              "n_segs", "max_lb", "map_next"):
        assert int(r1[f]) == int(r2[f]), f
    for x, y in zip(rows1, rows2):
        assert np.array_equal(x, y)
    n = sum(int(v[0]) for v in rows1[0])
    assert np.array_equal(t1[:n], t2[:n])
    if m1 is not None:
        assert np.array_equal(m1, m2)


def _full(ops, pay, kind, pool, gp):
    if kind in (0, 1):
        at, r, rows, text = regcpu.replay(ops, pay, pool_rows=pool if kind == 1 else None)
        return at, r, rows, text, None
    at, r, rows, text, maps = regcpu.replay_props(ops, pay, gp, pool_rows=pool if kind in (3, 7) else 0,
                                                  wide=kind >= 6)
    return at, r, rows, text, maps


@pytest.mark.parametrize("kind,gen,gid,n,clients", [(0, 2, 1, 6000, 8), (1, 2, 2, 6000, 8), (0, 5, 3, 4000, 3),
                                                    (2, 3, 4, 5000, 8), (3, 3, 5, 5000, 8), (6, 3, 6, 1200, 40),
                                                    (7, 3, 2, 1100, 40), (2, 2, 8, 3000, 16)])
def test_continued_replay_equals_one_pass(kind, gen, gid, n, clients):
    ops, pay = regcpu.generated(gen, gid, n, n_clients=clients, seed=1000)
    gp = regcpu.GenProps() if kind >= 2 else None
    pool = 24 if kind in (1, 3) else 32
    full = _full(ops, pay, kind, pool, gp)
    assert int(full[1]["status"]) == 0
    if kind in (0, 1):  # the one-pass replay is itself the oracle's
        regcpu.compare(ops, pay, pool_rows=pool if kind == 1 else None)
    rng = random.Random(gid)
    for cut in _cuts(ops, rng, 4) + [1]:
        at, resumed, r, rows, text, maps = regcpu.replay_split(ops, pay, cut, kind=kind, pool_rows=pool, gp=gp)
        assert resumed == cut, "the continuation started over instead of resuming"
        _same(full, (at, r, rows, text, maps if kind >= 2 else None))


def test_continued_replay_after_arena_compaction():
    """The checkpoint carries the live merge-arena semispace (offsets kept), so arena text written
    before the cut is read back after it, across compactions on both sides (a small arena)."""
    ops, pay = regcpu.generated(2, 21, 8000, n_clients=4, seed=7)
    arena = len(pay) // 3 + 256
    full = regcpu.replay(ops, pay, arena_cap=arena)
    assert int(full[1]["status"]) == 0 and int(full[1]["n_gc"]) > 2
    for cut in _cuts(ops, random.Random(5), 3):
        at, resumed, r, rows, text, _ = regcpu.replay_split(ops, pay, cut, arena_cap=arena)
        assert resumed == cut
        _same((full[0], full[1], full[2], full[3], None), (at, r, rows, text, None))
