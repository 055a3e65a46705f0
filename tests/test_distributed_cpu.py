"""Multi-GPU structure on CPU (gloo, world_size 2): LPT doc sharding + the final summary all-gather.
Summaries here come from the oracle (no GPU in this container); on the box the same gather runs over
RCCL with the engine's mte_summaries records."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fluidframework_amd.mte import SUMMARY_DTYPE
from fluidframework_amd.shard import gather_summaries, lpt_assign, zipf_op_counts


def test_lpt_balances_zipf():
    counts = zipf_op_counts(4096, seed=1)
    for world in (2, 4, 8):
        shards = lpt_assign(counts, world)
        assert sorted(np.concatenate(shards).tolist()) == list(range(4096))
        loads = [counts[s].sum() for s in shards]
        # the critical path is the 1M-op doc; LPT keeps every rank within one max-doc of the mean
        assert max(loads) - min(loads) <= counts.max()
        for s in shards:
            assert list(counts[s]) == sorted(counts[s], reverse=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from oracle import OracleDoc
    from tests.test_builder_cpu import random_log
    from tests.oplog import dumps

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    docs = [d for d in range(6) if d % world == rank]  # this rank's shard
    recs = np.zeros(len(docs), dtype=SUMMARY_DTYPE)
    for i, d in enumerate(docs):
        o = OracleDoc()
        o.apply_json(dumps(random_log(100 + d, n=150)))
        recs[i]["checksum"] = o.checksum()
        recs[i]["doc_id"] = d
        recs[i]["ops"] = o.ops_applied()
        recs[i]["length"] = len(o.text())
    allrecs = gather_summaries(recs)
    q.put((rank, allrecs.tobytes()))
    dist.destroy_process_group()


def test_summary_gather_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = np.frombuffer(res[0], dtype=SUMMARY_DTYPE)
    b = np.frombuffer(res[1], dtype=SUMMARY_DTYPE)
    assert a.tobytes() == b.tobytes()
    assert sorted(a["doc_id"].tolist()) == list(range(6))
    # every rank sees the same per-doc checksums a single process computes
    from oracle import OracleDoc
    from tests.oplog import dumps
    from tests.test_builder_cpu import random_log

    for rec in a:
        o = OracleDoc()
        o.apply_json(dumps(random_log(100 + int(rec["doc_id"]), n=150)))
        assert int(rec["checksum"]) == o.checksum()


# bench.py's shard plans at CPU scale: C4 (Zipf, LPT) and C5 (equal documents, strided; kind 5)
PLANS = {"C4": dict(kind=2, docs=96, ops=0, zipf_lo=50, zipf_hi=3000), "C5": dict(kind=5, docs=40, ops=1500)}


def _plan(config, world, rank):
    from fluidframework_amd.shard import plan_shard

    c = PLANS[config]
    extra = {k: c[k] for k in ("zipf_lo", "zipf_hi") if k in c}
    return plan_shard(config, world, rank, c["docs"], c["ops"], **extra)


def _bench_shard_worker(rank, world, port, q, config="C4"):
    """One rank of bench.py's C4 / C5 path at CPU scale: plan_shard -> generate (global ids) -> replay
    -> summary records -> all-gather (gloo here; RCCL's mte_gather_summaries on the box)."""
    import torch.distributed as dist

    from oracle import generate_batch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids, counts = _plan(config, world, rank)
    _, cks, sts = generate_batch(PLANS[config]["kind"], ids, counts, n_clients=8, seed=1000, threads=2)
    recs = np.zeros(len(ids), dtype=SUMMARY_DTYPE)
    recs["checksum"] = cks
    recs["status"] = sts
    recs["doc_id"] = ids
    recs["ops"] = counts
    allrecs = gather_summaries(recs)
    q.put((rank, allrecs.tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("config", ["C4", "C5"])
def test_bench_shard_and_gather_world2_equals_world1(config):
    """bench.py's sharding at world 2 replays exactly the documents of world 1 (C4: LPT over Zipf
    op counts; C5: equal documents strided over the ranks): the gathered, rank-concatenated summary
    records, sorted by global id, equal a single-process run."""
    from oracle import generate_batch

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_shard_worker, args=(r, 2, port, q, config)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    g = np.frombuffer(res[0], dtype=SUMMARY_DTYPE)
    g = g[np.argsort(g["doc_id"])]
    n = PLANS[config]["docs"]
    ids, counts = _plan(config, 1, 0)
    assert sorted(g["doc_id"].tolist()) == list(range(n)) == sorted(ids.tolist())
    order = np.argsort(ids)
    _, cks, sts = generate_batch(PLANS[config]["kind"], ids[order], counts[order], n_clients=8, seed=1000, threads=4)
    assert g["checksum"].tolist() == cks and all(s == 0 for s in sts)
    loads = [_plan(config, 2, r)[1].sum() for r in range(2)]
    if config == "C4":  # LPT: rank loads differ by at most the longest document
        assert abs(loads[0] - loads[1]) <= 3000
    else:  # strided equal documents: the ranks' document counts differ by at most one
        assert abs(len(_plan(config, 2, 0)[0]) - len(_plan(config, 2, 1)[0])) <= 1
