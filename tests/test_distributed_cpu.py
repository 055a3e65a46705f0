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


def _bench_shard_worker(rank, world, port, q):
    """One rank of bench.py's C4 path at CPU scale: plan_shard -> generate (global ids) -> replay ->
    summary records -> all-gather (gloo here; RCCL's mte_gather_summaries on the box)."""
    import torch.distributed as dist

    from fluidframework_amd.shard import plan_shard
    from oracle import generate_batch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids, counts = plan_shard("C4", world, rank, 96, 0, zipf_lo=50, zipf_hi=3000)
    _, cks, sts = generate_batch(2, ids, counts, n_clients=8, seed=1000, threads=2)
    recs = np.zeros(len(ids), dtype=SUMMARY_DTYPE)
    recs["checksum"] = cks
    recs["status"] = sts
    recs["doc_id"] = ids
    recs["ops"] = counts
    allrecs = gather_summaries(recs)
    q.put((rank, allrecs.tobytes()))
    dist.destroy_process_group()


def test_bench_shard_and_gather_world2_equals_world1():
    """bench.py's sharding at world 2 replays exactly the documents of world 1: the gathered,
    rank-concatenated summary records, sorted by global id, equal a single-process run."""
    from fluidframework_amd.shard import plan_shard
    from oracle import generate_batch

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    g = np.frombuffer(res[0], dtype=SUMMARY_DTYPE)
    g = g[np.argsort(g["doc_id"])]
    ids, counts = plan_shard("C4", 1, 0, 96, 0, zipf_lo=50, zipf_hi=3000)
    assert sorted(g["doc_id"].tolist()) == list(range(96)) == sorted(ids.tolist())
    order = np.argsort(ids)
    _, cks, sts = generate_batch(2, ids[order], counts[order], n_clients=8, seed=1000, threads=4)
    assert g["checksum"].tolist() == cks and all(s == 0 for s in sts)
    # LPT: rank loads differ by at most the longest document
    loads = [plan_shard("C4", 2, r, 96, 0, zipf_lo=50, zipf_hi=3000)[1].sum() for r in range(2)]
    assert abs(loads[0] - loads[1]) <= 3000
