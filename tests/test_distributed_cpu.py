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
