"""Document sharding across GPUs: documents are independent, so the only multi-GPU
structure is (1) an LPT assignment of documents to ranks balanced by op count and (2) one final
all-gather of 32-byte per-document summary records (RCCL over xGMI on the GPU box; gloo in CPU tests).
No collective touches the replay data path."""
import heapq

import numpy as np

from .mte import SUMMARY_DTYPE


def lpt_assign(op_counts, world):
    """Longest-processing-time-first: docs sorted by op count (desc), each to the least-loaded rank.
    Returns a list of doc-id arrays, one per rank, each ordered longest-first (so the longest
    document starts at t=0 inside the rank's kernel)."""
    order = np.argsort(-np.asarray(op_counts, dtype=np.int64), kind="stable")
    heap = [(0, r) for r in range(world)]
    shards = [[] for _ in range(world)]
    for d in order:
        load, r = heapq.heappop(heap)
        shards[r].append(int(d))
        heapq.heappush(heap, (load + int(op_counts[d]), r))
    return [np.asarray(s, dtype=np.int64) for s in shards]


def zipf_op_counts(n_docs, seed=0, lo=1000, hi=1_000_000):
    """C4 op counts: rank r (a random permutation of docs) gets clamp(floor(1e6 / r), 1e3, 1e6)."""
    rng = np.random.default_rng(seed)
    ranks = rng.permutation(n_docs) + 1
    return np.clip(hi // ranks, lo, hi).astype(np.int64)


def plan_shard(config, world, rank, docs, ops, zipf_lo=1000, zipf_hi=1_000_000):
    """The documents rank `rank` of `world` replays, as GLOBAL ids with their op counts (bench.py).
    C4: Zipf op counts over `docs` documents, LPT-assigned, longest first (strong scaling: the same
    262,144 documents at every world size). C5: `docs` equal documents, strided over the ranks.
    C2/C3 (weak scaling): `docs` documents per rank, ids rank*docs .. rank*docs+docs-1."""
    if config == "C4":
        counts = zipf_op_counts(docs, seed=0, lo=zipf_lo, hi=zipf_hi)
        mine = lpt_assign(counts, world)[rank]
        return mine.astype(np.int64), counts[mine].astype(np.int64)
    if config == "C5":
        ids = np.arange(rank, docs, world, dtype=np.int64)
        return ids, np.full(len(ids), ops, dtype=np.int64)
    ids = np.arange(rank * docs, (rank + 1) * docs, dtype=np.int64)
    return ids, np.full(docs, ops, dtype=np.int64)


def gather_summaries_rccl(engine, group=None):
    """The product path of the final gather: RCCL all-gather of the engine's summary records
    (include/mte.h mte_gather_summaries). torch.distributed only carries rank 0's 128-byte RCCL id."""
    import torch.distributed as dist

    from . import mte

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    obj = [mte.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    comm = engine.rccl_comm(obj[0], rank, world)
    try:
        return engine.gather_summaries(rank, world, comm)
    finally:
        mte.rccl_comm_destroy(comm)


def gather_summaries(summaries, group=None, device=None):
    """All-gather every rank's mte_doc_summary records (numpy SUMMARY_DTYPE) with torch.distributed.
    Ranks may hold different numbers of docs; counts are exchanged first."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    raw = np.ascontiguousarray(summaries).view(np.uint8)
    t = torch.from_numpy(raw.copy())
    if device is not None:
        t = t.to(device)
    n = torch.tensor([raw.size], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    mx = int(max(int(s.item()) for s in sizes))
    padded = torch.zeros(mx, dtype=torch.uint8, device=t.device)
    padded[: raw.size] = t
    outs = [torch.zeros_like(padded) for _ in range(world)]
    dist.all_gather(outs, padded, group=group)
    recs = [o[: int(s.item())].cpu().numpy().view(SUMMARY_DTYPE) for o, s in zip(outs, sizes)]
    return np.concatenate(recs) if recs else np.zeros(0, SUMMARY_DTYPE)
