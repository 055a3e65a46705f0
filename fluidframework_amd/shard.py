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
