"""bench.py — headline benchmark of the MI355X merge-tree replay engine.

Default workload (BASELINE.json configs[1], "C2"): 4096 synthetic SharedString documents x 10,000
sequenced ops each, insert/remove only, 8 simulated writers plus a read-only observer (SURVEY §8d
generator, run on the GPU). A step = one replay of the whole batch (Client.applyMsg for every
message of every document, client.ts:805-836) from empty state to every document's final state,
inputs resident in HBM. Multi-GPU: documents are sharded by doc id (each rank replays its own
4096-doc shard; weak scaling); the only collective is the final all-gather of 32-B per-document
summary records over RCCL/xGMI, outside the timed region.

Other configs (--config): C3 (65,536 docs x 10k ops with annotate, forced ties and overlapping
removes, per GPU, weak), C4 (262,144 docs, Zipf op counts clamp(1e6/r, 1e3, 1e6), LPT-sharded over
the ranks, strong), C5 (1,024 docs x 1M ops, MSN lag <= 64 so zamboni runs continuously, sharded
over the ranks, strong).

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sequenced ops applied/sec (whole node) + achieved HBM GB/s, 256k docs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
OP_RECORD_B, LEAF_BLOCK_B = 32, 512  # SURVEY §8(d) algorithmic bytes per op: 32 + P + 512
# SURVEY §8(d) configs. docs: per GPU for weak-scaling configs, whole job for strong ones.
CONFIGS = {
    "C2": {"docs": 4096, "ops": 10000, "kind": 2, "scaling": "weak", "steps": 5, "warmup": 1,
           "desc": "insert/remove around a 2048-char target"},
    "C3": {"docs": 65536, "ops": 10000, "kind": 3, "scaling": "weak", "steps": 3, "warmup": 1,
           "desc": "45/35/20 insert/remove/annotate, 15% forced ties and overlapping removes"},
    "C4": {"docs": 262144, "ops": 0, "kind": 2, "scaling": "strong", "steps": 2, "warmup": 0,
           "desc": "Zipf op counts clamp(1e6/r, 1e3, 1e6), C2 mix, LPT-sharded"},
    "C5": {"docs": 1024, "ops": 1000000, "kind": 5, "scaling": "strong", "steps": 2, "warmup": 0,
           "desc": "1M-op docs, C2 mix with MSN lag <= 64 (continuous zamboni)"},
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 5; 2 for C4/C5)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 1; 0 for C4/C5)")
    ap.add_argument("--docs", type=int, default=None)
    ap.add_argument("--ops", type=int, default=None)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--kind", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify-docs", type=int, default=32, help="docs checked against the oracle after timing")
    a = ap.parse_args()
    c = CONFIGS[a.config]
    a.docs = c["docs"] if a.docs is None else a.docs
    a.ops = c["ops"] if a.ops is None else a.ops
    a.kind = c["kind"] if a.kind is None else a.kind
    a.steps = c["steps"] if a.steps is None else a.steps
    a.warmup = c["warmup"] if a.warmup is None else a.warmup
    return a


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")  # RCCL over xGMI
    from fluidframework_amd import mte

    cfg = CONFIGS[args.config]
    eng = mte.Engine(local)
    t0 = time.time()
    # per-rank shard: distinct seeds => distinct documents
    if cfg["scaling"] == "weak":
        n_local, per_doc = args.docs, None
    elif args.config == "C4":
        from fluidframework_amd.shard import lpt_assign, zipf_op_counts

        counts = zipf_op_counts(args.docs, seed=0)
        mine = lpt_assign(counts, world)[rank]  # longest first
        n_local, per_doc = len(mine), counts[mine]
    else:  # C5: equal documents, contiguous shards
        n_local, per_doc = len(range(rank, args.docs, world)), None
    eng.generate(args.kind, n_local, args.ops, n_clients=args.clients, seed=1000 + rank, ops_per_doc=per_doc)
    gen_s = time.time() - t0
    log(f"rank {rank}: generated {n_local} docs ({args.config}) in {gen_s:.1f} s")
    batch = eng.export_batch()
    ops_np = mte.batch_ops(batch)
    ins = ops_np["type"] == mte.MTE_OP_INSERT
    payload_chars = int(ops_np["b"][ins].sum())
    n_ops_rank = int(len(ops_np))

    def step():
        return eng.replay()

    for _ in range(args.warmup):
        w = step()
        log(f"warmup step: {w['kernel_ms']:.1f} ms kernel, {w['ops']} ops")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    kms, lds_ms = [], []
    st = None
    for _ in range(args.steps):
        st = step()
        kms.append(st["kernel_ms"])
        lds_ms.append(eng.run_info()["lds_ms"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert st["failed_docs"] == 0, st
    ops_applied = st["ops"]
    total_ops = ops_applied
    if world > 1:  # shards may differ (C4): sum what every rank applied
        t = torch.tensor([ops_applied], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        total_ops = int(t.item())
    ms_per_step = elapsed / args.steps * 1000.0
    value = total_ops * args.steps / elapsed

    log(f"timed {args.steps} steps: {ms_per_step:.1f} ms/step, {value / 1e6:.1f} Mops/s")
    # final summary gather (RCCL all-gather of 32-B records), outside the timed region
    t1 = time.time()
    summ = eng.summaries()
    snap_host_s = time.time() - t1
    snap_bytes = int(summ["snapshot_bytes"].sum())
    if world > 1:
        from fluidframework_amd.shard import gather_summaries

        gathered = len(gather_summaries(summ, device="cuda"))
    else:
        gathered = len(summ)

    # roofline on the replay kernel: algorithmic bytes per launch / HIP-event kernel time
    alg_bytes = n_ops_rank * (OP_RECORD_B + LEAF_BLOCK_B) + payload_chars  # 1 B/char ASCII payload
    kernel_ms = sum(kms) / len(kms)
    info = eng.run_info()
    achieved = alg_bytes / (kernel_ms / 1000.0) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_replay.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("docs") == args.docs and pmc.get("ops") == args.ops and pmc.get("kind") == args.kind:
                traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    # verify a sample of documents against the CPU oracle (checker only)
    verified = None
    cpu = None
    if rank == 0:
        from oracle import replay_batch

        nv = min(args.verify_docs, n_local)
        if nv:
            o_ops, cks, sts = replay_batch(ctypes.addressof(batch), 0, nv, threads=args.cpu_threads)
            assert all(sts[d] == 0 for d in range(nv)), "oracle reports failing documents"
            verified = all(int(summ["checksum"][d]) == cks[d] and int(summ["status"][d]) == sts[d] for d in range(nv))
        log(f"oracle verification of {nv} docs: {verified}")
        if not args.no_cpu_baseline:
            # bounded sample: grow the doc count until ~cpu_seconds of oracle replay on cpu_threads threads
            nd = max(args.cpu_threads, 16)
            while True:
                nd = min(nd, n_local)
                c0 = time.perf_counter()
                c_ops, _, _ = replay_batch(ctypes.addressof(batch), 0, nd, threads=args.cpu_threads,
                                           with_snapshot=False)
                dt = time.perf_counter() - c0
                log(f"cpu baseline sample: {nd} docs, {c_ops} ops in {dt:.2f} s")
                if dt >= args.cpu_seconds * 0.5 or nd >= n_local:
                    break
                nd = int(nd * min(8.0, max(2.0, args.cpu_seconds / max(dt, 1e-3))))
            cpu = {"value": c_ops / dt, "unit": "ops/s", "cores": args.cpu_threads, "kind": "port",
                   "sample": f"oracle (tree-shaped C++ restatement) replaying docs 0..{nd - 1} of the same {args.config} batch "
                             f"({c_ops} ops, replay only) on {args.cpu_threads} threads in {dt:.2f} s"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "ops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": cfg["scaling"],
            "vs_baseline": None, "dtype": "int32", "data": "synthetic (GPU generator, SURVEY §8d)",
            "config": {"workload": f"{args.config}: {args.docs} docs"
                                   + (" per GPU" if cfg["scaling"] == "weak" else " per job")
                                   + (f" x {args.ops} ops" if args.ops else "") + f", {cfg['desc']}, {args.clients} writers",
                       "config_id": args.config, "docs_per_gpu": n_local, "ops_per_doc": args.ops or "zipf",
                       "clients": args.clients, "parallelism": f"doc-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "replay pass: mte::k_lds<false> + mte::k_hbmq<false> (concurrent streams)",
                         "kernel_ms": kernel_ms, "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "extra": {"ops_per_step_per_gpu": ops_applied, "lds_pass_ms": sum(lds_ms) / len(lds_ms),
                      "hbm_pass_ms": info["hbm_ms"], "docs_rerun_hbm": info["spilled"],
                      "docs_continued_hbm": info["continued"], "docs_hbm_waves": info["hbm_docs"],
                      "lds_groups": info["lds_groups"], "hbm_wave_slots": info["hbm_waves"], "gen_s": gen_s, "snapshot_host_s": snap_host_s,
                      "snapshot_bytes": snap_bytes, "summaries_gathered": gathered, "oracle_verified_docs": verified},
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
