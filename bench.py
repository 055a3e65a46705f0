"""bench.py — headline benchmark of the MI355X merge-tree replay engine.

Default workload = the configuration BASELINE.json's metric is quoted on ("... 256k docs"), C4:
262,144 synthetic SharedString documents with Zipf-skewed op counts clamp(1e6/r, 1e3, 1e6)
(268.6 M sequenced ops, one document of 1 M ops), 8 simulated writers plus a read-only observer
(SURVEY §8d generator, run on the GPU). A step = one replay of the whole batch (Client.applyMsg for
every message of every document, client.ts:805-836) from empty state to every document's final
state, inputs resident in HBM.

Multi-GPU: documents are sharded by GLOBAL doc id, one process per GPU. C4 is strong
scaling: the same 262,144 documents at every N, LPT-assigned by op count, each document seeded by
its global id, so an N-GPU run replays exactly the documents of the 1-GPU run. The only collective
is the final RCCL all-gather of the 32-B per-document summary records (outside the timed region).
`python bench.py --gpus N` with no WORLD_SIZE in the environment spawns the N ranks itself
(fresh processes, before anything touches a GPU); under torch.distributed.run it is one rank.

Other configs (--config): C2 (4,096 docs x 10k ops per GPU, weak), C3 (65,536 docs x 10k ops with
annotate, forced ties and overlapping removes, per GPU, weak), C5 (1,024 docs x 1M ops, MSN lag <= 64
so zamboni runs continuously, strided over the ranks, strong).

Prints ONE JSON line (rank 0). Exits non-zero if a document fails or the oracle check disagrees.
"""
import argparse
import ctypes
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sequenced ops applied/sec (whole node) + achieved HBM GB/s, 256k docs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# measured on the box (tools/microbench/stream.hip, profiles/r06/stream.txt): float4 streams over 4 GiB
# buffers, best of 10 launches -- read-only, write-only and copy (read + write bytes)
HBM_MEASURED_GBS = {"read": 6175.1, "write": 5386.2, "copy": 4679.2, "source": "profiles/r06/stream.txt"}
OP_RECORD_B, LEAF_BLOCK_B = 32, 512  # SURVEY §8(d) algorithmic bytes per op: 32 + P + 512
# SURVEY §8(d) configs. docs: per GPU for weak-scaling configs, whole job for strong ones.
CONFIGS = {
    "C2": {"docs": 4096, "ops": 10000, "kind": 2, "scaling": "weak", "steps": 5, "warmup": 1,
           "desc": "insert/remove around a 2048-char target"},
    "C3": {"docs": 65536, "ops": 10000, "kind": 3, "scaling": "weak", "steps": 3, "warmup": 1,
           "desc": "45/35/20 insert/remove/annotate, 15% forced ties and overlapping removes"},
    "C4": {"docs": 262144, "ops": 0, "kind": 2, "scaling": "strong", "steps": 3, "warmup": 1,
           "desc": "Zipf op counts clamp(1e6/r, 1e3, 1e6), C2 mix, LPT-sharded by global doc id"},
    "C5": {"docs": 1024, "ops": 1000000, "kind": 5, "scaling": "strong", "steps": 2, "warmup": 0,
           "desc": "1M-op docs, C2 mix with MSN lag <= 64 (continuous zamboni)"},
}
GEN_SEED = 1000  # one seed for every rank: documents differ by global id only


def ops_to_messages(ops, pay, lo, hi):
    """Op records [lo, hi) of a generated document (one message per record: C2 / C5 mixes carry text
    inserts and removes only) as the ISequencedDocumentMessage JSON the builder ingests."""
    out = []
    for o in ops[lo:hi]:
        t = int(o["type"])
        if t == 0:
            a, b = int(o["a"]), int(o["b"])
            c = {"pos1": int(o["pos1"]), "seg": pay[a:a + b].tobytes().decode("utf-16-le"), "type": 0}
        else:
            c = {"pos1": int(o["pos1"]), "pos2": int(o["a"]), "type": 1}
        out.append({"clientId": f"w{int(o['client'])}", "sequenceNumber": int(o["seq"]),
                    "referenceSequenceNumber": int(o["ref_seq"]), "minimumSequenceNumber": int(o["msn"]),
                    "type": "op", "contents": c})
    return out


def catchup_probe(args, n_docs=16, n_ops=20000):
    """What a summarizer catching up C5-shaped documents meets: each document of
    a generated C5-mix batch is cut at a random message, its prefix replayed and summarized on the GPU
    (SnapshotV1, chunk size 10 000: the reference's default), and the summary loaded with the rest of
    the log (SnapshotLoader + applyMsg). Outcomes by document: loaded, the reference's own "insert
    failed" (loadBody's never-cleared batch), refused (MTE_DOC_UNSUPPORTED: the aliased re-link),
    and how many summaries had body chunks. Product path only (the oracle is not used)."""
    import numpy as np

    from fluidframework_amd import mte
    rng = np.random.default_rng(7)
    t0 = time.time()
    g = mte.Engine(0)
    g.generate(5, n_docs, n_ops, n_clients=8, seed=GEN_SEED)
    b = g.export_batch()
    ops = mte.batch_ops(b).copy()
    npay = b.doc_payload_offsets[b.n_docs]
    pay = np.frombuffer(bytes((ctypes.c_uint16 * npay).from_address(ctypes.addressof(b.payload.contents))),
                        dtype=np.uint16)
    cuts, logs = [], []
    pre = mte.Builder()
    for d in range(n_docs):
        lo, hi = b.doc_op_offsets[d], b.doc_op_offsets[d + 1]
        p0 = b.doc_payload_offsets[d]
        cut = int(rng.integers((hi - lo) // 4, 3 * (hi - lo) // 4))
        msgs = ops_to_messages(ops, pay[p0:], lo, hi)
        logs.append(msgs)
        cuts.append(cut)
        pre.add_doc(msgs[:cut], observer="__observer__")
    g.close()
    e = mte.Engine(0)
    e.load(pre.batch())
    e.replay()
    summaries = [e.snapshot_json(d) for d in range(n_docs)]
    body = sum(1 for s in summaries if len(json.loads(s)["entries"]) > 1)
    cu = mte.Builder()
    for d in range(n_docs):
        cu.add_doc_from_summary(summaries[d], logs[d][cuts[d]:], observer="__observer__")
    e.load(cu.batch())
    e.replay()
    st = [e.status(d)[0] for d in range(n_docs)]
    e.close()
    return {"docs": n_docs, "ops_per_doc": n_ops, "summaries_with_body_chunks": body,
            "loaded": st.count(0), "insert_failed": st.count(1), "refused": st.count(4),
            "other": n_docs - st.count(0) - st.count(1) - st.count(4), "seconds": round(time.time() - t0, 2)}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="C4", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=None, help="timed steps (config default)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (config default)")
    ap.add_argument("--docs", type=int, default=None)
    ap.add_argument("--ops", type=int, default=None)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--catchup-probe", type=int, default=1, help="0: skip the catch-up outcome probe")
    ap.add_argument("--kind", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--cpu-threads", type=int, default=None, help="default: one per host core available")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify-docs", type=int, default=32, help="docs checked against the oracle after timing")
    ap.add_argument("--opt", action="append", default=[], help="engine option key=value (A/B runs; repeatable)")
    a = ap.parse_args(argv)
    c = CONFIGS[a.config]
    a.docs = c["docs"] if a.docs is None else a.docs
    a.ops = c["ops"] if a.ops is None else a.ops
    a.kind = c["kind"] if a.kind is None else a.kind
    a.steps = c["steps"] if a.steps is None else a.steps
    a.warmup = c["warmup"] if a.warmup is None else a.warmup
    return a


def host_cores():
    """(cores this process can use, how that was determined): its CPU affinity, capped by the cgroup
    CPU quota (cpu.max), which is what bounds a container's parallel CPU throughput."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    why = f"sched_getaffinity {avail}, os.cpu_count {os.cpu_count()}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            why += f", cgroup cpu.max quota {q} CPUs"
            avail = min(avail, q)
    except (OSError, ValueError):
        pass
    return avail, why


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for the CPU baseline's record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_entry(rank, world, port, argv):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run(parse(argv))


def launch(args, argv):
    """`--gpus N` without a launcher: N fresh rank processes (spawned before any GPU call here)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, args.gpus, port, argv)) for r in range(args.gpus)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    return max(abs(p.exitcode or 0) for p in procs)


def run(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")  # RCCL; carries only barriers, the max-time reduce and the RCCL id
    from fluidframework_amd import mte
    from fluidframework_amd.shard import gather_summaries_rccl, plan_shard

    cfg = CONFIGS[args.config]
    eng = mte.Engine(local)
    for kv in args.opt:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    t0 = time.time()
    ids, counts = plan_shard(args.config, world, rank, args.docs, args.ops)
    n_local = len(ids)
    eng.generate(args.kind, n_local, args.ops, n_clients=args.clients, seed=GEN_SEED, ops_per_doc=counts,
                 doc_ids=ids)
    gen_s = time.time() - t0
    log(f"rank {rank}/{world}: generated {n_local} docs ({args.config}, {int(counts.sum())} ops) in {gen_s:.1f} s")
    batch = eng.export_batch()
    ops_np = mte.batch_ops(batch)
    ins = ops_np["type"] == mte.MTE_OP_INSERT
    payload_chars = int(ops_np["b"][ins].sum())
    n_ops_rank = int(len(ops_np))

    for _ in range(args.warmup):
        w = eng.replay()
        log(f"warmup step: {w['kernel_ms']:.1f} ms kernel, {w['ops']} ops")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    kms = []
    st = None
    solo_steps, solo_clk = [], []
    for _ in range(args.steps):
        st = eng.replay()
        kms.append(st["kernel_ms"])
        solo_steps.append(eng.get_info("solo_us") / 1000.0)  # host-side read of the last pass's events
        # the critical wave's s_memtime cycles and s_memrealtime (100 MHz) ticks over its replay
        solo_clk.append((eng.get_info("solo_cycles"), eng.get_info("solo_ref_ticks"),
                         eng.get_info("solo_start_delay_ticks")))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if st["failed_docs"]:
        log(f"FAILED documents: {st}")
        sys.exit(3)
    ops_applied = st["ops"]
    total_ops = ops_applied
    if world > 1:  # shards differ in size (C4): sum what every rank applied
        t = torch.tensor([ops_applied], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        total_ops = int(t.item())
    ms_per_step = elapsed / args.steps * 1000.0
    value = total_ops * args.steps / elapsed
    log(f"timed {args.steps} steps: {ms_per_step:.1f} ms/step, {value / 1e6:.1f} Mops/s")
    info = eng.run_info()
    solo = [eng.doc_result(d) for d in range(min(info["solo"], n_local))]

    # final summary gather (RCCL all-gather of 32-B records), outside the timed region
    t1 = time.time()
    summ = eng.summaries()  # this rank's records: checksum of text + SnapshotV1 bytes per document
    snap_host_s = time.time() - t1
    gathered = len(gather_summaries_rccl(eng)) if world > 1 else len(summ)
    snap_bytes = int(summ["snapshot_bytes"].sum())

    # roofline of the replay pass: algorithmic bytes per launch / HIP-event pass time
    # + the SnapshotV1 bytes the pass emits (emit.hip, inside the timed step)
    alg_bytes = n_ops_rank * (OP_RECORD_B + LEAF_BLOCK_B) + payload_chars + snap_bytes  # 1 B/char ASCII payload
    kernel_ms = sum(kms) / len(kms)
    achieved = alg_bytes / (kernel_ms / 1000.0) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_replay_{args.config}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("docs") == n_local and pmc.get("ops") == int(counts.sum()) and pmc.get("kind") == args.kind:
                traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    # verify a sample of this rank's documents against the CPU oracle (checker only)
    from oracle import replay_batch

    nv = min(args.verify_docs, n_local)
    verified = True
    if nv:
        o_ops, cks, sts = replay_batch(ctypes.addressof(batch), 0, nv, threads=min(16, nv))
        verified = all(sts[d] == 0 for d in range(nv)) and all(
            int(summ["checksum"][d]) == cks[d] and int(summ["status"][d]) == sts[d] and int(summ["doc_id"][d]) == ids[d]
            for d in range(nv))
    if world > 1:
        t = torch.tensor([1 if verified else 0], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        verified = bool(t.item())
    log(f"oracle verification of {nv} docs per rank (incl. the longest): {verified}")
    if not verified:
        sys.exit(4)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import replay_list

        cores, why = host_cores()
        threads = args.cpu_threads or cores
        # bounded, size-stratified sample of the same batch: every k-th document of the LPT order
        # (longest first, so the critical-path document is in it and the op-count distribution is
        # kept); k from a short calibration so the sample takes ~cpu_seconds on `threads` threads
        mid = n_local // 2
        m = min(n_local - mid, 64 * threads)
        c0 = time.perf_counter()
        cal = replay_list(ctypes.addressof(batch), np.arange(mid, mid + m), threads=threads)
        per_s = cal / max(time.perf_counter() - c0, 1e-3)
        k = 1
        while k < n_local and counts[::k].sum() / per_s > args.cpu_seconds:
            k *= 2
        sample = np.arange(0, n_local, k)
        c0 = time.perf_counter()
        c_ops = replay_list(ctypes.addressof(batch), sample, threads=threads)
        dt = time.perf_counter() - c0
        log(f"cpu baseline sample: every {k}th doc ({len(sample)} docs), {c_ops} ops in {dt:.2f} s on {threads} threads")
        cpu = {"value": c_ops / dt, "unit": "ops/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
               "sample": f"oracle (tree-shaped C++ restatement of the reference path) replaying every {k}th "
                         f"document ({len(sample)} docs, {c_ops} ops, replay only, longest first) of the same "
                         f"{args.config} batch on {threads} threads, one per usable host core ({why}), in {dt:.2f} s"}

    probe = catchup_probe(args) if rank == 0 and args.catchup_probe else None

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "ops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": cfg["scaling"],
            "vs_baseline": None, "dtype": "int32", "data": "synthetic (GPU generator, SURVEY §8d)",
            "config": {"workload": f"{args.config}: {args.docs} docs"
                                   + (" per GPU" if cfg["scaling"] == "weak" else " per job")
                                   + (f" x {args.ops} ops" if args.ops else f", {total_ops} ops")
                                   + f", {cfg['desc']}, {args.clients} writers",
                       "config_id": args.config, "docs_per_gpu": n_local, "ops_per_doc": args.ops or "zipf",
                       "ops_per_step": total_ops, "clients": args.clients, "parallelism": f"doc-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "measured_peak_gbs": HBM_MEASURED_GBS,
                         "kernel": "replay pass: mte::k_solo + mte::k_rows (the bulk; k_lds / k_hbmq for batches the rows cannot take) + mte::k_rows_cont (concurrent streams) + SnapshotV1 emission (mte::k_emit_count/k_emit_write, overlapped with k_solo)",
                         "kernel_ms": kernel_ms, "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "extra": {"ops_per_step_rank0": ops_applied, "longest_doc_ops": int(counts.max()),
                      "solo_docs": info["solo"], "solo_modes": [r["mode"] for r in solo],
                      "solo_ms_last_step": info.get("solo_us", 0) / 1000.0,  # critical-path workgroups' pass
                      "kernel_ms_steps": [round(x, 1) for x in kms],
                      "solo_ms_steps": [round(x, 1) for x in solo_steps],
                      # per step: the critical wave's shader cycles (G) and its clock (cycles / 100 MHz
                      # reference ticks): a slow step with the same cycles ran at a lower clock
                      "solo_gcycles_steps": [round(c / 1e9, 4) for c, _, _ in solo_clk],
                      "solo_clock_ghz_steps": [round(c / (r / 100e6) / 1e9, 4) if r else None for c, r, _ in solo_clk],
                      # the critical wave's start after the bulk kernel's first wave (ms, 100 MHz clock)
                      "solo_start_delay_ms_steps": [round(dl / 1e5, 3) for _, _, dl in solo_clk],
                      "lds_ms_last_step": info.get("lds_ms", 0.0), "hbm_ms_last_step": info.get("hbm_ms", 0.0),
                      "solo_lead_ms": info.get("solo_lead_us", 0) / 1000.0,  # pass start -> solo start
                      "solo_tail_ms": info.get("solo_tail_us", 0) / 1000.0,  # solo end -> pass end
                      "us_per_op_critical_path": (info.get("solo_us", 0) / max(int(counts.max()), 1)) if info["solo"] else None,
                      "docs_rerun_hbm": info["spilled"], "docs_continued_hbm": info["continued"],
                      "docs_hbm_waves": info["hbm_docs"], "lds_groups": info["lds_groups"],
                      "hbm_wave_slots": info["hbm_waves"], "rows_waves_per_cu": eng.get_info("rows"),
                      "gen_s": gen_s, "summary_s": snap_host_s,
                      "snapshot_bytes": snap_bytes, "summaries_gathered": gathered, "oracle_verified_docs": nv,
                      "catchup_probe": probe},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args, argv))
    run(args)


if __name__ == "__main__":
    main()
