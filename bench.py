"""Benchmark: checkpoint actions reconciled/sec on MI355X (BASELINE.json metric), config C2.

One "step" = the device half of Scan.getScanFiles over one checkpoint already resident in HBM:
commit-tail key build + probe table, checkpoint page-header parse, level/value decode of every
projected add/remove leaf, URI-canonical key hashing of every add row, probe, selection and
ScanMetrics counters (delta_amd.kernel.GpuScan.run + sync).

Workload (configs[1]): 10M-AddFile single-part checkpoint with 2-key
partitionValues maps and stats_parsed (read schema: add without stats + remove), plus a 100-commit
JSON tail (50 adds + 50 removes each). Synthetic, seed 20250218.

Multi-GPU (one process per GPU, torch.distributed over RCCL for the barrier/max only): each rank
owns one checkpoint part of the same size (part i -> rank i) and replicates the commit tail; the
path has no data exchange, so scaling is weak and no collective runs inside the timed region.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, Chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs. "shared": one table sharded over the ranks by checkpoint
# file (strong scaling); otherwise every rank reconciles its own table (weak scaling).
CONFIGS = {
    "c1": dict(rows=1_000_000, shared=False, stats=False, predicate=None,
               spec=dict(pv_keys=1, n_commits=100, adds_per_commit=50, removes_per_commit=50),
               desc="C1: %d-AddFile single-part uncompressed checkpoint per GPU, 100-commit JSON tail; "
                    "read schema add(no stats)+remove"),
    "c2": dict(rows=10_000_000, shared=False, stats=False, predicate=None,
               spec=dict(pv_keys=2, with_stats_parsed=True, n_commits=100, adds_per_commit=50, removes_per_commit=50),
               desc="C2: %d-AddFile single-part checkpoint per GPU, 2-key partitionValues, stats_parsed present, "
                    "100-commit JSON tail; read schema add(no stats)+remove"),
    "c3": dict(rows=100_000_000, shared=True, stats=False, predicate=None,
               spec=dict(n_parts=64, compression="snappy", n_commits=1000, adds_per_commit=100,
                         removes_per_commit=100, readd_frac=0.1, dup_frac=0.05),
               desc="C3: %d-AddFile 64-part snappy checkpoint sharded over the GPUs by part, 1k commits "
                    "(100 adds + 100 removes each); read schema add(no stats)+remove"),
    "c4": dict(rows=50_000_000, shared=False, stats=True, predicate=("id", ">", 25_000_000),
               spec=dict(n_parts=8, dv_frac=0.3, with_stats=True, n_commits=100, adds_per_commit=50,
                         removes_per_commit=50),
               desc="C4: %d-AddFile 8-part checkpoint per GPU, 30%% with deletion vectors, predicate id > 25000000 "
                    "over stats; read schema add(with stats)+remove"),
    "c5": dict(rows=10_000_000, shared=True, stats=False, predicate=None,
               spec=dict(n_parts=16, v2_sidecars=16, compression="snappy", data_page_version="2.0",
                         delta_binary_packed=True, hot_frac=0.6, n_commits=100, adds_per_commit=50,
                         removes_per_commit=50),
               desc="C5: %d-AddFile V2 checkpoint (manifest + 16 sidecars, snappy, v2 pages, DELTA_BINARY_PACKED, "
                    "60%% of paths under one hot partition) sharded over the GPUs by file; "
                    "read schema add(no stats)+remove+sidecar"),
}


def table_spec(cfg, rows, seed, compression=None):
    from delta_amd import synth
    kw = dict(cfg["spec"])
    if compression is not None:
        kw["compression"] = compression
    return synth.TableSpec(n_adds=rows, seed=seed, extra={"progress": True}, **kw)


def make_table(root, rows, seed, compression, cfg=None):
    from delta_amd import synth
    return synth.write_table(root, table_spec(cfg or CONFIGS["c2"], rows, seed, compression))


def pmc_traffic(kernel, rows, compression):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of the same workload
    (tools/pmc.sh + tools/pmc_summary.py --json: separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE
    doubled for gfx950's half-count of wide loads, KB -> bytes), or None when no profile matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("rows") != rows or d.get("compression") != compression or kernel not in d.get("kernels", {}):
        return None
    return {"bytes": d["kernels"][kernel], "source": "profiles/pmc_traffic.json (%s)" % d.get("profile", "?")}


def cpu_baseline(rows, reps, seed, compression, cfg_name="c2"):
    """Oracle (plain C restatement, single thread) on a bounded sample of the same workload: one
    single-part checkpoint with the config's encodings."""
    from oracle import ref
    d = tempfile.mkdtemp(prefix="dk_cpu_")
    try:
        cfg = dict(CONFIGS[cfg_name])
        cfg["spec"] = dict(cfg["spec"], n_parts=1, v2_sidecars=0)
        make_table(d, rows, seed + 99, compression, cfg)
        seg = ref.load_log_segment(d)
        path = seg.checkpoints[0].path
        leaves = ref.ADD_LEAVES + (["add.stats"] if cfg["stats"] else []) + ["remove.path", "remove.deletionVector.storageType",
                                   "remove.deletionVector.pathOrInlineDv", "remove.deletionVector.offset",
                                   "remove.deletionVector.sizeInBytes", "remove.deletionVector.cardinality"]
        with open(path, "rb") as f:
            data = f.read()
        total_rows, t_total = 0, 0.0
        for _ in range(reps):
            t0 = time.perf_counter()
            pf = ref.ParquetFile(data)
            cols = {leaf: pf.read(leaf) for leaf in leaves}
            ks = ref.lib().dkr_keyset_new()
            ref.probe_checkpoint(cols, pf.num_rows, ks, ref.Counters())
            ref.lib().dkr_keyset_free(ks)
            t_total += time.perf_counter() - t0
            total_rows += pf.num_rows
        return {"value": total_rows / t_total, "unit": "actions/s", "cores": 1, "kind": "port",
                "sample": "%d x %d-row %s-shaped checkpoint, decode (%d leaves) + key + probe, oracle/dk_ref.c"
                          % (reps, rows, cfg_name.upper(), len(leaves))}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=None, help="checkpoint adds (default: the config's)")
    ap.add_argument("--compression", default=None, help="override the config's codec")
    ap.add_argument("--cpu-rows", type=int, default=1_000_000)
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workdir", default=None)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from delta_amd import kernel as K

    cfg = CONFIGS[args.config]
    rows = args.rows or cfg["rows"]
    compression = args.compression or cfg["spec"].get("compression", "none")
    if cfg["shared"]:
        # one table for all ranks: rank 0 writes it, the others wait at the barrier
        work = args.workdir or os.path.join(tempfile.gettempdir(), "dk_bench_%s_%d" % (args.config, rows))
    else:
        work = args.workdir or tempfile.mkdtemp(prefix="dk_bench_r%d_" % rank)
    t0 = time.time()
    if args.workdir and os.path.isdir(os.path.join(work, "_delta_log")):
        log("[rank %d] reusing table in %s" % (rank, work))
    elif rank == 0 or not cfg["shared"]:
        shutil.rmtree(work, ignore_errors=True)
        info = make_table(work, rows, 20250218 + (0 if cfg["shared"] else rank), compression, cfg)
        log("[rank %d] generated %d-row table in %.1fs" % (rank, info["checkpoint_rows"], time.time() - t0))
    if dist is not None and cfg["shared"]:
        dist.barrier()

    eng = K.GpuEngine(device=local if world > 1 else 0, timing=True)
    # snapshot load: the first (cold: code-object load, first allocations) and the median of 5 warm
    # loads, as the reference's JMH harness measures after warm-up iterations
    t0 = time.perf_counter()
    snap = K.Table.forPath(eng, work).getLatestSnapshot(eng)
    snapshot_cold_ms = (time.perf_counter() - t0) * 1e3
    warm = []
    for _ in range(5):
        t0 = time.perf_counter()
        snap = K.Table.forPath(eng, work).getLatestSnapshot(eng)
        warm.append((time.perf_counter() - t0) * 1e3)
    snapshot_ms = sorted(warm)[len(warm) // 2]
    sb = snap.getScanBuilder().withStats(cfg["stats"])
    if cfg["predicate"]:
        from delta_amd.expressions import Column, Literal, Predicate
        col, op, lit = cfg["predicate"]
        sb = sb.withFilter(Predicate(op, Column(col), Literal.ofLong(lit)))
    if cfg["shared"] and world > 1:
        sb = sb.withShard(world, rank)
    scan = sb.build()
    t0 = time.perf_counter()
    scan.prepare(eng)
    prepare_s = time.perf_counter() - t0
    n_ckpt_rows = sum(scan.ckpt.num_rows(i) for i in range(len(scan.ckpt_files)))
    n_tail = int(scan.tail.rows)
    bytes_read, bytes_written = scan.ckpt.traffic()

    def barrier():
        if dist is not None:
            dist.barrier()
            import torch
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        scan.run()
        scan.sync()
    counters = scan.metrics.as_tuple()
    # reset kernel timers: only the timed steps count
    barrier()
    stats0 = scan.kernel_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        scan.run()
        scan.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    stats1 = scan.kernel_stats()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel averages over the timed steps only
    kern = {}
    for name, (avg1, c1) in stats1.items():
        avg0, c0 = stats0.get(name, (0.0, 0))
        if c1 > c0:
            kern[name] = (avg1 * c1 - avg0 * c0) / (c1 - c0)
    step_us = kern.pop("step_total", None)
    if cfg["shared"]:
        # every rank replays the whole tail; the checkpoint rows are split among the ranks
        tot = n_ckpt_rows
        if dist is not None:
            import torch
            tt = torch.tensor([n_ckpt_rows], dtype=torch.int64, device="cuda")
            dist.all_reduce(tt)
            tot = int(tt.item())
        units = tot + n_tail
    else:
        units = (n_ckpt_rows + n_tail) * world
    value = units * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    dom = max(kern.items(), key=lambda kv: kv[1]) if kern else ("none", 0.0)
    step_bytes = bytes_read + bytes_written
    step_gbs = step_bytes / (step_us * 1e-6) / 1e9 if step_us else None
    # roofline of the dominant decode kernel: algorithmic bytes of one launch (byte model in
    # dk_parquet_kernel_traffic) / its average launch time (HIP events, engine stream)
    modelled = [k for k in ("k_tile_decode", "k_string_copy") if k in kern]
    rk = max(modelled, key=lambda k: kern[k]) if modelled else None
    k_read, k_written = scan.ckpt.kernel_traffic(rk) if rk else (0, 0)
    k_bytes = k_read + k_written
    achieved = k_bytes / (kern[rk] * 1e-6) / 1e9 if rk else None
    pmc = pmc_traffic(rk, n_ckpt_rows, compression) if rk else None

    result = {
        "metric": "checkpoint actions reconciled/sec (node) + snapshot load ms, 100M AddFile",
        "value": value,
        "unit": "actions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if cfg["shared"] else "weak",
        "vs_baseline": None,
        "dtype": "u8/int64",
        "data": "synthetic (seed 20250218; delta_amd/synth.py)",
        "config": {"workload": cfg["desc"] % rows, "name": args.config,
                   "compression": compression,
                   "parallelism": ("strong: checkpoint files round-robin over %d GPU(s), tail on every GPU" % world
                                   if cfg["shared"] else "weak: one checkpoint per GPU"),
                   "checkpoint_rows_per_gpu": n_ckpt_rows, "json_tail_rows": n_tail,
                   "checkpoint_files_per_gpu": len(scan.ckpt_files)},
        "snapshot_load_ms": snapshot_ms,
        "snapshot_load_cold_ms": snapshot_cold_ms,
        "snapshot_load_phases_ms": {k: round(v, 3) for k, v in snap.load_ms.items()},
        "prepare_s": prepare_s,
        "counters": counters,
        "kernels_us": {k: round(v, 2) for k, v in sorted(kern.items(), key=lambda kv: -kv[1])},
        "roofline": {"bound": "hbm", "kernel": rk, "kernel_us": kern.get(rk),
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": pmc["bytes"] if pmc else None,
                     "traffic_source": pmc["source"] if pmc else None,
                     "algorithmic_bytes": k_bytes, "algorithmic_read": k_read, "algorithmic_written": k_written,
                     "dominant_kernel": dom[0], "dominant_kernel_us": dom[1],
                     "step": {"device_us": step_us, "algorithmic_bytes": step_bytes, "bytes_read": bytes_read,
                              "bytes_written": bytes_written, "achieved_gbs": step_gbs,
                              "frac": (step_gbs / HBM_PEAK_GBS) if step_gbs else None}},
    }
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        result["cpu_baseline"] = cpu_baseline(args.cpu_rows, args.cpu_reps, 20250218, compression, args.config)
    if rank == 0:
        print(json.dumps(result), flush=True)
    scan.close()
    eng.close()
    if dist is not None and cfg["shared"]:
        dist.barrier()          # every rank is done with the shared table
    if not args.workdir and (rank == 0 or not cfg["shared"]):
        shutil.rmtree(work, ignore_errors=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
