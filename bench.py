"""Benchmark: checkpoint actions reconciled/sec on MI355X (BASELINE.json metric), config C3 by default.

BASELINE.json's metric is quoted at 100M AddFile: configs[2] (C3) = a 100M-AddFile
64-part snappy checkpoint + 1k JSON commits (100 adds + 100 removes each, re-adds and duplicates),
read schema add(without stats) + remove. It fits one MI355X (≈40 GB of HBM), so N=1 runs all of it.

Three timed regions:
  1. `value`: one "step" = the device half of Scan.getScanFiles over inputs already resident in HBM
     (commit-tail key build + probe table, page-header parse, snappy, level/value decode of every
     projected add/remove leaf, URI-canonical key hashing, probe, selection, ScanMetrics counters).
     value = (checkpoint rows + tail rows) x steps / wall time between barriers.
  2. `end_to_end`: getScanFiles until fully consumed, as BenchmarkParallelCheckpointReading.java:
     110-139 consumes it (iterate the selected rows, sum add.size): host file read + H2D + decode +
     reconcile + D2H of the selection and add.size; actions/s = addFilesSeen / that wall time
     (BASELINE.md "Metric definitions"). `jmh_op_ms` adds the snapshot load, as the JMH op does.
  3. `snapshot_load_ms`: Table.forPath(...).getLatestSnapshot (cold and warm).

Multi-GPU (one process per GPU): C3 is one table sharded over the ranks by checkpoint row groups
(delta_amd/shard.py, strong scaling); each step ends with the exchange that assembles the result --
ScanMetrics counters and the selection bitmaps of every shard, packed on the GPU and all-gathered over
RCCL. The other configs give every rank its own table (weak scaling, no collective).
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


# BASELINE.json configs. "shared": one table sharded over the ranks by checkpoint row
# groups (strong scaling); otherwise every rank reconciles its own table (weak scaling).
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
               desc="C3: %d-AddFile 64-part snappy checkpoint (row groups sharded over the GPUs) + 1k JSON commits "
                    "(100 adds + 100 removes each, 10%% re-adds, 5%% duplicates); read schema add(no stats)+remove"),
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
                    "60%% of paths under one hot partition) row groups sharded over the GPUs; "
                    "read schema add(no stats)+remove+sidecar"),
}


def table_spec(cfg, rows, seed, compression=None):
    from delta_amd import synth
    kw = dict(cfg["spec"])
    if compression is not None:
        kw["compression"] = compression
    return synth.TableSpec(n_adds=rows, seed=seed, extra={"progress": True}, **kw)


def make_table(root, rows, seed, compression, cfg):
    from delta_amd import synth
    return synth.write_table(root, table_spec(cfg, rows, seed, compression))


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
    for e in (d if isinstance(d, list) else [d]):
        if e.get("rows") == rows and e.get("compression") == compression and kernel in e.get("kernels", {}):
            return {"bytes": e["kernels"][kernel], "source": "profiles/pmc_traffic.json (%s)" % e.get("profile", "?")}
    return None


def cpu_baseline(files, with_stats, threads, reps_single=2):
    """The oracle (plain C restatement of parquet-mr decode + URI keys + probe, oracle/dk_ref.c) on a
    bounded sample of the same workload: whole checkpoint parts of the bench table, decoded (every
    projected leaf), keyed and probed. Single thread over `reps_single` parts, then `threads` threads
    with one part each (ctypes releases the GIL inside the C decoder)."""
    import concurrent.futures as cf
    from oracle import ref
    leaves = ref.ADD_LEAVES + (["add.stats"] if with_stats else []) + [
        "remove.path", "remove.deletionVector.storageType", "remove.deletionVector.pathOrInlineDv",
        "remove.deletionVector.offset", "remove.deletionVector.sizeInBytes", "remove.deletionVector.cardinality"]

    def one(path):
        pf = ref.ParquetFile.open(path)
        cols = {leaf: pf.read(leaf) for leaf in leaves}
        ks = ref.lib().dkr_keyset_new()
        ref.probe_checkpoint(cols, pf.num_rows, ks, ref.Counters())
        ref.lib().dkr_keyset_free(ks)
        return pf.num_rows

    ref.lib()
    sample = files[:max(1, reps_single)]
    t0 = time.perf_counter()
    n1 = sum(one(p) for p in sample)
    v1 = n1 / (time.perf_counter() - t0)
    out = {"value": v1, "unit": "actions/s", "cores": 1, "kind": "port",
           "sample": "%d checkpoint part(s) of the bench table (%d rows): decode of %d leaves + URI key + probe, "
                     "oracle/dk_ref.c (CPU restatement, not DefaultEngine)" % (len(sample), n1, len(leaves))}
    if threads > 1 and len(files) > 1:
        par = [files[i % len(files)] for i in range(threads)]
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            nT = sum(ex.map(one, par))
        vT = nT / (time.perf_counter() - t0)
        out["threads"] = {"value": vT, "unit": "actions/s", "cores": threads,
                          "sample": "%d parts on %d threads (%d rows)" % (len(par), threads, nT)}
    return out


def wait_for(marker, timeout_s):
    t0 = time.time()
    while not os.path.exists(marker):
        if time.time() - t0 > timeout_s:
            raise TimeoutError("table generation did not finish: " + marker)
        time.sleep(0.5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=None, help="checkpoint adds (default: the config's)")
    ap.add_argument("--compression", default=None, help="override the config's codec")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--e2e-reps", type=int, default=2)
    ap.add_argument("--workdir", default=None)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg = CONFIGS[args.config]
    rows = args.rows or cfg["rows"]
    compression = args.compression or cfg["spec"].get("compression", "none")

    # 1. the table, before anything touches the GPU (the generator forks worker processes)
    if cfg["shared"]:
        work = args.workdir or os.path.join(tempfile.gettempdir(), "dk_bench_%s_%d_w%d" % (args.config, rows, world))
    else:
        work = args.workdir or os.path.join(tempfile.gettempdir(), "dk_bench_%s_%d_r%d" % (args.config, rows, rank))
    marker = os.path.join(work, ".ready")
    t0 = time.time()
    if os.path.exists(marker):
        log("[rank %d] reusing table in %s" % (rank, work))
    elif rank == 0 or not cfg["shared"]:
        shutil.rmtree(work, ignore_errors=True)
        info = make_table(work, rows, 20250218 + (0 if cfg["shared"] else rank), compression, cfg)
        open(marker, "w").close()
        log("[rank %d] generated %d-row table in %.1fs" % (rank, info["checkpoint_rows"], time.time() - t0))
    else:
        wait_for(marker, 1800)

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from delta_amd import kernel as K

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        return int(t.item())

    eng = K.GpuEngine(device=local if world > 1 else 0, timing=True)
    # 3. snapshot load: the first (cold: code-object load, first allocations) and the median of 5
    # warm loads, as the reference's JMH harness measures after warm-up iterations
    t0 = time.perf_counter()
    snap = K.Table.forPath(eng, work).getLatestSnapshot(eng)
    snapshot_cold_ms = (time.perf_counter() - t0) * 1e3
    warm = []
    for _ in range(5):
        t0 = time.perf_counter()
        snap = K.Table.forPath(eng, work).getLatestSnapshot(eng)
        warm.append((time.perf_counter() - t0) * 1e3)
    snapshot_ms = sorted(warm)[len(warm) // 2]
    # the same snapshot load with a Spark-style checksum file at the snapshot version (Spark writes
    # one per commit; ChecksumReader.getCRCInfo then answers the P&M pass alone)
    snapshot_crc_ms = None
    if world == 1 or not cfg["shared"]:
        from delta_amd import synth
        crc = synth.write_crc(work, snap.getVersion())
        try:
            warm_crc = []
            for _ in range(5):
                t0 = time.perf_counter()
                K.Table.forPath(eng, work).getLatestSnapshot(eng)
                warm_crc.append((time.perf_counter() - t0) * 1e3)
            snapshot_crc_ms = sorted(warm_crc)[len(warm_crc) // 2]
        finally:
            os.remove(crc)

    def build_scan(s):
        sb = s.getScanBuilder().withStats(cfg["stats"])
        if cfg["predicate"]:
            from delta_amd.expressions import Column, Literal, Predicate
            col, op, lit = cfg["predicate"]
            sb = sb.withFilter(Predicate(op, Column(col), Literal.ofLong(lit)))
        if cfg["shared"] and world > 1:
            sb = sb.withShard(world, rank)
        return sb.build()

    # 1. device steps
    scan = build_scan(snap)
    t0 = time.perf_counter()
    scan.prepare(eng)
    prepare_s = time.perf_counter() - t0
    n_ckpt_rows = sum(scan.ckpt.num_rows(i) for i in range(len(scan.ckpt_files))) if scan.ckpt else 0
    n_tail = int(scan.tail.rows)
    bytes_read, bytes_written = scan.ckpt.traffic() if scan.ckpt else (0, 0)
    merged = None

    def step():
        nonlocal merged
        scan.run()
        scan.sync()
        if dist is not None and cfg["shared"]:
            # the exchange: ScanMetrics counters and every shard's selection bitmap (packed on the
            # GPU) all-gathered over RCCL; row data stays on the GPU that decoded it
            from delta_amd import shard
            merged = shard.gather_selections(shard.scan_units(scan, device_bits=True), scan.tail_metrics.as_tuple(),
                                             scan.ckpt_metrics.as_tuple(), device="cuda")

    for _ in range(args.warmup):
        step()
    counters = merged[0] if merged else scan.metrics.as_tuple()
    barrier()
    stats0 = scan.kernel_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    stats1 = scan.kernel_stats()

    # per-kernel averages over the timed steps only
    kern = {}
    for name, (avg1, c1) in stats1.items():
        avg0, c0 = stats0.get(name, (0.0, 0))
        if c1 > c0:
            kern[name] = (avg1 * c1 - avg0 * c0) / (c1 - c0)
    step_us = kern.pop("step_total", None)
    if cfg["shared"]:
        units = sum_over_ranks(n_ckpt_rows) + n_tail      # every rank replays the whole tail
    else:
        units = (n_ckpt_rows + n_tail) * world
    value = units * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    dom = max(kern.items(), key=lambda kv: kv[1]) if kern else ("none", 0.0)
    step_bytes = bytes_read + bytes_written
    step_gbs = step_bytes / (step_us * 1e-6) / 1e9 if step_us else None
    # roofline of the dominant kernel that has a byte model (dk_parquet_kernel_traffic):
    # algorithmic bytes of one launch / its average launch time (HIP events, engine stream)
    modelled = [k for k in ("k_snap_frag", "k_tile_decode", "k_string_copy") if k in kern]
    rk = max(modelled, key=lambda k: kern[k]) if modelled else None
    k_read, k_written = scan.ckpt.kernel_traffic(rk) if rk else (0, 0)
    k_bytes = k_read + k_written
    achieved = k_bytes / (kern[rk] * 1e-6) / 1e9 if rk else None
    pmc = pmc_traffic(rk, n_ckpt_rows, compression) if rk else None
    ckpt_files = list(scan.ckpt_files)
    scan.close()

    # 2. end to end: getScanFiles until consumed (the JMH consumer sums add.size of selected rows)
    e2e = None
    if not args.no_e2e:
        runs = []
        for _ in range(args.e2e_reps):
            barrier()
            t_a = time.perf_counter()
            s2 = K.Table.forPath(eng, work).getLatestSnapshot(eng)
            t_b = time.perf_counter()
            sc2 = build_scan(s2)
            size_sum, n_sel = 0, 0
            t_p = t_r = None
            it = sc2.getScanFiles(eng)      # prepare (host read + H2D) + device step + counters
            t_r = time.perf_counter()
            import numpy as np
            for b in it:
                # the JMH consumer (BenchmarkParallelCheckpointReading.java:124-135): sum add.size
                # over the selected rows
                col = b.data["add.size"]
                v = col.fixed.view("<i8")
                if b.selection is None:
                    size_sum += int(v.sum())
                    n_sel += b.size
                else:
                    size_sum += int(np.add.reduce(v, where=b.selection))
                    n_sel += int(np.count_nonzero(b.selection))
            t_c = time.perf_counter()
            seen = sc2.metrics.addFilesSeen
            prep_ms = {k: round(v, 2) for k, v in sc2.prepare_ms.items()}
            sc2.close()
            runs.append((t_c - t_b, t_b - t_a, seen, n_sel, size_sum, t_r - t_b, t_c - t_r))
        gsf_s, snap_s, seen, n_sel, size_sum, open_run_s, consume_s = min(runs)
        gsf_s = max_over_ranks(gsf_s)
        snap_s = max_over_ranks(snap_s)
        seen_all = sum_over_ranks(seen) - (world - 1) * (n_tail and scan.tail_metrics.addFilesSeen) \
            if cfg["shared"] else sum_over_ranks(seen)
        e2e = {"getScanFiles_ms": gsf_s * 1e3, "snapshot_load_ms": snap_s * 1e3,
               "jmh_op_ms": (gsf_s + snap_s) * 1e3,
               "actions_per_s": seen_all / gsf_s, "jmh_op_actions_per_s": seen_all / (gsf_s + snap_s),
               "addFilesSeen": seen_all, "selected_rows_rank0": n_sel, "size_sum_rank0": size_sum,
               "phases_ms": {"prepare_and_device_step": open_run_s * 1e3, "consume": consume_s * 1e3,
                             "prepare": dict(prep_ms)},
               "reps": args.e2e_reps,
               "includes": "host read of the projected column chunks + H2D + device decode/reconcile + "
                           "D2H of selection and add.size + host sum over selected rows"}

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
                   "parallelism": ("strong: checkpoint row groups in %d contiguous runs (one per GPU), tail on every "
                                   "GPU, counters + selection bitmaps all-gathered over RCCL each step" % world
                                   if cfg["shared"] else "weak: one table per GPU"),
                   "checkpoint_rows_per_gpu": n_ckpt_rows, "json_tail_rows": n_tail,
                   "checkpoint_files_per_gpu": len(ckpt_files)},
        "snapshot_load_ms": snapshot_ms,
        "snapshot_load_cold_ms": snapshot_cold_ms,
        "snapshot_load_with_crc_ms": snapshot_crc_ms,
        "snapshot_load_phases_ms": {k: round(v, 3) for k, v in snap.load_ms.items()},
        "end_to_end": e2e,
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
        result["cpu_baseline"] = cpu_baseline(ckpt_files, cfg["stats"], args.cpu_threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.barrier()          # every rank is done with the shared table
    if not args.workdir and (rank == 0 or not cfg["shared"]):
        shutil.rmtree(work, ignore_errors=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
