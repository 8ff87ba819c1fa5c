"""Benchmark: checkpoint actions reconciled/sec on MI355X (BASELINE.json metric), config C3 by default.

BASELINE.json's metric is quoted at 100M AddFile: configs[2] (C3) = a 100M-AddFile
64-part snappy checkpoint + 1k JSON commits (100 adds + 100 removes each, re-adds and duplicates),
read schema add(without stats) + remove. It fits one MI355X, so N=1 runs all of it.

`value` is BASELINE.md's metric ("Metric definitions"): actions/s = ScanMetrics.numAddFilesSeen ÷
getScanFiles wall time until fully consumed. One timed "step" = one getScanFiles over the table, as
BenchmarkParallelCheckpointReading.java:110-139 runs it: a fresh scan on the loaded snapshot, host
read of the projected column chunks, H2D, device decode + reconcile, D2H of the selection and of
add.size, and the consumer summing add.size over the selected rows. The other regions are reported
beside it:
  device_step       the device half of getScanFiles over inputs already resident in HBM (commit-tail
                    keys + table, page headers, snappy, level/value decode of every projected leaf,
                    URI-canonical key hashes, probe, selection, counters); the roofline is measured
                    here, per kernel, with HIP events on the replay stream;
  snapshot_load_ms  Table.forPath(...).getLatestSnapshot (cold, warm, and with a .crc).

Multi-GPU, one process per GPU over RCCL: `python bench.py --gpus N` starts N ranks itself (a
parent that never touches the GPU spawns N children with RANK / LOCAL_RANK / WORLD_SIZE), or the
driver's `torch.distributed.run --nproc-per-node N bench.py --gpus N` does. C3 is ONE table whose
checkpoint row groups are cut into N contiguous runs (delta_amd/shard.py). With the default
`--exchange owner`, each rank parses only the commit files j = rank (mod N), the keys are owned by
hash, and three RCCL all-to-alls resolve every commit-tail action and every checkpoint row at its
key's owner (the protocol and its RCCL collectives inside libdkgpu: dk_replay_owner_run over
shard.OwnerComm.rccl; `owner_exchange_ms`); each rank consumes its own scan files and
counters and consumer sums are all-reduced. `--exchange allgather` keeps the whole commit tail on
every rank and ends the device step with one RCCL all-gather of counters and selection bitmaps
(shard.SelectionExchange, `exchange_ms`).

`--dry-run`: no GPU; the launcher, the row-group planning and the exchange run over gloo on the CPU
with placeholder selections (tests/test_bench_launcher.py).
"""
import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONSUME_PROFILE = os.environ.get("DK_CONSUME_PROFILE", "0") not in ("", "0")   # consume-phase split
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, Chip-level parameters)
METRIC = "checkpoint actions reconciled/sec (node) + snapshot load ms, 100M AddFile"
REMOVE_LEAVES = ["remove.path", "remove.deletionVector.storageType", "remove.deletionVector.pathOrInlineDv",
                 "remove.deletionVector.offset", "remove.deletionVector.sizeInBytes",
                 "remove.deletionVector.cardinality"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs. "shared": one table sharded over the ranks by checkpoint row
# groups (strong scaling); otherwise every rank reconciles its own table (weak scaling).
CONFIGS = {
    "c1": dict(rows=1_000_000, shared=False, stats=False, predicate=None,
               spec=dict(pv_keys=1, n_commits=100, adds_per_commit=50, removes_per_commit=50),
               desc="C1: %d-AddFile single-part uncompressed checkpoint per GPU, 100-commit JSON tail; "
                    "read schema add(no stats)+remove"),
    "c2": dict(rows=10_000_000, shared=False, stats=True, predicate=None,
               spec=dict(pv_keys=2, compression="snappy", with_stats=True, with_stats_parsed=True, n_commits=100,
                         adds_per_commit=50, removes_per_commit=50),
               desc="C2: %d-AddFile single-part snappy checkpoint per GPU, 2-key partitionValues, stats JSON + "
                    "stats_parsed, 100-commit JSON tail; read schema add(with stats)+remove (C2b)"),
    "c2a": dict(rows=10_000_000, shared=False, stats=False, predicate=None,
                spec=dict(pv_keys=2, compression="snappy", with_stats=True, with_stats_parsed=True, n_commits=100,
                          adds_per_commit=50, removes_per_commit=50),
                desc="C2a: %d-AddFile single-part snappy checkpoint per GPU, 2-key partitionValues, stats JSON + "
                     "stats_parsed, 100-commit JSON tail; read schema add(no stats)+remove"),
    "c3": dict(rows=100_000_000, shared=True, stats=False, predicate=None,
               spec=dict(n_parts=64, compression="snappy", n_commits=1000, adds_per_commit=100,
                         removes_per_commit=100, readd_frac=0.1, dup_frac=0.05),
               desc="C3: %d-AddFile 64-part snappy checkpoint (row groups sharded over the GPUs) + 1k JSON commits "
                    "(100 adds + 100 removes each, 10%% re-adds, 5%% duplicates); read schema add(no stats)+remove"),
    "c4": dict(rows=50_000_000, shared=True, stats=True, predicate=("id", ">", 25_000_000),
               spec=dict(n_parts=8, dv_frac=0.3, with_stats=True, with_stats_parsed=True, n_commits=100,
                         adds_per_commit=50, removes_per_commit=50),
               desc="C4: %d-AddFile 8-part checkpoint (row groups sharded over the GPUs), 30%% with deletion "
                    "vectors, predicate id > 25000000 over stats_parsed; read schema add(with stats)+remove"),
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
    (tools/pmc.sh + tools/pmc_summary.py --json: separate FETCH_SIZE / WRITE_SIZE passes, KB -> bytes,
    FETCH_SIZE doubled only for kernels calibrated as 16 B/lane streaming readers), or None."""
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


# ------------------------------------------------------------------------------------------------
# launcher: N ranks from one command, before anything touches the GPU
# ------------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv):
    """Parent of an N-rank run: starts N fresh child processes of this script (one per GPU) with
    the torch.distributed environment and returns the worst exit code. It imports nothing that
    initialises HIP; children are started, never exec'd into."""
    n = args.gpus
    env0 = dict(os.environ)
    env0.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), DK_BENCH_CHILD="1")
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0:
                    rc = rc or c
                    for q in procs:            # one rank failed: the others would wait forever
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            p.kill()
    return rc


# ------------------------------------------------------------------------------------------------
# CPU baseline + full-size parity (the oracle: test infrastructure, used here only as the checker
# and the reported CPU baseline)
# ------------------------------------------------------------------------------------------------
def oracle_skipping(work, cfg):
    """The oracle's own data-skipping predicate for the config's filter (oracle/skipping_filter.py
    restates constructDataSkippingFilter; the product planner is not used) and its stats types."""
    if not cfg["predicate"]:
        return None
    from delta_amd.expressions import Column, Literal, Predicate
    from oracle import ref
    from oracle import skipping_filter as osf
    _, meta, _ = ref.load_protocol_metadata(work)
    col, op, lit = cfg["predicate"]
    pf, data = osf.split(Predicate(op, Column(col), Literal.ofLong(lit)), meta["partitionColumns"])
    if pf is not None:
        raise SystemExit("bench.py: the CPU baseline restates data-skipping filters only")
    schema = osf.StatsSchema(meta["schemaString"], meta["partitionColumns"])
    node = osf.build(data, schema) if data is not None else None
    if node is None:
        return None
    osf.check(node, schema)
    return node, osf.stat_types(node, schema)


def _mask_rows(sel, want):
    """Indices of the rows whose selection bit is `want`, for a mask where they are rare: a scan of
    the mask 8 rows per uint64 word finds the words holding any, then only those words' rows are
    looked at (np.flatnonzero over the whole mask costs more than the sum it feeds)."""
    import numpy as np
    n = len(sel)
    w = n // 8 * 8
    words = np.ascontiguousarray(sel[:w]).view(np.uint8).view(np.uint64)
    full = np.uint64(0x0101010101010101 if not want else 0)    # a word of 8 rows with no `want` bit
    hit = np.flatnonzero(words != full)
    idx = (hit[:, None] * 8 + np.arange(8)).ravel()
    idx = idx[sel[idx] == want]
    rest = np.flatnonzero(sel[w:] == want) + w
    return np.concatenate([idx, rest]) if len(rest) else idx


def masked_sum(v, sel):
    """(sum(v[sel]), count of selected rows) for the JMH-shaped consumer, without numpy's branchy masked reduction on
    irregular selections (`sum(where=)` runs 6-8x slower on a 50 % / 70 % random mask than on a
    near-uniform one): near-uniform masks keep it, irregular ones take a branch-free blocked
    multiply-add (the same sum)."""
    import numpy as np
    n = len(v)
    k = int(np.count_nonzero(sel))
    if k == n:
        return int(v.sum()), k
    if k == 0:
        return 0, 0
    if n - k < n // 16:                             # nearly all selected: the whole sum minus the few
        return int(v.sum()) - int(v[_mask_rows(sel, False)].sum()), k
    if k < n // 16:                                 # nearly none selected: the few
        return int(v[_mask_rows(sel, True)].sum()), k
    tot, B = 0, 1 << 16
    for i in range(0, n, B):
        tot += int(np.dot(v[i:i + B], sel[i:i + B].astype(np.int64)))
    return tot, k


def cpu_share():
    """CPUs this process may run on (sched_getaffinity, i.e. `nproc`) and the cgroup CPU quota, if
    any (cpu.max): the GPU box shows the whole machine's cores but grants one GPU's share."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return aff, quota


def cpu_baseline(work, files, cfg, threads, got=None, single_rows=12_500_000):
    """The oracle (oracle/dk_ref.c: parquet-mr decode of every projected leaf + java.net.URI keys +
    probe + data skipping over add.stats; oracle/ref.py: commit-tail replay) on the bench table.

    1 thread: whole checkpoint parts (up to 8, at most ~`single_rows` rows) decoded, probed against
    the real tail key set and, with a filter, skipped.
    `threads` threads: the WHOLE table (tail + every part, runs of row groups per task) -- this run
    is also the full-size parity check: its five counters and every checkpoint row's selection bit
    (after data skipping) are compared with the GPU's (`got`)."""
    import numpy as np
    from oracle import ref
    ref.lib()
    with_stats = cfg["stats"]
    skipping = oracle_skipping(work, cfg)
    out = {"unit": "actions/s", "kind": "port"}
    leaves = ref.ADD_LEAVES + (["add.stats"] if with_stats or skipping else []) + REMOVE_LEAVES
    seg = ref.load_log_segment(work)
    t0 = time.perf_counter()
    keyset_res = ref.replay_tail_keyset(work, with_stats=with_stats or skipping is not None)
    tail_s = time.perf_counter() - t0

    def one(path):
        pf = ref.ParquetFile.open(path)
        cols = {leaf: pf.read(leaf) for leaf in leaves}
        sel = ref.probe_checkpoint(cols, pf.num_rows, keyset_res, ref.Counters())
        if skipping is not None:
            from oracle import skipping as sk
            sk.apply_to_column(cols.get(ref.STATS_LEAF), sel, *skipping)
        return pf.num_rows

    sample, n_rows = [], 0
    for p in files:
        if len(sample) >= 8 or (sample and n_rows >= single_rows):
            break
        sample.append(p)
        n_rows += ref.ParquetFile.open(p).num_rows
    t0 = time.perf_counter()
    n1 = sum(one(p) for p in sample)
    v1 = n1 / (time.perf_counter() - t0)
    ref.lib().dkr_keyset_free(keyset_res)
    out.update(value=v1, cores=1,
               sample="%d of %d checkpoint part(s) of the bench table (%d rows): decode of %d leaves + URI key + "
                      "probe against the commit-tail key sets%s, oracle/dk_ref.c (CPU restatement, not "
                      "DefaultEngine); the commit-tail replay (Python, %d commits) took %.2f s more"
                      % (len(sample), len(files), n1, len(leaves),
                         " + data skipping over add.stats (oracle/dk_skip.c)" if skipping else "",
                         len(seg.deltas), tail_s))
    if threads > 1:
        t0 = time.perf_counter()
        res = ref.replay(work, with_stats=with_stats, threads=threads, keep_cols=False,
                         extra_leaves=REMOVE_LEAVES, skipping=skipping)
        dt = time.perf_counter() - t0
        seen = res.counters.addFilesSeen
        used = min(threads, getattr(res, "pool_tasks", threads))
        full = {"value": seen / dt, "unit": "actions/s", "cores": used, "seconds": dt,
                "sample": "the whole table: commit-tail replay (Python, serial) + %d checkpoint files decoded, probed"
                          "%s in %d tasks (runs of row groups) on %d threads"
                          % (len(res.checkpoint), " and skipped" if skipping else "",
                             getattr(res, "pool_tasks", 0), used)}
        out["threads"] = full
        if got is not None:
            counters, tail_paths, bits = got
            oc = res.counters.as_tuple()
            bad = [i for i, b in enumerate(res.checkpoint)
                   if not np.array_equal(np.packbits(b.selected.astype(bool), bitorder="little"), bits[i])]
            otail = [a["path"] for a in res.json_rows]
            out["parity"] = {"counters_gpu": list(counters), "counters_oracle": list(oc),
                             "counters_match": tuple(counters) == tuple(oc),
                             "tail_selected_match": tail_paths == otail, "tail_selected": len(otail),
                             "checkpoint_files": len(res.checkpoint),
                             "checkpoint_rows": int(sum(b.n_rows for b in res.checkpoint)),
                             "checkpoint_bits_match": not bad and len(bits) == len(res.checkpoint),
                             "mismatched_files": bad[:8]}
    return out


def wait_for(marker, timeout_s):
    t0 = time.time()
    while not os.path.exists(marker):
        if time.time() - t0 > timeout_s:
            raise TimeoutError("table generation did not finish: " + marker)
        time.sleep(0.5)


def dry_run(args, cfg, work, world, rank):
    """CPU rehearsal of the multi-rank path over gloo: launcher, planning (shard.plan_units over the
    checkpoint footers, read by the product's host footer parser) and the one-collective exchange with
    placeholder selections (bit = row parity). Rank 0 checks every checkpoint row came back exactly
    once, in replay order."""
    import numpy as np
    import torch.distributed as dist
    from delta_amd import kernel as K
    from delta_amd import shard
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    seg = K.build_log_segment(work)
    files = [f.path for f in sorted(seg.checkpoints, key=lambda f: os.path.basename(f.path), reverse=True)]
    rg = [K.row_group_rows(f) for f in files]
    units = shard.plan_units(rg, world, rank)
    meta = shard.unit_layout(rg, units)
    ex = shard.SelectionExchange(meta)

    def write_bits(i, dst):
        f, r0, n = meta[i]
        rows = np.arange(r0, r0 + n)
        dst.copy_(__import__("torch").from_numpy(np.packbits((rows % 2 == 0), bitorder="little")))

    t0 = time.perf_counter()
    res = ex.exchange([0] * 5, [sum(n for _, _, n in meta)] + [0] * 4, write_bits)
    dt = time.perf_counter() - t0
    ok = None
    if rank == 0:
        counters, sels = res
        total = sum(sum(r) for r in rg)
        cover = {}
        for f, r0, n, bits in sels:
            want = np.packbits(np.arange(r0, r0 + n) % 2 == 0, bitorder="little")
            assert np.array_equal(bits, want), (f, r0)
            cover.setdefault(f, []).append((r0, n))
        for f, rs in cover.items():
            rs.sort()
            assert rs[0][0] == 0 and all(a[0] + a[1] == b[0] for a, b in zip(rs, rs[1:])), f
            assert rs[-1][0] + rs[-1][1] == sum(rg[f])
        ok = counters[0] == total and len(cover) == len(files)
        print(json.dumps({"metric": METRIC, "value": None, "unit": "actions/s", "n_gpus": world,
                          "dry_run": True, "backend": dist.get_backend(), "ranks": dist.get_world_size(),
                          "checkpoint_files": len(files), "checkpoint_rows": total, "units": len(sels),
                          "exchange_ms": dt * 1e3, "ok": bool(ok)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if (rank != 0 or ok) else 1


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=None, help="checkpoint adds (default: the config's)")
    ap.add_argument("--compression", default=None, help="override the config's codec")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the whole-table CPU baseline (default: nproc, capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--full-row-steps", type=int, default=2,
                    help="timed steps of the full-row consumer reported beside the headline (0: skip)")
    ap.add_argument("--device-steps", type=int, default=None, help="timed device-only steps (default: --steps)")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo rehearsal of launcher + planning + exchange")
    ap.add_argument("--exchange", default="owner", choices=["owner", "allgather", "alltoall"],
                    help="multi-GPU: owner (default) = each rank parses 1/N of the commit files and the key table "
                         "is partitioned by key hash: commit-tail actions, then every checkpoint row's key hash, "
                         "then the hash hits' keys go to their owner over RCCL all-to-all and are answered exactly "
                         "(delta-spark's repartition by path); allgather = every rank parses the whole commit tail "
                         "and probes its rows against its own copy of the key table, selection bitmaps all-gathered; "
                         "alltoall = allgather's tail, checkpoint rows pre-filtered by their path-hash owner "
                         "(DESIGN.md §6)")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--jmh-ops", type=int, default=3,
                    help="timed JMH-shaped operations (engine + forPath + snapshot + getScanFiles consumed)")
    args = ap.parse_args(argv)

    env_world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if args.gpus is None:
        args.gpus = env_world or 1
    if args.gpus > 1 and env_world == 0:
        return launch(args, argv)               # the parent: spawn one child per GPU, touch nothing
    world = env_world or 1
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
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

    if args.dry_run:
        rc = dry_run(args, cfg, work, world, rank)
        if not args.workdir and rank == 0:
            shutil.rmtree(work, ignore_errors=True)
        return rc

    import numpy as np
    dist = None
    backend = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        backend = dist.get_backend()
        if dist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: RCCL world is %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))

    from delta_amd import kernel as K

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    def reduce_over_ranks(xs, op):
        if dist is None:
            return list(xs)
        import torch
        t = torch.tensor(list(xs), dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=op)
        return [float(v) for v in t.cpu().tolist()]

    def max_over_ranks(x):
        return reduce_over_ranks([x], dist.ReduceOp.MAX if dist else None)[0]

    def sum_over_ranks(xs):
        return [int(round(v)) for v in reduce_over_ranks(xs, dist.ReduceOp.SUM if dist else None)]

    t0 = time.perf_counter()
    eng = K.GpuEngine(device=local if world > 1 else 0, timing=True)
    engine_create_ms = (time.perf_counter() - t0) * 1e3     # includes the code-object / allocator warm-up

    # ---- region 3: snapshot load (cold: code-object load + first allocations; warm: median of 5) ----
    t0 = time.perf_counter()
    snap = K.Table.forPath(eng, work).getLatestSnapshot(eng)
    snapshot_cold_ms = (time.perf_counter() - t0) * 1e3
    cold_phases = {k: round(v, 3) for k, v in snap.load_ms.items()}
    warm = []
    for _ in range(5):
        t0 = time.perf_counter()
        snap = K.Table.forPath(eng, work).getLatestSnapshot(eng)
        warm.append((time.perf_counter() - t0) * 1e3)
    snapshot_ms = sorted(warm)[len(warm) // 2]
    snapshot_crc_ms = None
    if rank == 0 and (world == 1 or not cfg["shared"]):
        # with a Spark-style checksum file at the snapshot version (ChecksumReader.getCRCInfo then
        # answers the P&M pass alone)
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

    a2a = args.exchange == "alltoall" and cfg["shared"] and world > 1
    owner = None
    owner_comm_error = None
    if args.exchange == "owner" and cfg["shared"] and world > 1:
        from delta_amd import shard
        try:
            owner = shard.OwnerComm.rccl()     # RCCL over xGMI, owned by libdkgpu (dk_comm_create)
        except Exception as e:                 # noqa: BLE001 -- every rank fails the same way here
            # the communicator could not be created (RCCL init): run the replicated-tail mode instead
            # and say so in the line
            owner_comm_error = "%s: %s" % (type(e).__name__, str(e)[:200])
            print("[rank %d] owner communicator failed (%s); exchange = allgather" % (rank, owner_comm_error),
                  file=sys.stderr)
        # every rank takes the same mode: a communicator that failed anywhere drops it everywhere
        if max_over_ranks(0.0 if owner is not None else 1.0) > 0 and owner is not None:
            owner.close()
            owner = None
            owner_comm_error = owner_comm_error or "a peer rank could not create its communicator"
    owner_ms = []
    a2a_ms = []

    def hash_exchange(side):
        from delta_amd import shard
        import torch
        te = time.perf_counter()
        shard.exchange_hash_owner(side, device="cuda")
        torch.cuda.synchronize()
        a2a_ms.append((time.perf_counter() - te) * 1e3)

    def build_scan(s):
        sb = s.getScanBuilder().withStats(cfg["stats"])
        if cfg["predicate"]:
            from delta_amd.expressions import Column, Literal, Predicate
            col, op, lit = cfg["predicate"]
            sb = sb.withFilter(Predicate(op, Column(col), Literal.ofLong(lit)))
        if cfg["shared"] and world > 1:
            sb = sb.withShard(world, rank, exchange=hash_exchange if a2a else None, owner=owner)
        return sb.build()

    # ---- region 1: the device step over inputs resident in HBM (roofline) ----
    scan = build_scan(snap)
    t0 = time.perf_counter()
    scan.prepare(eng)
    prepare_s = time.perf_counter() - t0
    n_ckpt_rows = sum(scan.ckpt.num_rows(i) for i in range(len(scan.ckpt_files))) if scan.ckpt else 0
    n_tail = int(scan.tail.rows)
    bytes_read, bytes_written = scan.ckpt.traffic() if scan.ckpt else (0, 0)
    exchange = None
    if dist is not None and cfg["shared"] and not a2a and owner is None:
        from delta_amd import shard
        meta = [(scan.ckpt_index[fi], scan.ckpt.row_offset(fi), scan.ckpt.num_rows(fi))
                for fi in range(len(scan.ckpt_files or []))]
        exchange = shard.SelectionExchange(meta, device="cuda")
    ex_ms = []
    merged = None

    def device_step():
        nonlocal merged
        scan.run()
        scan.sync()
        if owner is not None:
            owner_ms.append(dict(owner.ms))
        if exchange is not None:
            import ctypes as C
            import torch
            torch.cuda.synchronize()
            te = time.perf_counter()
            offs = (C.c_int64 * max(1, len(exchange.slots)))(*[off for off, _ in exchange.slots])

            def write_all(i, dst):
                if i == 0:   # every file of this rank in one call, straight into the collective buffer
                    base = exchange.buf.data_ptr()
                    K.check(K.lib().dk_replay_ckpt_selection_bits_all(scan._rh, C.c_void_p(base), offs, 1))
            merged = exchange.exchange(scan.tail_metrics.as_tuple(), scan.ckpt_metrics.as_tuple(), write_all)
            torch.cuda.synchronize()
            ex_ms.append((time.perf_counter() - te) * 1e3)

    dsteps = args.device_steps if args.device_steps is not None else args.steps
    for _ in range(args.warmup):
        device_step()
    del a2a_ms[:]
    device_counters = merged[0] if merged else scan.metrics.as_tuple()
    if a2a:      # the result stays where it was decoded; the counters of the world, for the report
        device_counters = tuple(scan.tail_metrics.as_tuple()[i] + v
                                for i, v in enumerate(sum_over_ranks(scan.ckpt_metrics.as_tuple())))
    if owner is not None:     # every rank's counters are its share: tail actions it owns + its rows
        device_counters = tuple(sum_over_ranks(scan.metrics.as_tuple()))
    del owner_ms[:]
    barrier()
    stats0 = scan.kernel_stats()
    t0 = time.perf_counter()
    for _ in range(dsteps):
        device_step()
    barrier()
    dev_elapsed = max_over_ranks(time.perf_counter() - t0)
    a2a_dev = sorted(a2a_ms)[len(a2a_ms) // 2] if a2a_ms else None
    stats1 = scan.kernel_stats()
    kern = {}
    for name, (avg1, c1) in stats1.items():
        avg0, c0 = stats0.get(name, (0.0, 0))
        if c1 > c0:
            kern[name] = (avg1 * c1 - avg0 * c0) / (c1 - c0)
    step_us = kern.pop("step_total", None)
    dom = max(kern.items(), key=lambda kv: kv[1]) if kern else ("none", 0.0)
    step_bytes = bytes_read + bytes_written
    step_gbs = step_bytes / (step_us * 1e-6) / 1e9 if step_us else None
    # roofline of the dominant kernel with a byte model (dk_parquet_kernel_traffic):
    # algorithmic bytes of one launch / its average launch time (HIP events on the replay stream)
    modelled = [k for k in ("k_snap_frag", "k_tile_decode", "k_string_copy", "k_probe") if k in kern]
    rk = max(modelled, key=lambda k: kern[k]) if modelled else None
    # every modelled kernel's own roofline fraction (same byte models, same HIP-event averages)
    kern_roof = {}
    for k in modelled:
        r_, w_ = scan.ckpt.kernel_traffic(k)
        gbs = (r_ + w_) / (kern[k] * 1e-6) / 1e9
        kern_roof[k] = dict(us=round(kern[k], 1), algorithmic_bytes=r_ + w_, gbs=round(gbs, 1),
                            frac=round(gbs / HBM_PEAK_GBS, 4))
    k_read, k_written = scan.ckpt.kernel_traffic(rk) if rk else (0, 0)
    k_bytes = k_read + k_written
    achieved = k_bytes / (kern[rk] * 1e-6) / 1e9 if rk else None
    pmc = pmc_traffic(rk, n_ckpt_rows, compression) if rk else None
    ckpt_files = list(scan.ckpt_files)
    if cfg["shared"] and owner is not None:
        dev_units = sum_over_ranks([n_ckpt_rows + n_tail])[0]       # each rank parsed its share of the tail
    elif cfg["shared"]:
        dev_units = sum_over_ranks([n_ckpt_rows])[0] + n_tail      # the tail is replicated, counted once
    else:
        dev_units = sum_over_ranks([n_ckpt_rows + n_tail])[0]
    scan.close()

    # ---- the headline: getScanFiles until fully consumed ----
    capture = {}

    def e2e_step(capture_result=False):
        """One getScanFiles on the loaded snapshot, consumed as the JMH benchmark consumes it
        (BenchmarkParallelCheckpointReading.java:124-135: sum add.size over the selected rows)."""
        sc = build_scan(snap)
        size_sum, n_sel = 0, 0
        tail_paths, bits = [], []
        it = sc.getScanFiles(eng)
        t_c, t_c0 = time.perf_counter(), time.monotonic()
        cprof = CONSUME_PROFILE and not capture_result
        t_w = t_v = t_s = 0.0
        waits, arrivals = [], []
        t_a = time.perf_counter()
        for b in it:
            if cprof:
                t_b = time.perf_counter(); t_w += t_b - t_a; waits.append(round((t_b - t_a) * 1e3, 2))
                arrivals.append((round(time.monotonic() * 1e3, 2), b.file_index, b.size))
            v = b.data["add.size"].fixed.view("<i8")
            if cprof:
                t_d = time.perf_counter(); t_v += t_d - t_b
            if b.selection is None:
                size_sum += int(v.sum())
                n_sel += b.size
            else:
                s_, k_ = masked_sum(v, b.selection)
                size_sum += s_
                n_sel += k_
            if cprof:
                t_a = time.perf_counter(); t_s += t_a - t_d
            if capture_result:
                if b.file_index < 0:
                    pc = b.data["add.path"]
                    tail_paths = [pc.string(int(r)).decode("utf-8", "replace") for r in b.selected_rows()]
                else:
                    sel = np.ones(b.size, bool) if b.selection is None else b.selection
                    bits.append(np.packbits(sel, bitorder="little"))
        b = v = None            # the consumer keeps no batch (a kept batch is copied out at close)
        consume_ms = (time.perf_counter() - t_c) * 1e3
        seen = sc.metrics.addFilesSeen if not (cfg["shared"] and world > 1 and rank > 0 and owner is None) \
            else sc.ckpt_metrics.addFilesSeen                  # a replicated tail counts once
        if capture_result:
            capture.update(counters=sc.metrics.as_tuple(), tail_paths=tail_paths, bits=bits)
        phases = dict(sc.prepare_ms)
        phases["consume"] = consume_ms
        if cprof:   # DK_CONSUME_PROFILE=1: where the consumer's time goes
            t_e = time.perf_counter()
            waits.append(round((t_e - t_a) * 1e3, 2))     # the last next(): StopIteration (final sync)
            phases.update(consume_wait=t_w * 1e3 + waits[-1], consume_column=t_v * 1e3, consume_sum=t_s * 1e3)
            log("consume waits (ms, per next()):", waits)
            if os.environ.get("DK_VERBOSE"):     # batch arrivals on the [dk] timeline's clock
                log("consume starts at monotonic %.3f ms; arrivals (monotonic ms, file, rows):" % (t_c0 * 1e3),
                    arrivals, "; ends at monotonic %.3f ms" % (time.monotonic() * 1e3))
        t_x = time.perf_counter()
        sc.close()
        phases["close"] = (time.perf_counter() - t_x) * 1e3
        if cprof:
            phases.update(getattr(sc, "close_ms", {}))
        return seen, n_sel, size_sum, phases

    for i in range(args.warmup):
        e2e_step(capture_result=(i == 0 and world == 1))
    barrier()
    t0 = time.perf_counter()
    seen_tot = sel_tot = size_tot = 0
    phase_sum = {}
    step_ms = []                                    # each timed step's wall time (this rank)
    for _ in range(args.steps):
        ts = time.perf_counter()
        seen, n_sel, size_sum, phases = e2e_step()
        step_ms.append((time.perf_counter() - ts) * 1e3)
        seen_tot += seen
        sel_tot += n_sel
        size_tot += size_sum
        for k, v in phases.items():
            phase_sum[k] = phase_sum.get(k, 0.0) + v
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    seen_all, sel_all, size_all = sum_over_ranks([seen_tot, sel_tot, size_tot])
    value = seen_all / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- beside the headline: a consumer that reads every selected scan file's path, partition
    # values and size (a connector's split planner, MultiThreadedTableReader.java:204-251), not only
    # add.size (the JMH shape above) ----
    FULL_LEAVES = ("add.path", "add.partitionValues.key_value.key", "add.partitionValues.key_value.value",
                   "add.size")

    def full_row_step():
        sc = build_scan(snap)
        n_sel = path_bytes = pv_entries = size_sum = d2h = 0
        t_a = time.perf_counter()
        for b in sc.getScanFiles(eng):
            cols = [b.data[leaf] for leaf in FULL_LEAVES]
            pc, kc, vc, sz = cols
            sel = np.ones(b.size, bool) if b.selection is None else b.selection
            lens = np.diff(pc.offs[:b.size + 1])                  # path bytes per row
            nent = np.diff(kc.row_offs[:b.size + 1])              # partitionValues entries per row
            path_bytes += masked_sum(lens, sel)[0]
            pv_entries += masked_sum(nent, sel)[0]
            s_, k_ = masked_sum(sz.fixed.view("<i8"), sel)
            size_sum += s_
            n_sel += k_
            if b.file_index >= 0:                                 # device-decoded: the D2H of its leaves
                d2h += sum(int(a.nbytes) for c in cols if c is not None
                           for a in (c.row_def, c.row_offs, c.entry_def, c.fixed, c.offs, c.chars) if a is not None)
        b = cols = pc = kc = vc = sz = sel = None
        ms = (time.perf_counter() - t_a) * 1e3
        phases = dict(sc.prepare_ms)
        seen = sc.metrics.addFilesSeen if not (cfg["shared"] and world > 1 and rank > 0 and owner is None) \
            else sc.ckpt_metrics.addFilesSeen
        sc.close()
        return seen, n_sel, path_bytes, pv_entries, size_sum, d2h, ms + phases.get("plan_files", 0) + \
            phases.get("checkpoint_open", 0) + phases.get("device_run", 0)

    full_row = None
    if args.full_row_steps > 0:
        full_row_step()                                          # warm-up
        barrier()
        t_f = time.perf_counter()
        fr = [full_row_step() for _ in range(args.full_row_steps)]
        barrier()
        f_el = max_over_ranks(time.perf_counter() - t_f)
        f_seen, f_sel, f_pb, f_pv, f_d2h = sum_over_ranks([sum(x[0] for x in fr), sum(x[1] for x in fr),
                                                          sum(x[2] for x in fr), sum(x[3] for x in fr),
                                                          sum(x[5] for x in fr)])
        k = args.full_row_steps
        full_row = {"consumer": "reads add.path, add.partitionValues and add.size of every selected scan file "
                                "(path length, partition entries, size sum)",
                    "ms_per_step": f_el / k * 1e3, "actions_per_s": f_seen / f_el, "steps": k,
                    "selected_per_step": f_sel // k, "path_bytes_per_step": f_pb // k,
                    "partition_entries_per_step": f_pv // k,
                    "d2h_bytes_per_step": f_d2h // k, "leaves": list(FULL_LEAVES)}

    # ---- beside the headline: the JMH operation itself (BenchmarkParallelCheckpointReading.java:110-139):
    # a new engine, Table.forPath, getLatestSnapshot, getScanState, getScanFiles consumed (sum of
    # add.size), engine closed -- one warm-up op, then --jmh-ops timed ops, average time per op ----
    jmh = None
    if args.jmh_ops > 0 and world == 1:
        def jmh_op():
            t_o = time.perf_counter()
            e2 = K.GpuEngine()
            sn = K.Table.forPath(e2, work).getLatestSnapshot(e2)
            sb = sn.getScanBuilder().withStats(cfg["stats"])
            if cfg["predicate"]:
                from delta_amd.expressions import Column, Literal, Predicate
                col, op, lit = cfg["predicate"]
                sb = sb.withFilter(Predicate(op, Column(col), Literal.ofLong(lit)))
            sc = sb.build()
            sc.getScanState(e2)
            size_sum = 0
            for b in sc.getScanFiles(e2):
                v = b.data["add.size"].fixed.view("<i8")
                size_sum += int(v.sum()) if b.selection is None else masked_sum(v, b.selection)[0]
            b = v = None
            seen = sc.metrics.addFilesSeen
            sc.close()
            e2.close()
            return seen, size_sum, (time.perf_counter() - t_o) * 1e3
        jmh_op()                                                  # warm-up (JMH's warm-up iterations)
        ops = [jmh_op() for _ in range(args.jmh_ops)]
        ms = sum(o[2] for o in ops) / len(ops)
        jmh = {"definition": "BenchmarkParallelCheckpointReading.benchmark: new engine + Table.forPath + "
                             "getLatestSnapshot + getScanState + getScanFiles consumed (sum of add.size over the "
                             "selected rows) + engine close; average time per op after one warm-up op",
               "ms_per_op": ms, "ops": len(ops), "ops_ms": [round(o[2], 2) for o in ops],
               "actions_per_s": ops[0][0] / (ms * 1e-3), "addFilesSeen_per_op": ops[0][0],
               "size_sum_matches_headline": ops[0][1] == size_all // args.steps}

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "actions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        # the spread of the timed steps (rank 0's clock): a step must not depend on the previous
        # step's teardown (the pinned staging ring, no per-open pinning)
        "step_ms_p50": round(float(np.percentile(step_ms, 50)), 3) if step_ms else None,
        "step_ms_p90": round(float(np.percentile(step_ms, 90)), 3) if step_ms else None,
        "step_ms_min_max": [round(min(step_ms), 3), round(max(step_ms), 3)] if step_ms else None,
        "higher_is_better": True,
        "scaling": "strong" if cfg["shared"] else "weak",
        "vs_baseline": None,
        "dtype": "u8/int64",
        "data": "synthetic (seed 20250218; delta_amd/synth.py)",
        "config": {"workload": cfg["desc"] % rows, "name": args.config, "compression": compression,
                   "parallelism": (("strong: checkpoint row groups in %d contiguous runs (one per GPU); " % world +
                                    ("commit files round-robin over the GPUs; keys owned by hash: commit-tail actions, "
                                     "checkpoint row hashes and hash hits' keys resolved by their owner over RCCL "
                                     "all-to-all (exchange=owner)" if owner is not None else
                                     "commit tail on every GPU; checkpoint rows routed to the owner of their path hash "
                                     "and answered over RCCL all-to-all (exchange=alltoall)" if a2a else
                                     "commit tail on every GPU; device step ends with one RCCL all-gather of counters "
                                     "+ selection bitmaps"))
                                   if cfg["shared"] else "weak: one table per GPU"),
                   "exchange": (("allgather (owner communicator failed: %s)" % owner_comm_error) if owner_comm_error
                                else args.exchange) if (cfg["shared"] and world > 1) else None,
                   "checkpoint_rows_per_gpu": n_ckpt_rows, "json_tail_rows": n_tail,
                   "checkpoint_files_per_gpu": len(ckpt_files)},
        "value_definition": "ScanMetrics.numAddFilesSeen / getScanFiles wall time until fully consumed "
                            "(BASELINE.md), summed over ranks / max-over-ranks time of the K timed steps",
        "ranks": world, "backend": backend or "none (1 process)",
        "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        "rccl_ranks": (dist.get_world_size() if dist is not None else None),
        "addFilesSeen_per_step": seen_all // args.steps, "selected_per_step": sel_all // args.steps,
        "size_sum_per_step": size_all // args.steps,
        "getScanFiles_phases_ms": {k: round(v / args.steps, 2) for k, v in phase_sum.items()},
        "device_step": {"ms": dev_elapsed / max(1, dsteps) * 1e3, "steps": dsteps,
                        "actions_per_s": dev_units * dsteps / dev_elapsed if dev_elapsed else None,
                        "counters": list(device_counters),
                        "exchange_ms": (sorted(ex_ms)[len(ex_ms) // 2] if ex_ms else a2a_dev),
                        "owner_exchange_ms": ({k: round(sorted(m[k] for m in owner_ms)[len(owner_ms) // 2], 3)
                                               for k in owner_ms[0]} if owner_ms else None),
                        "prepare_s": prepare_s},
        "full_row_consume": full_row,
        "jmh_op": jmh,
        "snapshot_load_ms": snapshot_ms,
        "snapshot_load_cold_ms": snapshot_cold_ms,
        "engine_create_ms": engine_create_ms,
        "snapshot_load_cold_phases_ms": cold_phases,
        "snapshot_load_with_crc_ms": snapshot_crc_ms,
        "snapshot_load_phases_ms": {k: round(v, 3) for k, v in snap.load_ms.items()},
        "kernels_us": {k: round(v, 2) for k, v in sorted(kern.items(), key=lambda kv: -kv[1])},
        "kernels_roofline": kern_roof,
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
        got = (capture["counters"], capture["tail_paths"], capture["bits"]) if capture else None
        aff, quota = cpu_share()
        # the pool's rule: one GPU's share of the box is 16 CPUs although nproc shows the machine
        threads = args.cpu_threads or min(aff, quota or 16)
        result["cpu_baseline"] = cpu_baseline(work, ckpt_files, cfg, threads, got=got)
        result["cpu_baseline_host"] = {"cpu_count": os.cpu_count(), "nproc": aff, "cgroup_cpus": quota,
                                       "threads_used": threads, "cpu": _cpu_model()}
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.barrier()          # every rank is done with the shared table
    if not args.workdir and (rank == 0 or not cfg["shared"]):
        shutil.rmtree(work, ignore_errors=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    sys.exit(main())
