"""One-GPU rehearsal of one rank of the N-GPU owner-partitioned scan (bench.py --gpus N, the default
exchange=owner), for the timing of the path the driver's 8-GPU run measures.

All N ranks' scans run in this process on one GPU: each rank opens only its contiguous run of row
groups (asynchronous open) and parses only its commit files j = rank (mod N); then every rank's
dk_replay_owner_run runs on its own thread over the library's in-process transport
(dk_comm_create_local: the same protocol and votes as over RCCL, buffers copied device to device).
Every rank is timed:

  open       prepare (footers, page headers, the commit-tail parse of its files + replay create)
             until its asynchronous open has finished decoding (the ranks run one after another, so
             each rank's H2D and decode have the GPU to themselves, as on its own GPU)
  hash       its owner run's decode-and-hash phase: the row key hashes, the routing counts and
             the row records packed (dk_comm_last_run's local steps of that phase)
  exchange   the local steps of its owner run's commit-tail and row / candidate exchanges
             (dk_comm_last_run: each step timed, and with DK_LOCAL_SERIAL=1, the default here, run
             alone on the device, so a rank's steps do not share the GPU with its peers' as they
             would not on its own GPU); the wall times of the concurrent run are reported beside it
  transfer   the bytes it sends through the all-to-alls at an assumed per-GPU all-to-all bandwidth
             (--a2a-gbs, default 300 GB/s: 7 xGMI links at ~43 GB/s each) + 30 us per collective
  consume    its scan-file batches consumed as bench.py's JMH-shaped consumer does (sum of add.size
             over the selected rows)

per_rank_ms = open + hash + exchange + transfer + consume; the rehearsed N-GPU step is the max over ranks.
Usage: python tools/rehearse_rank.py --world 8 [--config c3] [--workdir DIR] > out.json
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--a2a-gbs", type=float, default=300.0)
    ap.add_argument("--concurrent", action="store_true", help="ranks' local steps share the GPU (no DK_LOCAL_SERIAL)")
    args = ap.parse_args()
    if not args.concurrent:
        os.environ["DK_LOCAL_SERIAL"] = "1"
    import bench
    cfg = bench.CONFIGS[args.config]
    rows = args.rows or cfg["rows"]
    compression = cfg["spec"].get("compression", "none")
    work = args.workdir or os.path.join(tempfile.gettempdir(), "dk_rehearse_%s_%d" % (args.config, rows))
    marker = os.path.join(work, ".ready")
    if not os.path.exists(marker):
        import shutil
        shutil.rmtree(work, ignore_errors=True)
        t0 = time.time()
        bench.make_table(work, rows, 20250218, compression, cfg)
        open(marker, "w").close()
        print("table generated in %.1fs" % (time.time() - t0), file=sys.stderr)

    import numpy as np
    import torch
    torch.cuda.init()
    from delta_amd import kernel as K
    from delta_amd import shard
    from delta_amd._lib import check, lib

    world = args.world
    eng = K.GpuEngine(timing=False)
    snap = K.Table.forPath(eng, work).getLatestSnapshot(eng)
    steps = shard.OwnerComm.table_steps(eng, snap)
    comms = shard.OwnerComm.local(world, steps=steps)
    collectives = 11                            # per owner run without a collision (dk_comm.cpp)
    # iteration 0 warms the caching allocators (every rank's blocks, as each rank's process is warm
    # after bench.py's warm-up steps); iteration 1 is reported
    for it in range(2):
        scans, opened = [], {}
        for r in range(world):
            s = K.Table.forPath(eng, work).getLatestSnapshot(eng)
            sc = s.getScanBuilder().withStats(cfg["stats"]).withShard(world, r, owner=comms[r]).build()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sc.prepare(eng)
            t1 = time.perf_counter()
            if sc.ckpt is not None:
                check(lib().dk_parquet_sync(sc.ckpt._h))
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            opened[r] = {"prepare_ms": (t1 - t0) * 1e3, "open_ms": (t2 - t0) * 1e3,
                         "async_open": bool(sc.ckpt is not None and sc.ckpt.async_open),
                         "checkpoint_rows": int(sum(sc.ckpt.num_rows(i) for i in range(len(sc.ckpt_files)))) if sc.ckpt else 0,
                         "commit_files": len(sc.tail_commits), "tail_rows": int(sc.tail.rows),
                         "phases_ms": {k: round(v, 2) for k, v in sc.prepare_ms.items()}}
            scans.append(sc)
        for sc in scans:                        # as getScanFiles does in owner mode
            for leaf in sc.PREFETCH_LEAVES:
                if leaf in sc.ckpt.leaves:
                    check(lib().dk_replay_prefetch_leaf(sc._rh, leaf.encode()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        shard.run_local(scans)
        run_ms = (time.perf_counter() - t0) * 1e3
        counters = np.zeros(5, np.int64)
        consume = {}
        for r, sc in enumerate(scans):
            counters += np.array(sc.metrics.as_tuple())
            t0 = time.perf_counter()
            size_sum = n_sel = 0
            for b in sc._batches():
                v = b.data["add.size"].fixed.view("<i8")
                if b.selection is None:
                    size_sum += int(v.sum())
                    n_sel += b.size
                else:
                    s_, k_ = bench.masked_sum(v, b.selection)
                    size_sum += s_
                    n_sel += k_
            b = v = None
            consume[r] = ((time.perf_counter() - t0) * 1e3, n_sel)
        if it == 0:
            for sc in scans:
                sc.close()
    per_rank = {}
    for r in range(world):
        m = comms[r].ms
        ex = m["tail_local"] + m["row_local"]
        hs = m["decode_local"]
        tr = comms[r].bytes_sent / (args.a2a_gbs * 1e9) * 1e3 + comms[r].collectives * 0.03
        per_rank[r] = dict(opened[r], exchange_ms=round(ex, 3), hash_ms=round(hs, 3), owner_run_ms={k: round(v, 3) for k, v in m.items()},
                           owner_steps_ms={k: round(v, 3) for k, v in comms[r].steps_ms.items()},
                           bytes_sent=comms[r].bytes_sent, transfer_model_ms=round(tr, 3),
                           consume_ms=round(consume[r][0], 3), selected=consume[r][1],
                           per_rank_ms=round(opened[r]["open_ms"] + hs + ex + tr + consume[r][0], 2))
    step = max(v["per_rank_ms"] for v in per_rank.values())
    seen = int(counters[0])
    out = {"world": world, "config": args.config, "rows": rows, "counters": [int(x) for x in counters],
           "rehearsed_step_ms": round(step, 2), "rehearsed_actions_per_s": seen / (step * 1e-3),
           "collectives_per_run": collectives, "a2a_gbs_assumed": args.a2a_gbs, "per_rank": per_rank,
           "all_ranks_owner_run_ms": round(run_ms, 3),
           "note": "one process, one GPU, caches warmed by a first iteration: each rank's open ran alone "
                   "(its own H2D and decode); every rank's dk_replay_owner_run concurrently on its own thread "
                   "over the in-process transport (all ranks' exchange kernels share the GPU); transfer time "
                   "modelled from the bytes each rank sends"}
    for sc in scans:
        sc.close()
    for c in comms:
        c.close()
    plain = snap.getScanBuilder().withStats(cfg["stats"]).build()      # the unsharded scan's counters
    for _ in plain.getScanFiles(eng):
        pass
    out["counters_unsharded"] = list(plain.metrics.as_tuple())
    out["counters_match"] = out["counters_unsharded"] == out["counters"]
    plain.close()
    print(json.dumps(out, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
