"""Multi-rank sharding of the checkpoint half (delta_amd/shard.py).

CPU: ownership / merge units, and a world_size-2 torch.distributed (gloo, 127.0.0.1) run where each
rank reconciles its share of the checkpoint files with the oracle, gathers to rank 0, and the merged
result must equal the unsharded replay (ordered rows + ScanMetrics counters).
GPU: the product's sharded path (GpuScan.withShard) for 2 and 3 ranks simulated in one process.
"""
import os
import socket

import numpy as np
import pytest

from delta_amd import shard, synth
from tests.golden_util import TABLES


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_shard_output(table, world, rank, jbs=1024):
    from oracle import ref
    r = ref.replay(table, json_batch_size=jbs, shard=(world, rank))
    files = {}
    for b in r.checkpoint:
        files[b.file_index] = [ref.canon_add_from_cols(b.cols, int(i)) + (r.table_root,)
                               for i in np.nonzero(b.selected)[0]]
    tail = [ref.canon_add_from_json(a) + (r.table_root,) for a in r.json_rows]
    return shard.ShardOutput(rank, r.tail_counters.as_tuple(), r.ckpt_counters.as_tuple(), tail, files)


def _flatten(payloads):
    return [row for p in payloads for row in p]


def test_owned_files_partition():
    for n in (0, 1, 5, 64):
        for world in (1, 2, 3, 8):
            parts = [shard.owned_files(n, world, r) for r in range(world)]
            flat = sorted(i for p in parts for i in p)
            assert flat == list(range(n))
    with pytest.raises(ValueError):
        shard.owned_files(4, 2, 2)


def test_merge_orders_and_sums():
    a = shard.ShardOutput(0, (3, 3, 1, 1, 2), (10, 0, 7, 2, 0), tail=["t"], files={0: ["f0"], 2: ["f2"]})
    b = shard.ShardOutput(1, (3, 3, 1, 1, 2), (5, 0, 4, 0, 0), tail=["ignored"], files={1: ["f1"]})
    counters, payloads = shard.merge([b, a])
    assert counters == (18, 3, 12, 3, 2)
    assert payloads == [["t"], ["f0"], ["f1"], ["f2"]]
    with pytest.raises(ValueError):
        shard.merge([b])
    with pytest.raises(ValueError):
        shard.merge([a, shard.ShardOutput(1, a.tail_counters, a.ckpt_counters, None, {0: []})])


@pytest.mark.parametrize("world", [2, 3])
def test_oracle_shards_merge_to_full_replay(tmp_path, world):
    from oracle import ref
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=6_000, n_parts=5, n_commits=6, dv_frac=0.2,
                                                     ckpt_removes=50))
    full = ref.replay(str(tmp_path))
    counters, payloads = shard.merge([_oracle_shard_output(str(tmp_path), world, r) for r in range(world)])
    assert counters == full.counters.as_tuple()
    assert _flatten(payloads) == full.scan_files()


@pytest.mark.parametrize("name", ["multi-part-checkpoint", "v2-checkpoint-parquet"])
def test_oracle_shards_golden(name):
    from oracle import ref
    table = os.path.join(TABLES, name)
    full = ref.replay(table, json_batch_size=2)
    counters, payloads = shard.merge([_oracle_shard_output(table, 2, r, jbs=2) for r in range(2)])
    assert counters == full.counters.as_tuple()
    assert _flatten(payloads) == full.scan_files()


def _gloo_worker(rank, world, port, table, out_path):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        outs = shard.gather(_oracle_shard_output(table, world, rank))
        if rank == 0:
            from oracle import ref
            full = ref.replay(table)
            counters, payloads = shard.merge(outs)
            ok = counters == full.counters.as_tuple() and _flatten(payloads) == full.scan_files()
            with open(out_path, "w") as f:
                f.write("ok %d %d" % (len(_flatten(payloads)), counters[2]) if ok else "MISMATCH")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    table = str(tmp_path / "t")
    synth.write_table(table, synth.TableSpec(n_adds=8_000, n_parts=4, n_commits=8, dv_frac=0.1))
    out = str(tmp_path / "result.txt")
    mp.spawn(_gloo_worker, args=(2, _free_port(), table, out), nprocs=2, join=True)
    with open(out) as f:
        res = f.read()
    assert res.startswith("ok"), res


def test_oracle_shards_v2_sidecars(tmp_path):
    from oracle import ref
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=6_000, n_parts=5, v2_sidecars=5, n_commits=6,
                                                     ckpt_removes=50, hot_frac=0.6))
    full = ref.replay(str(tmp_path))
    counters, payloads = shard.merge([_oracle_shard_output(str(tmp_path), 3, r) for r in range(3)])
    assert counters == full.counters.as_tuple()
    assert _flatten(payloads) == full.scan_files()


@pytest.mark.gpu
@pytest.mark.parametrize("world,v2", [(2, 0), (3, 0), (3, 5)])
def test_gpu_shards_merge_to_oracle(tmp_path, world, v2):
    from delta_amd import kernel as K
    from oracle import ref
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=20_000, n_parts=5, n_commits=8, dv_frac=0.2,
                                                     ckpt_removes=100, v2_sidecars=v2))
    eng = K.GpuEngine()
    outs, scans = [], []
    for r in range(world):
        snap = K.Table.forPath(eng, str(tmp_path)).getLatestSnapshot(eng)
        o, sc = shard.gpu_shard_scan(eng, snap, world, r)
        outs.append(o)
        scans.append(sc)
    counters, batches = shard.merge(outs)
    rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in batches for i in b.selected_rows()]
    full = ref.replay(str(tmp_path))
    assert counters == full.counters.as_tuple()
    assert rows == full.scan_files()
    for sc in scans:
        sc.close()
    eng.close()


# ---- row-group sharding + bitmap gather (the product's plan_units / gather_selections) ----

def test_plan_units_cover_every_row_group_once():
    for rg in ([[100] * 10], [[1000, 1000], [1000], [500, 500, 500]], [[5]], [[1] * 3, [1] * 2], []):
        for world in (1, 2, 3, 8):
            units = [shard.plan_units(rg, world, r) for r in range(world)]
            flat = sorted((f, g) for u in units for (f, a, b) in u for g in range(a, b))
            assert flat == [(f, g) for f, rows in enumerate(rg) for g in range(len(rows))]
            for u in units:                      # contiguous runs, in replay order
                assert u == sorted(u)
    # a single-part checkpoint with several row groups spreads over the ranks
    assert all(shard.plan_units([[100] * 8], 4, r) for r in range(4))


def _oracle_units(table, world, rank):
    """This rank's units with selections from the oracle's full replay (bits packed LSB first)."""
    from delta_amd import kernel as K
    from oracle import ref
    r = ref.replay(table)
    files = [b.path for b in r.checkpoint]
    units = shard.plan_units([K.row_group_rows(p) for p in files], world, rank)
    rgs = [K.row_group_rows(p) for p in files]
    out = []
    for f, a, b in units:
        r0 = sum(rgs[f][:a])
        n = sum(rgs[f][a:b])
        sel = r.checkpoint[f].selected[r0:r0 + n].astype(bool)
        out.append((f, r0, n, np.packbits(sel, bitorder="little")))
    # the checkpoint part of the counters travels from rank 0 (per-unit splits are the GPU test's)
    ck = r.ckpt_counters.as_tuple() if rank == 0 else (0, 0, 0, 0, 0)
    return r, out, r.tail_counters.as_tuple(), ck


def _gloo_bits_worker(rank, world, port, table, out_path):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        full, units, tail, ck = _oracle_units(table, world, rank)
        counters, sels = shard.gather_selections(units, tail, ck)
        if rank == 0:
            ok = counters == full.counters.as_tuple()
            for b in full.checkpoint:                 # reassemble each file's selection from the units
                parts = [s for s in sels if s[0] == b.file_index]
                bits = np.concatenate([np.unpackbits(s[3], bitorder="little")[:s[2]] for s in parts])
                ok = ok and np.array_equal(bits.astype(bool), b.selected.astype(bool))
            with open(out_path, "w") as f:
                f.write("ok %d" % len(sels) if ok else "MISMATCH")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_world2_selection_bitmaps(tmp_path):
    """gloo world 2: plan_units splits a single-part checkpoint by row groups and uneven parts by
    rows; gather_selections reassembles the oracle's selection bits and counters on rank 0."""
    import torch.multiprocessing as mp
    for name, spec in (("single", dict(n_parts=1, row_group_size=1500)), ("uneven", dict(n_parts=3, row_group_size=2000))):
        table = str(tmp_path / name)
        synth.write_table(table, synth.TableSpec(n_adds=9_000, n_commits=6, dv_frac=0.1, **spec))
        out = str(tmp_path / (name + ".txt"))
        mp.spawn(_gloo_bits_worker, args=(2, _free_port(), table, out), nprocs=2, join=True)
        with open(out) as f:
            res = f.read()
        assert res.startswith("ok"), (name, res)


@pytest.mark.gpu
@pytest.mark.parametrize("world,spec", [(3, dict(n_parts=1, row_group_size=2500)), (4, dict(n_parts=3, row_group_size=3000))])
def test_gpu_row_group_shards(tmp_path, world, spec):
    """Single-part and uneven multi-part checkpoints split by row groups over simulated ranks: the
    merged rows equal the oracle's, and the bitmaps packed on the GPU equal the selections."""
    from delta_amd import kernel as K
    from oracle import ref
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=20_000, n_commits=8, dv_frac=0.2, **spec))
    eng = K.GpuEngine()
    outs, scans = [], []
    for r in range(world):
        snap = K.Table.forPath(eng, str(tmp_path)).getLatestSnapshot(eng)
        o, sc = shard.gpu_shard_scan(eng, snap, world, r)
        outs.append(o)
        scans.append(sc)
        for fi in range(len(sc.ckpt_files or [])):
            bits = np.unpackbits(sc.selection_bits(fi), bitorder="little")[:sc.ckpt.num_rows(fi)]
            sel = np.zeros(sc.ckpt.num_rows(fi), np.uint8)
            from delta_amd._lib import lib
            lib().dk_replay_ckpt_selection(sc._rh, fi, sel.ctypes.data, len(sel))
            assert np.array_equal(bits.astype(bool), sel.astype(bool))
    assert sum(1 for sc in scans if sc.ckpt_files) == world       # every rank got checkpoint rows
    counters, batches = shard.merge(outs)
    rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in batches for i in b.selected_rows()]
    full = ref.replay(str(tmp_path))
    assert counters == full.counters.as_tuple()
    assert rows == full.scan_files()
    for sc in scans:
        sc.close()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["allgather", "alltoall", "owner"])
def test_gpu_two_processes_gloo(tmp_path, mode):
    """Two processes on the GPU, each scanning its row-group shard with the product (alltoall: its
    rows routed to their path-hash owners and answered back), merge counters and selection bitmaps
    with gather_selections over gloo; rank 0 checks the oracle."""
    import json
    import subprocess
    import sys
    from oracle import ref
    table = str(tmp_path / "t")
    synth.write_table(table, synth.TableSpec(n_adds=30_000, n_parts=3, row_group_size=4000, n_commits=8, dv_frac=0.1))
    port = _free_port()
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "shard_worker.py")
    out = str(tmp_path / "res.json")
    procs = [subprocess.Popen([sys.executable, worker, table, out, mode],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port)))
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    with open(out) as f:
        res = json.load(f)
    full = ref.replay(table)
    assert tuple(res["counters"]) == full.counters.as_tuple()
    for b in full.checkpoint:
        bits = np.array(res["selection"][str(b.file_index)], dtype=bool)
        assert np.array_equal(bits, b.selected.astype(bool))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["owner_fail", "owner_prefetch_fail"])
def test_gpu_owner_failure_reaches_every_rank(tmp_path, mode):
    """Owner mode over gloo (the library's protocol through the callback transport), two GPU
    processes. owner_fail: a malformed commit file that only rank 1 parses (j = 1 of the newest-first
    replay order) fails rank 1's commit-tail parse; rank 0 must raise too (at the global-steps vote).
    owner_prefetch_fail: rank 1 fails after its prepare, before its owner run (the add.size
    prefetch); it answers the run's first vote with its error bit and rank 0 raises there. No rank
    waits for the other in a collective."""
    import json
    import subprocess
    import sys
    table = str(tmp_path / "t")
    synth.write_table(table, synth.TableSpec(n_adds=8_000, n_parts=2, row_group_size=2000, n_commits=4))
    if mode == "owner_fail":
        log = os.path.join(table, "_delta_log")
        commits = sorted(f for f in os.listdir(log) if f.endswith(".json"))
        with open(os.path.join(log, commits[-2]), "a") as f:    # second newest: replay index 1 -> rank 1
            f.write('{"add": {"path": \n')
    port = _free_port()
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "shard_worker.py")
    out = str(tmp_path / "res.json")
    procs = [subprocess.Popen([sys.executable, worker, table, out, mode],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port), DK_INJECT_PREFETCH_FAULT="1"))
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    res = [json.load(open(out + ".%d" % r)) for r in range(2)]
    assert res[0]["error"] == "OwnerPeerError", res
    assert res[1]["error"] not in (None, "OwnerPeerError"), res
