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
