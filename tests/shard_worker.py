"""One rank of tests/test_shard.py::test_gpu_two_processes_gloo (not a test module): scan this
rank's row-group shard on the GPU, gather counters + selection bitmaps over gloo, and have rank 0
write them to a JSON file. Usage: RANK=.. WORLD_SIZE=.. MASTER_ADDR/PORT=.. python shard_worker.py TABLE OUT [allgather|alltoall|owner]
(alltoall: the probe goes through the hash(path)-owner exchange; owner: the owner-partitioned
reconciliation; their collectives over gloo)"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch.distributed as dist
    from delta_amd import kernel as K
    from delta_amd import shard
    table, out = sys.argv[1], sys.argv[2]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    eng = K.GpuEngine()
    snap = K.Table.forPath(eng, table).getLatestSnapshot(eng)
    mode = sys.argv[3] if len(sys.argv) > 3 else "allgather"
    if mode in ("owner_fail", "owner_prefetch_fail"):
        # owner_fail: a malformed commit only rank 1 parses; owner_prefetch_fail: rank 1's add.size
        # prefetch fails between its prepare and its owner run (DK_INJECT_PREFETCH_FAULT=1). Every
        # rank must raise, none hang.
        scan = snap.getScanBuilder().withShard(world, rank, owner=shard.OwnerComm.over_torch()).build()
        try:
            list(scan.getScanFiles(eng))
            res = {"error": None}
        except Exception as e:      # noqa: BLE001
            res = {"error": type(e).__name__, "msg": str(e)[:300]}
        with open(out + ".%d" % rank, "w") as fh:
            json.dump(res, fh)
        scan.close()
        eng.close()
        dist.destroy_process_group()
        return
    if mode == "owner":      # owner-partitioned: every rank's counters are its share of the world's
        scan = snap.getScanBuilder().withShard(world, rank, owner=shard.OwnerComm.over_torch()).build()
    else:
        scan = snap.getScanBuilder().withShard(world, rank, exchange=shard.exchange_hash_owner if mode == "alltoall"
                                               else None).build()
    scan.prepare(eng)
    scan.run()
    scan.sync()
    if mode == "owner":
        counters, sels = shard.gather_selections(shard.scan_units(scan), (0,) * 5, scan.metrics.as_tuple())
    else:
        counters, sels = shard.gather_selections(shard.scan_units(scan), scan.tail_metrics.as_tuple(),
                                                 scan.ckpt_metrics.as_tuple())
    if rank == 0:
        files = {}
        for f, r0, n, bits in sels:
            files.setdefault(f, []).append(np.unpackbits(bits, bitorder="little")[:n])
        with open(out, "w") as fh:
            json.dump({"counters": list(counters),
                       "selection": {str(f): np.concatenate(v).astype(int).tolist() for f, v in files.items()}}, fh)
    scan.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
