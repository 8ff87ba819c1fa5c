"""Multi-GPU sharding of the checkpoint half of Scan.getScanFiles.

A checkpoint row's fate depends only on the commit-tail key sets: checkpoint adds are never
inserted into the "already returned" set and checkpoint removes are ignored
(kernel-api/.../internal/replay/ActiveAddFilesIterator.java:164,214-220).
Checkpoint files (multi-part parts, V2 manifest + sidecars) therefore shard across ranks with no
data-path exchange:

* rank r owns the checkpoint files whose replay-order index i has i % world == r
  (``owned_files``; replay order is LogSegment.allLogFilesReversed, LogSegment.java:166-178);
* every rank parses the (small) commit tail and builds its key table on its own GPU;
* results merge on one rank (``gather`` over torch.distributed, then ``merge``): the ScanMetrics
  counters are the tail part (taken once, from rank 0) plus the sum of the checkpoint parts, and the
  selected rows are emitted tail first, then checkpoint files in replay order.

The same merge serves GPU ranks (payloads are ``FilteredColumnarBatch``es) and the CPU tests
(payloads are oracle rows); it never looks inside a payload.
"""
from __future__ import annotations

from dataclasses import dataclass, field


def owned_files(n_files: int, world: int, rank: int) -> list:
    """Replay-order indices of the checkpoint files rank `rank` reconciles."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad shard (world=%r, rank=%r)" % (world, rank))
    return [i for i in range(n_files) if i % world == rank]


@dataclass
class ShardOutput:
    rank: int
    tail_counters: tuple                         # commit-tail part of the five ScanMetrics counters
    ckpt_counters: tuple                         # this rank's checkpoint part
    tail: object = None                          # commit-tail payload (used from rank 0 only)
    files: dict = field(default_factory=dict)    # replay-order checkpoint file index -> payload


def merge(outputs) -> tuple:
    """(counters, payloads in replay order) from every rank's ShardOutput."""
    outs = sorted(outputs, key=lambda o: o.rank)
    if not outs or outs[0].rank != 0 or [o.rank for o in outs] != list(range(len(outs))):
        raise ValueError("merge needs one output per rank 0..world-1")
    counters = list(outs[0].tail_counters)
    for o in outs:
        counters = [a + b for a, b in zip(counters, o.ckpt_counters)]
    files = {}
    for o in outs:
        for i, payload in o.files.items():
            if i in files:
                raise ValueError("checkpoint file %d produced by two ranks" % i)
            files[i] = payload
    payloads = ([outs[0].tail] if outs[0].tail is not None else []) + [files[i] for i in sorted(files)]
    return tuple(counters), payloads


def gather(output: ShardOutput, group=None):
    """All ranks' outputs on rank 0 (None elsewhere), over torch.distributed (gloo or RCCL)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bucket = [None] * world if dist.get_rank(group) == 0 else None
    dist.gather_object(output, bucket, dst=0, group=group)
    return bucket


def gpu_shard_scan(engine, snapshot, world: int, rank: int, with_stats: bool = False):
    """Run this rank's share of getScanFiles on its GPU. Returns (ShardOutput whose payloads are
    FilteredColumnarBatches with host-resident columns, the scan to close() when done)."""
    scan = snapshot.getScanBuilder().withStats(with_stats).withShard(world, rank).build()
    batches = list(scan.getScanFiles(engine))
    out = ShardOutput(rank, scan.tail_metrics.as_tuple(), scan.ckpt_metrics.as_tuple())
    for b in batches:
        if b.file_index < 0:
            out.tail = b
        else:
            out.files[b.file_index] = b
    return out, scan
