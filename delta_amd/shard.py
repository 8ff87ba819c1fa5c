"""Multi-GPU sharding of the checkpoint half of Scan.getScanFiles.

A checkpoint row's fate depends only on the commit-tail key sets: checkpoint adds are never
inserted into the "already returned" set and checkpoint removes are ignored
(kernel-api/.../internal/replay/ActiveAddFilesIterator.java:164,214-220).
Checkpoint files (multi-part parts, V2 manifest + sidecars) therefore shard across ranks with no
data-path exchange:

* the checkpoint's row groups, in replay order (LogSegment.allLogFilesReversed,
  LogSegment.java:166-178; rows in file order), are cut into ``world`` contiguous runs of about
  equal row counts (``plan_units``), so single-part and uneven multi-part checkpoints spread over
  every rank; a rank reads each of its files as the row-group range it owns
  (dk_parquet_open_rg). ``owned_files`` (whole files round-robin) is the coarser alternative;
* every rank parses the (small) commit tail and builds its key table on its own GPU;
* results merge on one rank: ``gather_selections`` all-gathers each rank's ScanMetrics counters and
  its selection bitmaps, packed on the GPU (dk_replay_ckpt_selection_bits), over RCCL (or gloo);
  the row data stays on the GPU that decoded it. The counters are the tail part (taken once, from
  rank 0) plus the sum of the checkpoint parts; selections come out tail first, then checkpoint
  rows in replay order. ``gather`` / ``merge`` do the same for whole payloads
  (host objects, used by tests).

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


def plan_units(rg_rows, world: int, rank: int) -> list:
    """This rank's share of the checkpoint: [(file index, first row group, end row group)] over
    `rg_rows` (row counts per row group, per file in replay order). The row groups form one
    sequence cut into `world` contiguous runs at the multiples of total / world."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad shard (world=%r, rank=%r)" % (world, rank))
    seq = [(f, g, n) for f, rows in enumerate(rg_rows) for g, n in enumerate(rows)]
    total = sum(n for _, _, n in seq) or 1
    mine, acc = [], 0
    for f, g, n in seq:
        # a row group belongs to the rank whose share of the row sequence holds its middle row
        owner = min(world - 1, int((acc + n / 2.0) * world / total))
        if owner == rank:
            if mine and mine[-1][0] == f and mine[-1][2] == g:
                mine[-1] = (f, mine[-1][1], g + 1)
            else:
                mine.append((f, g, g + 1))
        acc += n
    return mine


@dataclass
class ShardOutput:
    rank: int
    tail_counters: tuple                         # commit-tail part of the five ScanMetrics counters
    ckpt_counters: tuple                         # this rank's checkpoint part
    tail: object = None                          # commit-tail payload (used from rank 0 only)
    files: dict = field(default_factory=dict)    # (replay-order file index, first row) -> payload


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
            key = i if isinstance(i, tuple) else (i, 0)
            if key in files:
                raise ValueError("checkpoint rows %r produced by two ranks" % (key,))
            files[key] = payload
    payloads = ([outs[0].tail] if outs[0].tail is not None else []) + [files[i] for i in sorted(files)]
    return tuple(counters), payloads


def gather_selections(units, tail_counters, ckpt_counters, group=None, device=None):
    """All ranks' checkpoint selection bitmaps and counters on every rank, in two all-gathers
    (sizes, then one padded int64 header + one padded byte tensor per rank) -- RCCL when the
    tensors live on the GPU (backend "nccl"), gloo on the CPU.

    units: [(replay-order file index, first row, rows, packed bits (uint8 array or tensor))].
    Returns (counters, [(file index, first row, rows, bits numpy array)] in replay order)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = torch.device(device) if device is not None else torch.device("cpu")
    world = dist.get_world_size(group)
    head = [len(units)] + list(tail_counters) + list(ckpt_counters)
    for f, r0, n, _ in units:
        head += [f, r0, n]
    blobs = [b if isinstance(b, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(b, dtype=np.uint8))
             for _, _, _, b in units]
    bits = torch.cat([b.reshape(-1).to(dev) for b in blobs]) if blobs else torch.zeros(0, dtype=torch.uint8, device=dev)
    sizes = torch.tensor([len(head), bits.numel()], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    hmax = max(int(s[0]) for s in all_sizes)
    bmax = max(1, max(int(s[1]) for s in all_sizes))
    h = torch.zeros(hmax, dtype=torch.int64, device=dev)
    h[:len(head)] = torch.tensor(head, dtype=torch.int64, device=dev)
    b = torch.zeros(bmax, dtype=torch.uint8, device=dev)
    b[:bits.numel()] = bits
    hs = [torch.zeros_like(h) for _ in range(world)]
    bs = [torch.zeros_like(b) for _ in range(world)]
    dist.all_gather(hs, h, group=group)
    dist.all_gather(bs, b, group=group)
    counters = None
    sels = []
    for rk in range(world):
        hv = hs[rk].cpu().numpy()
        bv = bs[rk].cpu().numpy()
        nu = int(hv[0])
        tail, ck = hv[1:6], hv[6:11]
        counters = [int(x) for x in tail] if counters is None else counters
        counters = [a + int(c) for a, c in zip(counters, ck)]
        pos = 0
        for u in range(nu):
            f, r0, n = (int(x) for x in hv[11 + 3 * u: 14 + 3 * u])
            nb = (n + 7) // 8
            sels.append((f, r0, n, bv[pos:pos + nb].copy()))
            pos += nb
    sels.sort(key=lambda x: (x[0], x[1]))
    return tuple(counters), sels


class SelectionExchange:
    """The device-step exchange: every rank's five tail + five checkpoint ScanMetrics counters and
    its packed selection bitmaps land on the root rank in ONE collective.

    The unit layout (file, first row, rows) of every rank is exchanged once, when the exchange is
    built (``all_gather_object``, outside any timed region), so every rank knows every buffer's
    size. Each step then writes its counters (80 bytes) and its bitmaps straight into one
    fixed-size buffer on its own device (``write_bits(i, dst)`` fills unit i, e.g. with
    ``dk_replay_ckpt_selection_bits(..., dst_on_device=1)``), ``all_gather_into_tensor`` moves the
    world's buffers into one tensor (RCCL over xGMI when the tensors live on the GPU, gloo on the
    CPU), and only the root copies that tensor to the host, once."""

    HEAD = 80                               # 10 x int64 counters

    def __init__(self, units_meta, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dev = torch.device(device) if device is not None else torch.device("cpu")
        metas = [None] * self.world
        dist.all_gather_object(metas, [tuple(int(x) for x in u) for u in units_meta], group=group)
        self.metas = metas
        sizes = [self.HEAD + sum((n + 7) // 8 for _, _, n in m) for m in metas]
        self.size = max(sizes)
        self.buf = torch.zeros(self.size, dtype=torch.uint8, device=self.dev)
        self.out = torch.empty(self.size * self.world, dtype=torch.uint8, device=self.dev)
        self.slots = []                     # (offset, bytes) of this rank's units inside buf
        at = self.HEAD
        for _, _, n in metas[self.rank]:
            self.slots.append((at, (n + 7) // 8))
            at += (n + 7) // 8

    def exchange(self, tail_counters, ckpt_counters, write_bits, root=0):
        """(counters, [(file, first row, rows, bits)] in replay order) on the root, None elsewhere."""
        import numpy as np
        import torch
        import torch.distributed as dist
        head = torch.tensor(list(tail_counters) + list(ckpt_counters), dtype=torch.int64)
        self.buf[:self.HEAD].copy_(head.view(torch.uint8), non_blocking=False)
        for i, (off, nb) in enumerate(self.slots):
            write_bits(i, self.buf[off:off + nb])
        dist.all_gather_into_tensor(self.out, self.buf, group=self.group)
        if self.rank != root:
            return None
        host = self.out.cpu().numpy()                          # the one D2H
        counters, sels = None, []
        for rk in range(self.world):
            blk = host[rk * self.size:(rk + 1) * self.size]
            hv = blk[:self.HEAD].view(np.int64)
            counters = [int(x) for x in hv[:5]] if counters is None else counters
            counters = [a + int(c) for a, c in zip(counters, hv[5:10])]
            at = self.HEAD
            for f, r0, n in self.metas[rk]:
                nb = (n + 7) // 8
                sels.append((f, r0, n, blk[at:at + nb].copy()))
                at += nb
        sels.sort(key=lambda x: (x[0], x[1]))
        return tuple(counters), sels


def unit_layout(rg_rows, units):
    """(file, first row, rows) per planned unit [(file, first rg, end rg)] of plan_units, over the
    row counts per row group of every file (no pruning)."""
    out = []
    for f, a, b in units:
        out.append((f, sum(rg_rows[f][:a]), sum(rg_rows[f][a:b])))
    return out


def gather(output: ShardOutput, group=None):
    """All ranks' outputs on rank 0 (None elsewhere), over torch.distributed (gloo or RCCL)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bucket = [None] * world if dist.get_rank(group) == 0 else None
    dist.gather_object(output, bucket, dst=0, group=group)
    return bucket


def gpu_shard_scan(engine, snapshot, world: int, rank: int, with_stats: bool = False):
    """Run this rank's share of getScanFiles on its GPU. Returns (ShardOutput whose payloads are
    FilteredColumnarBatches with columns fetched on demand, the scan to close() when done)."""
    scan = snapshot.getScanBuilder().withStats(with_stats).withShard(world, rank).build()
    batches = list(scan.getScanFiles(engine))
    out = ShardOutput(rank, scan.tail_metrics.as_tuple(), scan.ckpt_metrics.as_tuple())
    for b in batches:
        if b.file_index < 0:
            out.tail = b
        else:
            out.files[(b.file_index, b.row_offset)] = b
    return out, scan


def scan_units(scan, device_bits=False):
    """This rank's (file index, first row, rows, packed selection bits) after scan.run() + sync():
    bits packed on the GPU, into a torch device tensor when device_bits (for RCCL), else host."""
    import numpy as np
    units = []
    for fi in range(len(scan.ckpt_files or [])):
        n = scan.ckpt.num_rows(fi)
        units.append((scan.ckpt_index[fi], scan.ckpt.row_offset(fi), n, scan.selection_bits(fi, device=device_bits)))
    return units


# ------------------------------------------------------------------------------------------------
# hash(path)-owner exchange ("alltoall" mode)
#
# delta-spark reconciles a snapshot by repartitioning every action by its path
# (spark/.../Snapshot.scala:478-483, repartition(coalesce(add.path, remove.path))). Here each rank
# decodes its row-group shard of the checkpoint; every add row with a fast-path key hash is routed
# as an 8-byte record {path hash} to its owner rank, path_owner(hash, world); the owner holds the
# commit-tail path hashes of its share and answers one byte per record (1: a tail key with that path
# hash exists); answers return in send order by the reverse all-to-all, and the origin selects the
# rows answered 0 and runs the exact key probe on the rest (dk_replay_exchange_*).
# ------------------------------------------------------------------------------------------------
def path_owner(path_hash: int, world: int) -> int:
    """The rank that owns a key: its canonical-path hash (seed 0, dk_uri.h) modulo the world size
    (a2a_owner in dk_kernels.hip)."""
    return int(path_hash % world)


class ExchangeSide:
    """One rank's side of the exchange over a GpuScan's replay (device buffers: torch tensors on the
    scan's GPU, filled and read by libdkgpu)."""

    def __init__(self, scan):
        import torch
        self.scan = scan
        self.world, self.rank = scan.shard
        self.device = torch.device("cuda", torch.cuda.current_device())

    def counts(self):
        import ctypes as C
        import numpy as np
        from ._lib import check, lib
        c = np.zeros(self.world, np.int64)
        check(lib().dk_replay_exchange_counts(self.scan._rh, c.ctypes.data_as(C.POINTER(C.c_int64))))
        return c

    def pack(self, n):
        import ctypes as C
        import torch
        from ._lib import check, lib
        send = torch.empty(max(1, n), dtype=torch.int64, device=self.device)
        check(lib().dk_replay_exchange_pack(self.scan._rh, C.c_void_p(send.data_ptr())))
        return send[:n]

    def filter(self, recv):
        import ctypes as C
        import torch
        from ._lib import check, lib
        recv = recv.to(self.device).contiguous()
        flags = torch.empty(max(1, recv.numel()), dtype=torch.uint8, device=self.device)
        torch.cuda.current_stream().synchronize()           # the received records have landed
        check(lib().dk_replay_exchange_filter(self.scan._rh, C.c_void_p(recv.data_ptr()), recv.numel(),
                                              C.c_void_p(flags.data_ptr())))
        return flags[:recv.numel()]

    def finish(self, back):
        import ctypes as C
        import torch
        from ._lib import check, lib
        back = back.to(self.device).contiguous()
        torch.cuda.current_stream().synchronize()
        check(lib().dk_replay_exchange_finish(self.scan._rh, C.c_void_p(back.data_ptr())))
        self._keep = back                                    # alive until the replay has read it


def exchange_hash_owner(side, group=None, device=None):
    """Drive one exchange for this rank over torch.distributed: sizes, records (all_to_all_single),
    the owners' answers back (the reverse all_to_all_single). device: where the collective's tensors
    live -- "cuda" for RCCL over xGMI, None / "cpu" for gloo. Returns the bytes this rank sent."""
    import torch
    import torch.distributed as dist
    dev = torch.device(device) if device is not None else torch.device("cpu")
    counts = side.counts()
    n_send = int(counts.sum())
    send = side.pack(n_send).to(dev)
    c = torch.tensor(counts, dtype=torch.int64, device=dev)
    rc = torch.empty_like(c)
    dist.all_to_all_single(rc, c, group=group)
    rcl = [int(x) for x in rc.cpu().tolist()]
    recv = torch.empty(max(1, sum(rcl)), dtype=torch.int64, device=dev)[:sum(rcl)]
    dist.all_to_all_single(recv, send, output_split_sizes=rcl, input_split_sizes=[int(x) for x in counts], group=group)
    flags = side.filter(recv).to(dev)
    back = torch.empty(max(1, n_send), dtype=torch.uint8, device=dev)[:n_send]
    dist.all_to_all_single(back, flags, output_split_sizes=[int(x) for x in counts], input_split_sizes=rcl, group=group)
    side.finish(back)
    return 9 * n_send


def exchange_local(sides):
    """The same exchange between ranks simulated in one process (every side's counts / pack first,
    then every owner's filter, then every origin's finish): tests and single-GPU rehearsals."""
    import torch
    world = len(sides)
    counts = [s.counts() for s in sides]
    sends = [s.pack(int(c.sum())) for s, c in zip(sides, counts)]
    offs = [[0] + list(torch.cumsum(torch.tensor(c), 0).tolist()) for c in counts]
    flags = []
    for o in range(world):
        recv = torch.cat([sends[s][offs[s][o]:offs[s][o + 1]].to(sends[o].device if sends[o].numel() else sends[s].device)
                          for s in range(world)]) if world else None
        flags.append((sides[o].filter(recv), [int(counts[s][o]) for s in range(world)]))
    for s in range(world):
        parts = []
        for o in range(world):
            f, seg = flags[o]
            a = sum(seg[:s])
            parts.append(f[a:a + seg[s]].to(sends[s].device))
        sides[s].finish(torch.cat(parts) if parts else torch.zeros(0, dtype=torch.uint8))


# ------------------------------------------------------------------------------------------------
# owner-partitioned reconciliation ("owner" mode)
#
# delta-spark repartitions ALL actions by path and resolves each partition with one owner
# (spark/src/main/scala/org/apache/spark/sql/delta/Snapshot.scala:476-485). Here the key
# (URI(path), dvUniqueId) with hash h belongs to rank h mod world. Every rank parses only the commit
# files j = rank (mod world) (their batches renumbered in the global replay order) and decodes only
# its row groups of the checkpoint; three exchanges resolve everything exactly:
#   1. commit-tail key records (32 B + the canonical key bytes) to their owners; each owner builds
#      the table of its keys and selects the actions routed to it (R2-R5); the answers come back;
#   2. every checkpoint row's 8-byte key hash to its owner; a hash no owned tail key has decides the
#      row (selected); the rest come back as candidates;
#   3. the candidates' canonical keys to their owners, answered byte-exactly (selected / duplicate /
#      tombstoned).
# The protocol and its collectives run inside libdkgpu (dk_replay_owner_run over a dk_comm,
# delta_amd/csrc/dk_comm.cpp): RCCL over xGMI, a caller's transport through callbacks, or the ranks of
# one process. No rank holds the whole commit tail; the ScanMetrics counters are summed over the ranks.
# ------------------------------------------------------------------------------------------------
REC_BYTES = 32                      # dk OwnerKeyRec


class OwnerPeerError(RuntimeError):
    """Another rank of the owner exchange failed (its own error is raised on that rank)."""


def _ptr_array(ptr, n, dtype):
    import ctypes as C
    import numpy as np
    if n <= 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,))


class OwnerComm:
    """One rank's dk_comm: ScanBuilder.withShard(world, rank, owner=OwnerComm...). The scan's
    prepare() all-reduces the commit files' batch counts through it (global_steps), run() hands the
    replay to dk_replay_owner_run, which runs the three exchanges and their votes in the library.
    Build with OwnerComm.rccl (RCCL over xGMI, the product), OwnerComm.over_torch (callbacks over a
    torch.distributed group: gloo on the CPU) or OwnerComm.local (every rank in this process)."""

    def __init__(self, handle, world, rank, keep=(), steps=None):
        self._h = handle
        self.world, self.rank = int(world), int(rank)
        self._keep = keep               # ctypes callbacks the library holds
        self._steps = steps             # local ranks: the global batch counts, known up front
        self.ms = {}
        self.bytes_sent = 0

    # ---- construction
    @classmethod
    def rccl(cls, group=None, device=None):
        """RCCL communicator over xGMI owned by libdkgpu; the 128-byte unique id goes from the
        group's first rank to the others over torch.distributed (a JVM host would use its own RPC)."""
        import ctypes as C
        import torch
        import torch.distributed as dist
        from ._lib import COMM_ID_BYTES, check, lib
        single = not (dist.is_available() and dist.is_initialized())     # one rank, no process group
        world, rank = (1, 0) if single else (dist.get_world_size(group), dist.get_rank(group))
        uid = (C.c_uint8 * COMM_ID_BYTES)()
        if rank == 0:
            check(lib().dk_comm_unique_id(uid))
        if not single:
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
            uid = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(box[0])
        dev = torch.cuda.current_device() if device is None else int(device)
        h = C.c_void_p()
        check(lib().dk_comm_create(uid, world, rank, dev, C.byref(h)))
        return cls(h, world, rank)

    @classmethod
    def over_torch(cls, group=None):
        """Callback transport over a torch.distributed group, host tensors (gloo)."""
        import ctypes as C
        import numpy as np
        import torch
        import torch.distributed as dist
        from ._lib import A2A_FN, ALLREDUCE_FN, check, dk_comm_callbacks, lib
        world, rank = dist.get_world_size(group), dist.get_rank(group)

        def a2a(_u, send, sbytes, recv, rbytes):
            try:
                sb = [int(sbytes[i]) for i in range(world)]
                rb = [int(rbytes[i]) for i in range(world)]
                st = torch.from_numpy(_ptr_array(send, sum(sb), np.uint8).copy())
                rt = torch.empty(sum(rb), dtype=torch.uint8)
                dist.all_to_all_single(rt, st, output_split_sizes=rb, input_split_sizes=sb, group=group)
                if sum(rb):
                    C.memmove(recv, rt.numpy().ctypes.data, sum(rb))
                return 0
            except BaseException:            # noqa: BLE001 -- reported as the callback's status
                return 1

        def allreduce(_u, vals, n, op):
            try:
                t = torch.from_numpy(_ptr_array(vals, n, np.int64).copy())
                dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX, group=group)
                C.memmove(vals, t.numpy().ctypes.data, 8 * n)
                return 0
            except BaseException:            # noqa: BLE001
                return 1
        cb = dk_comm_callbacks(None, A2A_FN(a2a), ALLREDUCE_FN(allreduce))
        h = C.c_void_p()
        check(lib().dk_comm_create_callbacks(C.byref(cb), world, rank, C.byref(h)))
        return cls(h, world, rank, keep=(cb,))

    @classmethod
    def local(cls, world, steps=None, on_device=True):
        """`world` ranks in this process (one thread each: run_local), exchanging through memory.
        steps: the commit files' global batch counts (LocalOwners.for_table), as their all-reduce
        would give them (the scans are prepared one after another)."""
        import ctypes as C
        from ._lib import check, lib
        hs = (C.c_void_p * world)()
        check(lib().dk_comm_create_local(world, 1 if on_device else 0, hs))
        return [cls(C.c_void_p(hs[r]), world, r, steps=steps) for r in range(world)]

    @staticmethod
    def table_steps(engine, snapshot):
        """Batches of every commit file (and JSON manifest part) from one parse of the whole tail."""
        import ctypes as C
        from ._lib import check, lib
        from .kernel import JsonTail
        commits = list(reversed(snapshot.log_segment.deltas))
        parts = snapshot._json_checkpoint_parts()
        t = JsonTail(engine, [d.path for d in commits], [d.version for d in commits], False, checkpoint_paths=parts)
        n = len(commits) + len(parts)
        steps = (C.c_int32 * max(1, n))()
        check(lib().dk_json_tail_file_steps(t._h, steps))
        t.close()
        return [steps[i] for i in range(n)]

    # ---- the scan's calls
    def _status(self, rc, side_error=None):
        from ._lib import STATUS_PEER, DkError, lib
        if rc == 0:
            return
        msg = lib().dk_last_error().decode("utf-8", "replace")
        if rc == STATUS_PEER:
            raise OwnerPeerError(msg)
        if side_error is not None:
            raise side_error
        raise DkError(msg)

    def global_steps(self, local, failed=False):
        """Batches of every commit file (replay order): this rank's counts summed over the ranks.
        Called from the scan's commit-tail thread. A rank whose commit-tail parse failed still takes
        part (failed=True, its counts zero) so that no peer waits for it: every rank then raises
        (in the reference every reader of the log sees the parse error)."""
        import numpy as np
        from ._lib import lib
        if self._steps is not None:
            return np.asarray(self._steps, dtype=np.int64)
        v = np.concatenate([np.asarray(local, dtype=np.int64).ravel(), [1 if failed else 0]]).astype(np.int64)
        import ctypes as C
        self._status(lib().dk_comm_allreduce_i64(self._h, v.ctypes.data_as(C.POINTER(C.c_int64)), len(v), 0))
        if v[-1] and not failed:
            raise OwnerPeerError("owner exchange: the commit-tail parse failed on another rank")
        return v[:-1]

    def abort(self):
        """A rank that fails after global_steps (checkpoint open, replay setup) answers the owner
        run's first vote with its error bit instead of running it, so its peers raise too."""
        from ._lib import lib
        if self._steps is None:
            self._status(lib().dk_comm_abort(self._h))

    def _last_run(self):
        import ctypes as C
        from ._lib import lib
        ms, b, n = (C.c_double * 8)(), C.c_int64(), C.c_int64()
        lib().dk_comm_last_run(self._h, ms, C.byref(b), C.byref(n))
        self.ms = {"tail_exchange": ms[0], "decode_hash": ms[1], "row_exchange": ms[2], "total": ms[3],
                   "tail_local": ms[4], "decode_local": ms[5], "row_local": ms[6], "collectives": ms[7]}
        self.bytes_sent = int(b.value)
        self.collectives = int(n.value)
        st = (C.c_double * 16)()
        lib().dk_comm_last_steps(self._h, st)
        names = ("begin", "tail_counts", "tail_pack", "tail_resolve", "reseed", "tail_finish", "run", "ckpt_counts",
                 "ckpt_pack", "ckpt_lookup", "ckpt_apply", "cand_counts", "cand_pack", "cand_verify", "cand_finish")
        self.steps_ms = {k: st[i] for i, k in enumerate(names)}

    def run_scan(self, scan):
        """The whole owner protocol of one scan run on this rank (dk_replay_owner_run)."""
        from ._lib import lib
        rc = lib().dk_replay_owner_run(scan._rh, self._h)
        self._last_run()
        self._status(rc)

    def run_side(self, side):
        """The same protocol over a Python stand-in for the device side (tests): `side` has the
        dk_owner_side calls with CPU torch tensors (tests/test_owner.py: CpuOwnerSide)."""
        import ctypes as C
        from ._lib import dk_owner_side, lib
        ad = _SideAdapter(side)
        rc = lib().dk_owner_protocol_run(C.byref(ad.struct), self._h)
        self._last_run()
        self._status(rc, ad.error)

    def close(self):
        from ._lib import lib
        if self._h:
            lib().dk_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:                    # noqa: BLE001 -- interpreter shutdown
            pass


class _SideAdapter:
    """dk_owner_side over a Python object whose calls take and return CPU torch tensors (the layout
    of the device calls: 32-byte key records, key bytes, 8-byte row hashes, one answer byte each)."""

    def __init__(self, side):
        import ctypes as C
        import numpy as np
        import torch
        from ._lib import SIDE_FNS, dk_owner_side
        self.side, self.error = side, None
        st = {}

        def guard(f):
            def g(*a):
                try:
                    return int(f(*a) or 0)
                except BaseException as e:      # noqa: BLE001 -- re-raised after the protocol returns
                    if self.error is None:
                        self.error = e
                    return 1
            return g

        def put(ptr, t):
            t = t.contiguous().view(torch.uint8).numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
            if t.nbytes:
                C.memmove(ptr, t.ctypes.data, t.nbytes)

        def u8(ptr, n):
            return torch.from_numpy(_ptr_array(ptr, n, np.uint8).copy())

        def counts2(ptr_a, ptr_b, key, fn):
            a, b = fn()
            st[key] = (int(np.sum(a)), int(np.sum(b)))
            for i in range(len(a)):
                ptr_a[i], ptr_b[i] = int(a[i]), int(b[i])

        def tail_pack(_u, recs, keys):
            r, k = side.tail_pack(*st["tail"])
            put(recs, r); put(keys, k)

        def tail_resolve(_u, recs, n, keys, nb, ans, flags):
            a, f = side.tail_resolve(u8(recs, n * REC_BYTES), u8(keys, nb))
            put(ans, a.to(torch.uint8))
            flags[0] = int(f)

        def ckpt_counts(_u, c):
            v = side.ckpt_counts()
            st["ckpt"] = int(np.sum(v))
            for i in range(len(v)):
                c[i] = int(v[i])

        def cand_pack(_u, recs, keys):
            r, k = side.cand_pack(*st["cand"])
            put(recs, r); put(keys, k)

        impl = {
            "begin": lambda _u: side.begin(),
            "tail_counts": lambda _u, a, b: counts2(a, b, "tail", side.tail_counts),
            "tail_pack": tail_pack,
            "tail_resolve": tail_resolve,
            "reseed": lambda _u: side.reseed(),
            "tail_finish": lambda _u, back: side.tail_finish(u8(back, st["tail"][0])),
            "run": lambda _u: side.run(),
            "ckpt_counts": ckpt_counts,
            "ckpt_pack": lambda _u, send: put(send, side.ckpt_pack(st["ckpt"])),
            "ckpt_lookup": lambda _u, recv, n, flags: put(flags, side.ckpt_lookup(
                torch.from_numpy(_ptr_array(recv, n, np.int64).copy())).to(torch.uint8)),
            "ckpt_apply": lambda _u, back: side.ckpt_apply(u8(back, st["ckpt"])),
            "cand_counts": lambda _u, a, b: counts2(a, b, "cand", side.cand_counts),
            "cand_pack": cand_pack,
            "cand_verify": lambda _u, recs, n, keys, nb, ans: put(ans, side.cand_verify(
                u8(recs, n * REC_BYTES), u8(keys, nb)).to(torch.uint8)),
            "cand_finish": lambda _u, back: side.cand_finish(u8(back, st["cand"][0])),
        }
        self._fns = [ftype(guard(impl[name])) for name, ftype in SIDE_FNS]
        self.struct = dk_owner_side(None, 0, *self._fns)


def run_local(scans):
    """Every scan's run() (each with its OwnerComm.local rank) on its own thread, then sync():
    the ranks of one process exchange through the library's in-process transport."""
    import threading
    errs = [None] * len(scans)

    def go(i):
        try:
            scans[i].run()
        except BaseException as e:           # noqa: BLE001 -- re-raised below
            errs[i] = e
    ts = [threading.Thread(target=go, args=(i,), daemon=True) for i in range(len(scans))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    for sc in scans:
        sc.sync()
