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
# No rank holds the whole commit tail; the ScanMetrics counters are summed over the ranks.
# ------------------------------------------------------------------------------------------------
REC_BYTES = 32                      # dk OwnerKeyRec
COLLISION = 4                       # dk E_COLLISION: a 64-bit hash collision at an owner
ERR_BIT = 1 << 20                   # vote bit: a rank failed at this step


class OwnerPeerError(RuntimeError):
    """Another rank of the owner exchange failed (its own error is raised on that rank)."""


class OwnerSide:
    """One rank's side of the owner-partitioned reconciliation over a GpuScan's replay. Buffers are
    torch uint8 / int64 tensors on the scan's GPU; every library call returns with its stream
    drained."""

    def __init__(self, scan):
        import torch
        self.scan = scan
        self.world, self.rank = scan.shard
        self.rh = scan._rh
        self.device = torch.device("cuda", torch.cuda.current_device())

    def _lib(self):
        from ._lib import check, lib
        return check, lib()

    def _buf(self, n, dtype=None):
        import torch
        return torch.empty(max(1, n), dtype=dtype or torch.uint8, device=self.device)[:n]

    def _in(self, t):
        import torch
        t = t.to(self.device).contiguous()
        torch.cuda.current_stream().synchronize()          # the collective's data has landed
        return t

    def begin(self):
        check, L = self._lib()
        check(L.dk_replay_owner_begin(self.rh))

    def tail_counts(self):
        import ctypes as C
        import numpy as np
        check, L = self._lib()
        recs, nbytes = np.zeros(self.world, np.int64), np.zeros(self.world, np.int64)
        check(L.dk_replay_owner_tail_counts(self.rh, recs.ctypes.data_as(C.POINTER(C.c_int64)),
                                            nbytes.ctypes.data_as(C.POINTER(C.c_int64))))
        return recs, nbytes

    def tail_pack(self, n, nbytes):
        import ctypes as C
        check, L = self._lib()
        recs, keys = self._buf(n * REC_BYTES), self._buf(nbytes)
        check(L.dk_replay_owner_tail_pack(self.rh, C.c_void_p(recs.data_ptr()), C.c_void_p(keys.data_ptr())))
        return recs, keys

    def tail_resolve(self, recs, keys):
        import ctypes as C
        check, L = self._lib()
        recs, keys = self._in(recs), self._in(keys)
        n = recs.numel() // REC_BYTES
        ans, flags = self._buf(n), C.c_int32(0)
        check(L.dk_replay_owner_tail_resolve(self.rh, C.c_void_p(recs.data_ptr()), n, C.c_void_p(keys.data_ptr()),
                                             keys.numel(), C.c_void_p(ans.data_ptr()), C.byref(flags)))
        return ans, int(flags.value)

    def reseed(self):
        check, L = self._lib()
        check(L.dk_replay_owner_reseed(self.rh))

    def tail_finish(self, back):
        import ctypes as C
        check, L = self._lib()
        back = self._in(back)
        check(L.dk_replay_owner_tail_finish(self.rh, C.c_void_p(back.data_ptr())))

    def run(self):
        check, L = self._lib()
        check(L.dk_replay_run(self.rh))

    def ckpt_counts(self):
        import ctypes as C
        import numpy as np
        check, L = self._lib()
        c = np.zeros(self.world, np.int64)
        check(L.dk_replay_owner_ckpt_counts(self.rh, c.ctypes.data_as(C.POINTER(C.c_int64))))
        return c

    def ckpt_pack(self, n):
        import ctypes as C
        import torch
        check, L = self._lib()
        send = self._buf(n, torch.int64)
        check(L.dk_replay_owner_ckpt_pack(self.rh, C.c_void_p(send.data_ptr())))
        return send

    def ckpt_lookup(self, recv):
        import ctypes as C
        check, L = self._lib()
        recv = self._in(recv)
        flags = self._buf(recv.numel())
        check(L.dk_replay_owner_ckpt_lookup(self.rh, C.c_void_p(recv.data_ptr()), recv.numel(),
                                            C.c_void_p(flags.data_ptr())))
        return flags

    def ckpt_apply(self, back):
        import ctypes as C
        check, L = self._lib()
        back = self._in(back)
        check(L.dk_replay_owner_ckpt_apply(self.rh, C.c_void_p(back.data_ptr())))

    def cand_counts(self):
        import ctypes as C
        import numpy as np
        check, L = self._lib()
        recs, nbytes = np.zeros(self.world, np.int64), np.zeros(self.world, np.int64)
        check(L.dk_replay_owner_cand_counts(self.rh, recs.ctypes.data_as(C.POINTER(C.c_int64)),
                                            nbytes.ctypes.data_as(C.POINTER(C.c_int64))))
        return recs, nbytes

    def cand_pack(self, n, nbytes):
        import ctypes as C
        check, L = self._lib()
        recs, keys = self._buf(n * REC_BYTES), self._buf(nbytes)
        check(L.dk_replay_owner_cand_pack(self.rh, C.c_void_p(recs.data_ptr()), C.c_void_p(keys.data_ptr())))
        return recs, keys

    def cand_verify(self, recs, keys):
        import ctypes as C
        check, L = self._lib()
        recs, keys = self._in(recs), self._in(keys)
        n = recs.numel() // REC_BYTES
        ans = self._buf(n)
        check(L.dk_replay_owner_cand_verify(self.rh, C.c_void_p(recs.data_ptr()), n, C.c_void_p(keys.data_ptr()),
                                            keys.numel(), C.c_void_p(ans.data_ptr())))
        return ans

    def cand_finish(self, back):
        import ctypes as C
        check, L = self._lib()
        back = self._in(back)
        check(L.dk_replay_owner_cand_finish(self.rh, C.c_void_p(back.data_ptr())))


class OwnerExchange:
    """The owner-partitioned reconciliation over torch.distributed (RCCL over xGMI when `device` is
    "cuda", gloo on the CPU): ScanBuilder.withShard(world, rank, owner=OwnerExchange(...)). Each
    step is timed into `ms` (phase -> milliseconds of the last run)."""

    def __init__(self, group=None, device=None):
        import torch
        self.group = group
        # "cuda" is pinned to this thread's current GPU now: global_steps runs on the scan's tail thread
        self.device = torch.device("cuda", torch.cuda.current_device()) if device == "cuda" else device
        self.ms = {}
        self.bytes_sent = 0

    def global_steps(self, local, failed=False):
        """Batches of every commit file (replay order): this rank's counts summed over the ranks.
        Called from the scan's commit-tail thread. A rank whose commit-tail parse failed still takes
        part (failed=True, its counts zero) so that no peer waits for it: every rank then raises
        (in the reference every reader of the log sees the parse error)."""
        import contextlib
        import numpy as np
        import torch
        import torch.distributed as dist
        dev = self._dev()
        v = np.concatenate([np.asarray(local, dtype=np.int64).ravel(), [1 if failed else 0]])
        with (torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()):
            t = torch.as_tensor(v, dtype=torch.int64).to(dev)
            dist.all_reduce(t, group=self.group)
            out = t.cpu().numpy()
        if out[-1] and not failed:
            raise OwnerPeerError("owner exchange: the commit-tail parse failed on another rank")
        return out[:-1]

    def abort(self):
        """A rank that fails after global_steps (checkpoint open, replay setup) answers the exchange's
        first vote with its error bit instead of running the exchange, so its peers raise too."""
        self._any(ERR_BIT)

    def _dev(self):
        import torch
        return torch.device(self.device) if self.device is not None else torch.device("cpu")

    def _a2a(self, send, send_counts, recv_counts=None):
        """all_to_all_single of a 1-D tensor cut into per-destination runs; recv_counts exchanged
        first unless given. Returns (received tensor on the transport device, recv_counts)."""
        import torch
        import torch.distributed as dist
        dev = self._dev()
        send = send.to(dev)
        sc = [int(x) for x in send_counts]
        if recv_counts is None:
            c = torch.tensor(sc, dtype=torch.int64, device=dev)
            rc = torch.empty_like(c)
            dist.all_to_all_single(rc, c, group=self.group)
            recv_counts = [int(x) for x in rc.cpu().tolist()]
        rcl = [int(x) for x in recv_counts]
        recv = torch.empty(max(1, sum(rcl)), dtype=send.dtype, device=dev)[:sum(rcl)]
        dist.all_to_all_single(recv, send, output_split_sizes=rcl, input_split_sizes=sc, group=self.group)
        self.bytes_sent += send.numel() * send.element_size()
        return recv, rcl

    def _any(self, flag):
        import torch
        import torch.distributed as dist
        t = torch.tensor([int(flag)], dtype=torch.int64, device=self._dev())
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def _step(self, fn):
        """Run this rank's local part of an exchange step, then vote on the MAX over ranks of the
        error bit: a local error, or any peer's, raises on every rank at the same step (a rank that
        raised before its next collective would leave its peers waiting in it)."""
        box = {}
        _, f = self._step_flag(lambda: box.__setitem__("out", fn()), {})
        return box.get("out"), f

    def __call__(self, side):
        import time
        t0 = time.perf_counter()
        self.bytes_sent = 0
        first = [True]
        while True:
            def pack():
                if first:
                    side.begin()
                    first.clear()
                recs_c, bytes_c = side.tail_counts()
                return (recs_c, bytes_c) + tuple(side.tail_pack(int(recs_c.sum()), int(bytes_c.sum())))
            (recs_c, bytes_c, recs, keys), _ = self._step(pack)
            rrecs, rrc = self._a2a(recs, recs_c * REC_BYTES)
            rkeys, _ = self._a2a(keys, bytes_c)
            box = {}

            def resolve():
                box["ans"], box["flag"] = side.tail_resolve(rrecs, rkeys)
            _, flag = self._step_flag(resolve, box)     # the collision vote carries the error bit
            if flag & COLLISION:                 # a hash collision at some owner: all ranks reseed
                side.reseed()
                continue
            back, _ = self._a2a(box["ans"], [c // REC_BYTES for c in rrc], recs_c)
            break
        t1 = time.perf_counter()

        def run_pack():
            side.tail_finish(back)
            side.run()
            c = side.ckpt_counts()
            return c, side.ckpt_pack(int(c.sum()))
        (c, send), _ = self._step(run_pack)
        t2 = time.perf_counter()
        recv, rc = self._a2a(send, c)
        flags, _ = self._step(lambda: side.ckpt_lookup(recv))
        back, _ = self._a2a(flags, rc, c)

        def apply_pack():
            side.ckpt_apply(back)
            cr, cb = side.cand_counts()
            return (cr, cb) + tuple(side.cand_pack(int(cr.sum()), int(cb.sum())))
        (cr, cb, recs, keys), _ = self._step(apply_pack)
        rrecs, rrc = self._a2a(recs, cr * REC_BYTES)
        rkeys, _ = self._a2a(keys, cb)
        ans, _ = self._step(lambda: side.cand_verify(rrecs, rkeys))
        back, _ = self._a2a(ans, [x // REC_BYTES for x in rrc], cr)
        side.cand_finish(back)
        t3 = time.perf_counter()
        self.ms = {"tail_exchange": (t1 - t0) * 1e3, "decode_hash": (t2 - t1) * 1e3, "row_exchange": (t3 - t2) * 1e3}

    def _step_flag(self, fn, box):
        """_step whose vote also carries the collision flag fn left in box["flag"]."""
        err = None
        try:
            fn()
        except BaseException as e:       # noqa: BLE001 -- re-raised after the vote
            err = e
        f = self._any(ERR_BIT if err is not None else int(box.get("flag", 0)))
        if f & ERR_BIT:
            if err is not None:
                raise err
            raise OwnerPeerError("owner exchange: another rank failed")
        return None, f


class OwnerLoopback:
    """The owner exchange between `world` scans in ONE process (tests and single-GPU rehearsals):
    the scans are prepared one after another (global_steps answers from the whole commit tail,
    counted once up front), then run() drives every side's exchanges in lockstep."""

    def __init__(self, global_steps):
        import numpy as np
        self._steps = np.asarray(global_steps, dtype=np.int64)
        self.sides = {}

    @classmethod
    def for_table(cls, engine, snapshot):
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
        return cls([steps[i] for i in range(n)])

    def global_steps(self, local, failed=False):
        return self._steps

    def abort(self):
        pass

    def __call__(self, side):
        self.sides[side.rank] = side       # run() drives them once every rank's side has arrived

    @staticmethod
    def _route(sends):
        """sends[s] = (1-D tensor, per-destination counts) -> per destination (concatenation over
        sources, per-source counts)."""
        import torch
        world = len(sends)
        out = []
        for d in range(world):
            parts, counts = [], []
            for s in range(world):
                t, cnt = sends[s]
                a = int(sum(cnt[:d]))
                parts.append(t[a:a + int(cnt[d])])
                counts.append(int(cnt[d]))
            dev = next((p.device for p in parts if p.numel()), sends[d][0].device)
            out.append((torch.cat([p.to(dev) for p in parts]) if parts else sends[d][0][:0], counts))
        return out

    def run(self, scans):
        """Every scan's run() with this loopback as its owner, then the exchanges in lockstep."""
        self.sides = {}
        for sc in scans:
            sc.run()                            # registers the side
        sides = [self.sides[r] for r in range(len(scans))]
        world = len(sides)
        for s in sides:
            s.begin()
        while True:
            cnts = [s.tail_counts() for s in sides]
            packed = [s.tail_pack(int(r.sum()), int(b.sum())) for s, (r, b) in zip(sides, cnts)]
            rrecs = self._route([(p[0], r * REC_BYTES) for p, (r, _) in zip(packed, cnts)])
            rkeys = self._route([(p[1], b) for p, (_, b) in zip(packed, cnts)])
            res = [sides[d].tail_resolve(rrecs[d][0], rkeys[d][0]) for d in range(world)]
            if any(f for _, f in res):
                for s in sides:
                    s.reseed()
                continue
            back = self._route([(res[d][0], [c // REC_BYTES for c in rrecs[d][1]]) for d in range(world)])
            for s in range(world):
                sides[s].tail_finish(back[s][0])
            break
        for s in sides:
            s.run()
        cs = [s.ckpt_counts() for s in sides]
        sends = [s.ckpt_pack(int(c.sum())) for s, c in zip(sides, cs)]
        recv = self._route([(t, c) for t, c in zip(sends, cs)])
        flags = [sides[d].ckpt_lookup(recv[d][0]) for d in range(world)]
        back = self._route([(flags[d], recv[d][1]) for d in range(world)])
        for s in range(world):
            sides[s].ckpt_apply(back[s][0])
        cc = [s.cand_counts() for s in sides]
        packed = [s.cand_pack(int(r.sum()), int(b.sum())) for s, (r, b) in zip(sides, cc)]
        rrecs = self._route([(p[0], r * REC_BYTES) for p, (r, _) in zip(packed, cc)])
        rkeys = self._route([(p[1], b) for p, (_, b) in zip(packed, cc)])
        ans = [sides[d].cand_verify(rrecs[d][0], rkeys[d][0]) for d in range(world)]
        back = self._route([(ans[d], [c // REC_BYTES for c in rrecs[d][1]]) for d in range(world)])
        for s in range(world):
            sides[s].cand_finish(back[s][0])
        for sc in scans:
            sc.sync()
