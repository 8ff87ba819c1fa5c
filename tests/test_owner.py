"""Owner-partitioned reconciliation, the multi-GPU "owner" mode (the protocol and its collectives in
libdkgpu: dk_replay_owner_run / dk_owner_protocol_run over a dk_comm, delta_amd/csrc/dk_comm.cpp;
delta_amd/shard.py: OwnerComm).

Each rank parses only the commit files j = rank (mod world) and decodes only its row groups of the
checkpoint; the key (URI(path), dvUniqueId) with hash h is owned by rank h mod world, which resolves
the commit-tail actions routed to it (R2-R5, App. A) and answers every rank's checkpoint rows for its
keys, first by hash, then byte-exactly.

CPU: gloo worlds 2 and 3 drive the library's protocol (dk_owner_protocol_run: global batch steps,
three all-to-all exchanges, the votes) through the callback transport (dk_comm_create_callbacks over
gloo) over a CPU stand-in for the device side (CpuOwnerSide: the oracle's JSON decode and canonical
keys, the same record layout, the owner rules restated), reassembled against the unsharded oracle
replay; a forced collision round checks the reseed vote; the in-process transport
(dk_comm_create_local) does the same with one thread per rank.
GPU: the product's owner mode (dk_replay_owner_run) for 2 and 3 ranks in one process over the
in-process transport equals the oracle -- rows in the reference order, counters -- including DV
swaps, checkpoint removes, JSON batch boundaries inside a commit (R5) and a data-skipping filter; a
one-rank RCCL communicator created through the C ABI does too.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from delta_amd import shard, synth

HERE = os.path.dirname(os.path.abspath(__file__))
REC = np.dtype([("h", "<u8"), ("kind", "<i4"), ("step", "<i4"), ("row", "<i4"), ("key_len", "<i4"),
                ("canon_len", "<i4"), ("src", "<i4")])
ADD, REMOVE = 1, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _h(key: bytes, seed: int) -> int:
    return int.from_bytes(hashlib.blake2b(key, digest_size=8, key=seed.to_bytes(4, "little")).digest(), "little") | 1


class CpuOwnerSide:
    """CPU stand-in for shard.OwnerSide: the same calls, buffers in the same layouts (CPU torch
    tensors), keys from the oracle (ref.action_key), the owner's rules restated in Python."""

    def __init__(self, table, world, rank, owner, bs=1024, collide_first=False, fail=None):
        import torch  # noqa: F401
        from delta_amd import kernel as K
        from oracle import ref
        self.world, self.rank, self.bs = world, rank, bs
        self.seed = 0
        self.collide = collide_first
        seg = ref.load_log_segment(table)
        commits = [f for f in seg.all_files_reversed() if f.kind == "commit"]
        mine = [j for j in range(len(commits)) if j % world == rank]
        batches = {j: list(ref.read_json_batches(commits[j].path, bs)) for j in mine}
        local = np.zeros(len(commits), np.int64)
        for j in mine:
            local[j] = len(batches[j])
        self.fail = fail
        if fail == "parse":                      # this rank's commit parse failed: vote, then raise
            owner.global_steps(local * 0, failed=True)
            raise ValueError("malformed commit")
        step0 = np.concatenate([[0], np.cumsum(owner.global_steps(local))])
        self.acts = []            # (kind, step, row, key, tail row id (commit, line))
        for j in mine:
            for b, batch in enumerate(batches[j]):
                for i, row in enumerate(batch):
                    for kind, name in ((REMOVE, "remove"), (ADD, "add")):
                        if row[name] is not None:
                            self.acts.append((kind, int(step0[j]) + b, i, ref.json_key(row[name]), (j, b * bs + i)))
        # this rank's checkpoint rows (row-group shard, replay order)
        full = ref.replay(table, json_batch_size=bs)
        self.full = full
        files = [x.path for x in full.checkpoint]
        rgs = [K.row_group_rows(p) for p in files]
        self.units = shard.unit_layout(rgs, shard.plan_units(rgs, world, rank))
        self.rows = []            # (file, row, key or None)
        for f, r0, n in self.units:
            pf = ref.ParquetFile.open(files[f])
            cols = {leaf: pf.read(leaf) for leaf in ref.ADD_LEAVES}
            pc = cols["add.path"]
            for r in range(r0, r0 + n):
                if pc.row_def[r] < pc.max_def:
                    self.rows.append((f, r, None))
                    continue
                row = ref.canon_add_from_cols(cols, r)
                dv = None if row[5] is None else row[5][:3]
                self.rows.append((f, r, ref.action_key(row[0], dv)))
        self.counters = [0] * 5

    # ---- commit tail
    def begin(self):
        self.counters = [0] * 5

    def _owner(self, key):
        return _h(key, self.seed) % self.world

    def tail_counts(self):
        self.sent = sorted(range(len(self.acts)), key=lambda i: self._owner(self.acts[i][3]))
        recs = np.zeros(self.world, np.int64)
        nbytes = np.zeros(self.world, np.int64)
        for i in self.sent:
            o = self._owner(self.acts[i][3])
            recs[o] += 1
            nbytes[o] += len(self.acts[i][3])
        return recs, nbytes

    def tail_pack(self, n, nbytes):
        import torch
        r = np.zeros(n, REC)
        keys = b""
        for pos, i in enumerate(self.sent):
            kind, step, row, key, _ = self.acts[i]
            r[pos] = (_h(key, self.seed), kind, step, row, len(key), len(key), i)
            keys += key
        return torch.from_numpy(r.view(np.uint8).copy()), torch.from_numpy(np.frombuffer(keys or b"\0", np.uint8)[:nbytes].copy())

    def tail_resolve(self, recs, keys):
        import torch
        r = recs.numpy().view(REC)
        kb = keys.numpy().tobytes()
        assert all(int(x["h"]) % self.world == self.rank for x in r)
        off, items = 0, []
        for x in r:
            items.append((int(x["kind"]), int(x["step"]), int(x["row"]), kb[off:off + int(x["key_len"])]))
            off += int(x["key_len"])
        assert off == len(kb)
        if self.collide:                         # the first round reports a collision on one owner
            self.collide = False
            return torch.zeros(len(items), dtype=torch.uint8), (4 if self.rank == 0 else 0)
        self.table = {}                          # key -> [first add (step, row) or None, min remove step]
        for kind, step, row, key in items:
            t = self.table.setdefault(key, [None, 1 << 62])
            if kind == ADD:
                t[0] = (step, row) if t[0] is None else min(t[0], (step, row))
            else:
                t[1] = min(t[1], step)
        ans = []
        for kind, step, row, key in items:
            if kind != ADD:
                self.counters[4] += 1
                ans.append(0)
                continue
            t = self.table[key]
            dup = t[0] != (step, row)
            chosen = not dup and t[1] > step
            self.counters[0] += 1
            self.counters[1] += 1
            self.counters[2] += chosen
            self.counters[3] += dup
            ans.append(1 if chosen else 0)
        return torch.tensor(ans, dtype=torch.uint8), 0

    def reseed(self):
        self.seed += 1
        self.counters = [0] * 5

    def tail_finish(self, back):
        b = back.numpy()
        assert len(b) == len(self.sent)
        self.tail_sel = {self.acts[i][4]: bool(v) for i, v in zip(self.sent, b) if self.acts[i][0] == ADD}

    # ---- checkpoint
    def run(self):
        pass

    def ckpt_counts(self):
        self.routed = sorted((i for i, x in enumerate(self.rows) if x[2] is not None),
                             key=lambda i: self._owner(self.rows[i][2]))
        c = np.zeros(self.world, np.int64)
        for i in self.routed:
            c[self._owner(self.rows[i][2])] += 1
        self.counters[0] += len(self.routed)
        return c

    def ckpt_pack(self, n):
        import torch
        assert n == len(self.routed)
        return torch.tensor([np.int64(np.uint64(_h(self.rows[i][2], self.seed))) for i in self.routed], dtype=torch.int64)

    def ckpt_lookup(self, recv):
        import torch
        if self.fail == "lookup":
            raise ValueError("lookup failed")
        hs = {_h(k, self.seed) for k in self.table}
        return torch.tensor([1 if int(np.uint64(np.int64(x))) in hs else 0 for x in recv.tolist()], dtype=torch.uint8)

    def ckpt_apply(self, back):
        b = back.numpy()
        self.sel = {(f, r): False for f, r, _ in self.rows}
        self.cands = []
        for i, v in zip(self.routed, b):
            f, r, _ = self.rows[i]
            if v == 0:
                self.sel[(f, r)] = True
                self.counters[2] += 1
            else:
                self.cands.append(i)

    def cand_counts(self):
        self.cands.sort(key=lambda i: self._owner(self.rows[i][2]))
        recs, nbytes = np.zeros(self.world, np.int64), np.zeros(self.world, np.int64)
        for i in self.cands:
            o = self._owner(self.rows[i][2])
            recs[o] += 1
            nbytes[o] += len(self.rows[i][2])
        return recs, nbytes

    def cand_pack(self, n, nbytes):
        import torch
        r = np.zeros(n, REC)
        keys = b""
        for pos, i in enumerate(self.cands):
            key = self.rows[i][2]
            r[pos] = (_h(key, self.seed), 3, 0, 0, len(key), len(key), pos)
            keys += key
        return torch.from_numpy(r.view(np.uint8).copy()), torch.from_numpy(np.frombuffer(keys or b"\0", np.uint8)[:nbytes].copy())

    def cand_verify(self, recs, keys):
        import torch
        r = recs.numpy().view(REC)
        kb = keys.numpy().tobytes()
        off, ans = 0, []
        for x in r:
            key = kb[off:off + int(x["key_len"])]
            off += int(x["key_len"])
            t = self.table.get(key)
            ans.append(0 if t is None else (1 if t[0] is not None else 2))
        return torch.tensor(ans, dtype=torch.uint8)

    def cand_finish(self, back):
        for i, v in zip(self.cands, back.numpy()):
            f, r, _ = self.rows[i]
            self.sel[(f, r)] = v == 0
            self.counters[2] += v == 0
            self.counters[3] += v == 1


def _gloo_worker(rank, world, port, table, out_path, bs, collide):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        ex = shard.OwnerComm.over_torch()
        side = CpuOwnerSide(table, world, rank, ex, bs=bs, collide_first=collide)
        ex.run_side(side)
        units = []
        for f, r0, n in side.units:
            bits = np.array([side.sel[(f, r)] for r in range(r0, r0 + n)], bool)
            units.append((f, r0, n, np.packbits(bits, bitorder="little")))
        counters, sels = shard.gather_selections(units, (0,) * 5, tuple(int(x) for x in side.counters))
        tails = [None] * world
        dist.all_gather_object(tails, sorted((k, v) for k, v in side.tail_sel.items() if v))
        res = {"rank": rank, "seed": side.seed, "bytes": ex.bytes_sent}
        if rank == 0:
            full = side.full
            ok = counters == full.counters.as_tuple()
            for b in full.checkpoint:
                parts = [s for s in sels if s[0] == b.file_index]
                bits = np.concatenate([np.unpackbits(s[3], bitorder="little")[:s[2]] for s in parts])
                ok = ok and np.array_equal(bits.astype(bool), b.selected.astype(bool))
            # the tail's selected adds, merged by (commit, line), are the oracle's json rows in order
            from oracle import ref
            seg = ref.load_log_segment(table)
            commits = [f for f in seg.all_files_reversed() if f.kind == "commit"]
            lines = {}
            for j, c in enumerate(commits):
                for b, batch in enumerate(ref.read_json_batches(c.path, bs)):
                    for i, row in enumerate(batch):
                        lines[(j, b * bs + i)] = row["add"]["path"] if row["add"] else None
            merged = sorted(k for t in tails for k, _ in t)
            ok = ok and [lines[tuple(k)] for k in merged] == [a["path"] for a in full.json_rows]
            res.update(ok=bool(ok), counters=list(counters), want=list(full.counters.as_tuple()))
        with open(out_path + ".%d" % rank, "w") as f:
            json.dump(res, f)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _gloo_fail_worker(rank, world, port, table, out_path, fail):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        ex = shard.OwnerComm.over_torch()
        err = None
        try:
            side = CpuOwnerSide(table, world, rank, ex, fail=fail if rank == world - 1 else None)
            if fail == "open" and rank == world - 1:
                ex.abort()                       # failed after global_steps (checkpoint open)
                raise ValueError("open failed")
            ex.run_side(side)
        except Exception as e:                   # noqa: BLE001
            err = type(e).__name__
        with open(out_path + ".%d" % rank, "w") as f:
            json.dump({"error": err}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail", ["parse", "open", "lookup"])
def test_gloo_owner_failure_on_one_rank(tmp_path, fail):
    """A failure on the last rank -- its commit-tail parse (at the global-steps vote), its checkpoint
    open (after it: the exchange's first vote), or an owner step inside the exchange -- raises on
    every rank; no rank is left waiting in a collective (the spawn would hang)."""
    import torch.multiprocessing as mp
    table = str(tmp_path / "t")
    synth.write_table(table, synth.TableSpec(n_adds=2_000, n_parts=2, row_group_size=500, n_commits=5,
                                             adds_per_commit=10, removes_per_commit=10))
    out = str(tmp_path / "res.json")
    mp.spawn(_gloo_fail_worker, args=(3, _free_port(), table, out, fail), nprocs=3, join=True)
    res = [json.load(open(out + ".%d" % r))["error"] for r in range(3)]
    assert res == ["OwnerPeerError", "OwnerPeerError", "ValueError"], res


@pytest.mark.parametrize("world,bs,collide", [(2, 1024, False), (3, 3, True)])
def test_gloo_owner_exchange(tmp_path, world, bs, collide):
    """gloo worlds 2 and 3: the product's owner-exchange driver with the CPU stand-in reassembles the
    oracle's scan files and counters; every rank parsed only its share of the commits; a collision
    vote reseeds every rank once."""
    import torch.multiprocessing as mp
    table = str(tmp_path / "t")
    synth.write_table(table, synth.TableSpec(n_adds=6_000, n_parts=3, row_group_size=1000, n_commits=7,
                                             adds_per_commit=20, removes_per_commit=20, dv_frac=0.15,
                                             ckpt_removes=30, readd_frac=0.2, dup_frac=0.1))
    out = str(tmp_path / "res.json")
    mp.spawn(_gloo_worker, args=(world, _free_port(), table, out, bs, collide), nprocs=world, join=True)
    res = [json.load(open(out + ".%d" % r)) for r in range(world)]
    assert res[0]["ok"], res[0]
    assert all(r["seed"] == (1 if collide else 0) for r in res), res
    assert all(r["bytes"] > 0 for r in res)


def _loopback_check(table, world, bs, predicate):
    """Body of test_gpu_owner_loopback, in a fresh process that imports torch before libdkgpu (the
    ranks' import order: both share torch's HIP runtime, which the exchange's device tensors need)."""
    import torch
    torch.cuda.init()
    from delta_amd import kernel as K
    from oracle import ref
    eng = K.GpuEngine(json_batch_size=bs)
    snap = K.Table.forPath(eng, table).getLatestSnapshot(eng)
    comms = shard.OwnerComm.local(world, steps=shard.OwnerComm.table_steps(eng, snap))
    scans = []
    for r in range(world):
        snap = K.Table.forPath(eng, table).getLatestSnapshot(eng)
        sb = snap.getScanBuilder()
        skipping = None
        if predicate:
            from delta_amd.expressions import Column, Literal, Predicate
            sb = sb.withFilter(Predicate(">", Column("id"), Literal.ofLong(predicate)))
            from tests.test_skipping import oracle_skipping
            skipping = oracle_skipping(table, Predicate(">", Column("id"), Literal.ofLong(predicate)))
        sc = sb.withShard(world, r, owner=comms[r]).build()
        sc.prepare(eng)
        scans.append(sc)
    full = ref.replay(table, json_batch_size=bs, with_stats=bool(predicate), skipping=skipping)
    n_commits = len(snap.log_segment.deltas)
    for sc in scans:                              # no rank parsed more than its share of the commits
        assert len(sc.tail_commits) <= -(-n_commits // world), (len(sc.tail_commits), n_commits)
    for step in range(2):                         # a second run reuses the replays
        shard.run_local(scans)
        counters = np.zeros(5, np.int64)
        tail, files = [], {}
        for sc in scans:
            counters += np.array(sc.metrics.as_tuple())
            for b in sc._batches():
                if b.file_index < 0:
                    tail.append(b)
                else:
                    files[(b.file_index, b.row_offset)] = b
        tail.sort(key=lambda b: b.commit_index)
        batches = tail + [files[k] for k in sorted(files)]
        rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in batches for i in b.selected_rows()]
        assert tuple(int(x) for x in counters) == full.counters.as_tuple(), (step, counters, full.counters.as_tuple())
        want = full.scan_files()
        if predicate:
            rows = [r[:-2] + r[-1:] for r in rows]          # the scan files without the stats column
            want = [r[:-2] + r[-1:] for r in want]
        assert rows == want, (step, len(rows), len(want))
    for sc in scans:
        sc.close()
    for c in comms:
        c.close()
    eng.close()
    print("ok")


@pytest.mark.gpu
@pytest.mark.parametrize("world,bs,spec,predicate", [
    (2, 1024, dict(n_parts=3, row_group_size=3000), None),
    (3, 3, dict(n_parts=1, row_group_size=2500, dv_frac=0.2, ckpt_removes=100, readd_frac=0.2, dup_frac=0.1), None),
    (2, 5, dict(n_parts=4, row_group_size=2000, dv_frac=0.3, with_stats=True), 8_000),
    (8, 1024, dict(n_parts=8, row_group_size=1000, compression="snappy", readd_frac=0.1, dup_frac=0.05), None),
])
def test_gpu_owner_loopback(tmp_path, world, bs, spec, predicate):
    """The product's owner mode (tail records routed and resolved by their owners, every checkpoint
    row's key hash routed, candidates verified byte-exactly on the device) for `world` ranks in one
    process, each rank's dk_replay_owner_run on its own thread over the in-process transport: merged
    rows (reference order) and counters equal the oracle's."""
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=20_000, n_commits=9, adds_per_commit=30,
                                                     removes_per_commit=30, **spec))
    root = os.path.dirname(HERE)
    code = ("import sys; sys.path.insert(0, %r); from tests.test_owner import _loopback_check; "
            "_loopback_check(%r, %d, %d, %r)" % (root, str(tmp_path), world, bs, predicate))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-4000:]


def _local_worker(rank, world, comms, table, bs, results):
    try:
        side = CpuOwnerSide(table, world, rank, comms[rank], bs=bs)
        comms[rank].run_side(side)
        results[rank] = side
    except BaseException as e:               # noqa: BLE001 -- reported by the test
        results[rank] = e


@pytest.mark.parametrize("world,bs", [(3, 5)])
def test_local_transport_owner_protocol(tmp_path, world, bs):
    """The library's in-process transport (dk_comm_create_local, host buffers), one thread per rank,
    drives the protocol over the CPU stand-in: the merged counters and checkpoint selections equal
    the unsharded oracle's."""
    import threading
    from oracle import ref
    table = str(tmp_path / "t")
    synth.write_table(table, synth.TableSpec(n_adds=3_000, n_parts=2, row_group_size=700, n_commits=6,
                                             adds_per_commit=15, removes_per_commit=15, dv_frac=0.2, readd_frac=0.2))
    seg = ref.load_log_segment(table)
    commits = [f for f in seg.all_files_reversed() if f.kind == "commit"]
    steps = [len(list(ref.read_json_batches(c.path, bs))) for c in commits]
    comms = shard.OwnerComm.local(world, steps=steps, on_device=False)
    results = [None] * world
    ts = [threading.Thread(target=_local_worker, args=(r, world, comms, table, bs, results)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert all(isinstance(x, CpuOwnerSide) for x in results), results
    full = results[0].full
    counters = np.sum([x.counters for x in results], axis=0)
    assert tuple(int(c) for c in counters) == full.counters.as_tuple()
    sel = {}
    for x in results:
        sel.update(x.sel)
    for b in full.checkpoint:
        got = np.array([sel[(b.file_index, r)] for r in range(len(b.selected))], bool)
        assert np.array_equal(got, b.selected.astype(bool))
    assert all(c.bytes_sent > 0 for c in comms)
    for c in comms:
        c.close()


def _rccl_world1_check(table):
    """Body of test_gpu_rccl_world1: one RCCL rank created through the C ABI (dk_comm_unique_id +
    dk_comm_create, no torch.distributed) runs the owner protocol of a whole scan."""
    import torch
    torch.cuda.init()
    from delta_amd import kernel as K
    from oracle import ref
    eng = K.GpuEngine()
    snap = K.Table.forPath(eng, table).getLatestSnapshot(eng)
    comm = shard.OwnerComm.rccl()
    sc = snap.getScanBuilder().withShard(1, 0, owner=comm).build()
    batches = list(sc.getScanFiles(eng))
    full = ref.replay(table)
    rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in batches for i in b.selected_rows()]
    assert sc.metrics.as_tuple() == full.counters.as_tuple(), (sc.metrics.as_tuple(), full.counters.as_tuple())
    assert rows == full.scan_files(), (len(rows), len(full.scan_files()))
    assert comm.ms["total"] > 0
    sc.close()
    comm.close()
    eng.close()
    print("ok")


@pytest.mark.gpu
def test_gpu_rccl_world1(tmp_path):
    """A one-rank RCCL communicator owned by libdkgpu (the path a JVM GpuScan takes: unique id in,
    dk_replay_owner_run) gives the oracle's scan files and counters."""
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=20_000, n_parts=2, row_group_size=4000, n_commits=6,
                                                     adds_per_commit=30, removes_per_commit=30, dv_frac=0.2))
    root = os.path.dirname(HERE)
    code = ("import sys; sys.path.insert(0, %r); from tests.test_owner import _rccl_world1_check; "
            "_rccl_world1_check(%r)" % (root, str(tmp_path)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-4000:]
