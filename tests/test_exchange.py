"""hash(path)-owner exchange, the multi-GPU "alltoall" mode (delta_amd/shard.py: path_owner,
exchange_hash_owner, exchange_local; dk_replay_exchange_*).

CPU: a world-2 gloo run of the product's exchange driver (exchange_hash_owner: sizes, records,
reverse all-to-all of the owners' answers) and routing function (path_owner) over a CPU stand-in for
the device side (CpuSide: the same four calls as shard.ExchangeSide, keys hashed by the product's
own dk_uri.h code compiled for the host, the oracle's decode, the oracle's exact probe for the
candidates). Rank 0 checks the reassembled selection bits and counters against the unsharded
oracle replay, and that every row an owner decided ("no commit-tail key has this path hash") is one
the oracle selects.
GPU: the product's exchange mode for 2 and 3 ranks simulated in one process (exchange_local) equals
the oracle, rows and counters.
"""
import ctypes as C
import json
import os
import socket
import subprocess

import numpy as np
import pytest

from delta_amd import shard, synth

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "_uri_shim.so")


def _shim():
    src = os.path.join(HERE, "native", "uri_shim.cpp")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(
            os.path.join(HERE, "..", "delta_amd", "csrc", "dk_uri.h"))):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO + ".tmp", src])
        os.replace(SO + ".tmp", SO)
    L = C.CDLL(SO)
    L.prod_simple_hash.argtypes = [C.c_char_p, C.c_int32, C.c_uint32, C.POINTER(C.c_uint64)]
    return L


def _simple_hash(L, s: bytes):
    h = C.c_uint64()
    return int(h.value) if L.prod_simple_hash(s, len(s), 0, C.byref(h)) else 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tail_paths(table):
    """Every add / remove path of the commit files after the checkpoint (the commit tail)."""
    from delta_amd import kernel as K
    seg = K.build_log_segment(table)
    out = []
    for d in seg.deltas:
        with open(d.path, "rb") as f:
            for line in f.read().split(b"\n"):
                if not line.strip():
                    continue
                o = json.loads(line)
                for k in ("add", "remove"):
                    if o.get(k):
                        out.append(o[k]["path"].encode())
    return out


class CpuSide:
    """CPU stand-in for shard.ExchangeSide: this rank's row-group shard of the oracle's replay."""

    def __init__(self, table, world, rank, full):
        from delta_amd import kernel as K
        from oracle import ref
        self.L = _shim()
        self.world, self.rank, self.full = world, rank, full
        files = [b.path for b in full.checkpoint]
        rgs = [K.row_group_rows(p) for p in files]
        self.units = shard.unit_layout(rgs, shard.plan_units(rgs, world, rank))
        self.rows = []            # (file, row, class, hp): class 0 no add, 1 routed, 2 local candidate
        for f, r0, n in self.units:
            pf = ref.ParquetFile.open(files[f])
            pc = pf.read("add.path")
            st = pf.read("add.deletionVector.storageType")
            for r in range(r0, r0 + n):
                if pc.row_def[r] < pc.max_def:
                    self.rows.append((f, r, 0, 0))
                    continue
                hp = _simple_hash(self.L, pc.string(r))
                dv = st is not None and st.row_def[r] >= 2
                self.rows.append((f, r, 2 if (hp == 0 or dv) else 1, hp))
        self.owned = {h for h in (_simple_hash(self.L, p) for p in _tail_paths(table))
                      if h and shard.path_owner(h, world) == rank}
        self.decided = []

    def counts(self):
        c = np.zeros(self.world, np.int64)
        for _, _, cls, hp in self.rows:
            if cls == 1:
                c[shard.path_owner(hp, self.world)] += 1
        return c

    def pack(self, n):
        import torch
        self.sent = sorted((i for i, x in enumerate(self.rows) if x[2] == 1),
                           key=lambda i: shard.path_owner(self.rows[i][3], self.world))
        assert len(self.sent) == n
        return torch.tensor([np.int64(np.uint64(self.rows[i][3])) for i in self.sent], dtype=torch.int64)

    def filter(self, recv):
        import torch
        hs = [int(np.uint64(np.int64(x))) for x in recv.tolist()]
        assert all(shard.path_owner(h, self.world) == self.rank for h in hs)
        return torch.tensor([1 if h in self.owned else 0 for h in hs], dtype=torch.uint8)

    def finish(self, back):
        b = back.tolist()
        assert len(b) == len(self.sent)
        answer = {i: v for i, v in zip(self.sent, b)}
        sel = {}
        for i, (f, r, cls, _) in enumerate(self.rows):
            exact = bool(self.full.checkpoint[f].selected[r])          # the exact key probe
            if cls == 1 and answer[i] == 0:
                self.decided.append((f, r, exact))
                sel[(f, r)] = True
            else:
                sel[(f, r)] = exact and cls != 0
        self.sel = sel

    def units_bits(self):
        out = []
        for f, r0, n in self.units:
            bits = np.array([self.sel[(f, r)] for r in range(r0, r0 + n)], bool)
            out.append((f, r0, n, np.packbits(bits, bitorder="little")))
        return out


def _gloo_worker(rank, world, port, table, out_path):
    import torch.distributed as dist
    from oracle import ref
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        full = ref.replay(table)
        side = CpuSide(table, world, rank, full)
        sent = shard.exchange_hash_owner(side)
        ck = full.ckpt_counters.as_tuple() if rank == 0 else (0, 0, 0, 0, 0)
        counters, sels = shard.gather_selections(side.units_bits(), full.tail_counters.as_tuple(), ck)
        wrong = [d for d in side.decided if not d[2]]
        res = {"rank": rank, "sent_bytes": sent, "decided": len(side.decided), "wrong_decisions": len(wrong)}
        if rank == 0:
            ok = counters == full.counters.as_tuple()
            for b in full.checkpoint:
                parts = [s for s in sels if s[0] == b.file_index]
                bits = np.concatenate([np.unpackbits(s[3], bitorder="little")[:s[2]] for s in parts])
                ok = ok and np.array_equal(bits.astype(bool), b.selected.astype(bool))
            res["ok"] = bool(ok)
        with open(out_path + ".%d" % rank, "w") as f:
            json.dump(res, f)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_path_owner_partitions():
    L = _shim()
    hs = [_simple_hash(L, ("p/part-%05d.parquet" % i).encode()) for i in range(4000)]
    assert all(hs)
    for world in (2, 3, 8):
        own = [shard.path_owner(h, world) for h in hs]
        assert set(own) == set(range(world))
        counts = np.bincount(own, minlength=world)
        assert counts.min() > 0.7 * len(hs) / world        # the hash spreads keys evenly


def test_gloo_world2_exchange(tmp_path):
    """world 2 over gloo: the product's exchange driver + routing reassemble the oracle's selection;
    no owner decision contradicts the exact probe."""
    import torch.multiprocessing as mp
    _shim()
    for name, spec in (("multi", dict(n_parts=3, row_group_size=2000)), ("single", dict(n_parts=1, row_group_size=1500))):
        table = str(tmp_path / name)
        synth.write_table(table, synth.TableSpec(n_adds=9_000, n_commits=8, dv_frac=0.1, ckpt_removes=40, **spec))
        out = str(tmp_path / (name + ".json"))
        mp.spawn(_gloo_worker, args=(2, _free_port(), table, out), nprocs=2, join=True)
        res = [json.load(open(out + ".%d" % r)) for r in range(2)]
        assert res[0]["ok"], (name, res)
        assert all(r["wrong_decisions"] == 0 for r in res), (name, res)
        assert sum(r["decided"] for r in res) > 0.8 * 9_000, (name, res)     # most rows decided by owners
        assert all(r["sent_bytes"] > 0 for r in res)


def _local_exchange_check(table, world):
    """Body of test_gpu_exchange_local, run in a fresh process that imports torch before libdkgpu (the
    order bench.py's ranks use: both then share torch's HIP runtime, which the exchange's device
    tensors need)."""
    import torch
    torch.cuda.init()
    from delta_amd import kernel as K
    from oracle import ref
    eng = K.GpuEngine()
    sides, scans = [], []
    for r in range(world):
        snap = K.Table.forPath(eng, table).getLatestSnapshot(eng)
        sc = snap.getScanBuilder().withShard(world, r, exchange=sides.append).build()
        sc.prepare(eng)
        scans.append(sc)
    full = ref.replay(table)
    for step in range(2):                     # a second run reuses the replay (counts, buffers)
        del sides[:]
        for sc in scans:
            sc.run()
        shard.exchange_local(sides)
        outs = []
        for r, sc in enumerate(scans):
            sc.sync()
            o = shard.ShardOutput(r, sc.tail_metrics.as_tuple(), sc.ckpt_metrics.as_tuple())
            for b in sc._batches():
                if b.file_index < 0:
                    o.tail = b
                else:
                    o.files[(b.file_index, b.row_offset)] = b
            outs.append(o)
        counters, batches = shard.merge(outs)
        rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in batches for i in b.selected_rows()]
        assert counters == full.counters.as_tuple(), (step, counters, full.counters.as_tuple())
        assert rows == full.scan_files(), step
    for sc in scans:
        sc.close()
    eng.close()
    print("ok")


@pytest.mark.gpu
@pytest.mark.parametrize("world,spec", [(2, dict(n_parts=3, row_group_size=3000)),
                                        (3, dict(n_parts=1, row_group_size=2500, dv_frac=0.2, ckpt_removes=100))])
def test_gpu_exchange_local(tmp_path, world, spec):
    """The product's exchange mode (route + pack + owner filter + apply + exact probe on the device)
    for `world` ranks simulated in one process: merged rows and counters equal the oracle's."""
    import sys
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=20_000, n_commits=8, **spec))
    root = os.path.dirname(HERE)
    code = ("import sys; sys.path.insert(0, %r); from tests.test_exchange import _local_exchange_check; "
            "_local_exchange_check(%r, %d)" % (root, str(tmp_path), world))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-4000:]
