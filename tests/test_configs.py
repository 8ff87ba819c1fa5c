"""GPU parity at the shapes of BASELINE.json's configurations, at reduced row
counts, plus one full-size C2 counter / selection check.

* C2: 2-key partitionValues, `stats` + `stats_parsed` in the checkpoint, snappy; read without stats
  (C2a) and with stats (C2b).
* C3: 64-part snappy checkpoint + 1k commits (100 adds + 100 removes each, 10% re-adds, 5%
  duplicates), unsharded and as 8 shards (ScanBuilder.withShard, delta_amd/shard.py) merged.
* C2 at 10M rows, as SURVEY §8(d) specifies it (snappy, 2-key partitionValues, `stats` +
  `stats_parsed`, read with stats): ScanMetrics counters, every checkpoint selection bit, the
  commit-tail rows and digests of every decoded leaf the scan files carry (path, partitionValues,
  size, modificationTime, stats) against the oracle.
"""
import zlib

import numpy as np
import pytest

from delta_amd import shard, synth
from tests.parity_util import assert_same, oracle_scan, product_scan

pytestmark = pytest.mark.gpu

C2 = dict(pv_keys=2, with_stats=True, with_stats_parsed=True, compression="snappy", n_commits=20,
          adds_per_commit=50, removes_per_commit=50)
C3 = dict(n_parts=64, compression="snappy", n_commits=1000, adds_per_commit=100, removes_per_commit=100,
          readd_frac=0.1, dup_frac=0.05)


@pytest.mark.parametrize("stats", [False, True], ids=["C2a", "C2b"])
def test_c2_shape(tmp_path, stats):
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=40_000, seed=synth.SEED + 2, **C2))
    assert_same(product_scan(str(tmp_path), with_stats=stats), oracle_scan(str(tmp_path), with_stats=stats))


@pytest.fixture(scope="module")
def c3_table(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("c3"))
    synth.write_table(d, synth.TableSpec(n_adds=64 * 1500, seed=synth.SEED + 3, **C3))
    return d


@pytest.fixture(scope="module")
def c3_oracle(c3_table):
    return oracle_scan(c3_table)


def test_c3_shape(c3_table, c3_oracle):
    p = product_scan(c3_table)
    assert_same(p, c3_oracle)
    assert p[2][4] == 1000 * 100            # every commit's removes were seen


def test_c3_shape_8_shards(c3_table, c3_oracle):
    from delta_amd import kernel as K
    from oracle import ref
    eng = K.GpuEngine()
    outs, scans = [], []
    for r in range(8):
        snap = K.Table.forPath(eng, c3_table).getLatestSnapshot(eng)
        o, sc = shard.gpu_shard_scan(eng, snap, 8, r)
        outs.append(o)
        scans.append(sc)
    counters, batches = shard.merge(outs)
    rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in batches for i in b.selected_rows()]
    assert counters == c3_oracle[2]
    assert rows == c3_oracle[1]
    for sc in scans:
        sc.close()
    eng.close()


def _col_digest(col):
    """crc32 over a decoded column's buffers (row_def, map offsets / entry levels, offsets, chars /
    fixed values)."""
    h = zlib.crc32(np.ascontiguousarray(col.row_def))
    for a in (getattr(col, "row_offs", None), getattr(col, "entry_def", None), col.offs, col.chars, col.fixed):
        if a is not None:
            h = zlib.crc32(np.ascontiguousarray(a), h)
    return h


C2_LEAVES = ("add.path", "add.partitionValues.key_value.key", "add.partitionValues.key_value.value", "add.size",
             "add.modificationTime", "add.stats")


@pytest.mark.timeout(900)
def test_c2_full_size_10m(tmp_path):
    from delta_amd import kernel as K
    from oracle import ref
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=10_000_000, **C2))
    eng = K.GpuEngine()
    snap = K.Table.forPath(eng, str(tmp_path)).getLatestSnapshot(eng)
    scan = snap.getScanBuilder().withStats(True).build()
    got_sel, got_tail, got_dig = [], None, None
    for b in scan.getScanFiles(eng):
        rows = b.selected_rows()
        if b.file_index < 0:
            got_tail = [ref.canon_add_from_cols(b.data, int(i)) for i in rows]
            continue
        got_sel.append(np.asarray(b.selection, dtype=bool))
        got_dig = [_col_digest(b.data[leaf]) for leaf in C2_LEAVES]
    counters = scan.metrics.as_tuple()
    scan.close()
    eng.close()
    r = ref.replay(str(tmp_path), with_stats=True)
    assert counters == r.counters.as_tuple()
    assert counters[0] > 10_000_000
    assert got_tail == [ref.canon_add_from_json(a) for a in r.json_rows]
    assert len(got_sel) == len(r.checkpoint) == 1
    want = r.checkpoint[0]
    assert np.array_equal(got_sel[0], want.selected.astype(bool))
    # the selected rows' content: every decoded leaf the rows come from is identical
    assert got_dig == [_col_digest(want.cols[leaf]) for leaf in C2_LEAVES]
