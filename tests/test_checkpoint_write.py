"""Checkpoint writing (Table.checkpoint -> SnapshotManager.checkpoint over CreateCheckpointIterator,
delta_amd/checkpoint.py) against the oracle's restatement (oracle/checkpoint.py).

CPU: the oracle on a hand-made log with a known answer (removes inside / outside the retention
window, duplicate and re-added files, repeated txn / domainMetadata / protocol / metaData).
GPU: the product writes the checkpoint of synthetic tables (classic and multi-part source
checkpoints, DVs); the file read back must equal the oracle's rows in order, _last_checkpoint must
carry the add count, and a fresh snapshot reading the new checkpoint must give the same scan files
(product and oracle) as before it was written.
"""
import json
import os

import pytest

from oracle import checkpoint as ock

DAY = 86_400_000


def _line(**kw):
    return json.dumps(kw)


def _handmade(d):
    log = os.path.join(d, "_delta_log")
    os.makedirs(log)
    meta = {"id": "m", "format": {"provider": "parquet", "options": {}},
            "schemaString": json.dumps({"type": "struct", "fields": []}), "partitionColumns": [],
            "configuration": {"delta.deletedFileRetentionDuration": "interval 2 days"}, "createdTime": 1}
    add = lambda p, dc=True: {"add": {"path": p, "partitionValues": {}, "size": 1, "modificationTime": 1,
                                      "dataChange": dc}}
    rm = lambda p, ts: {"remove": {"path": p, "deletionTimestamp": ts, "dataChange": True}}
    commits = [
        [{"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}, {"metaData": meta}, add("a"), add("b"),
         {"txn": {"appId": "x", "version": 1}}],
        [rm("a", 10 * DAY), add("c"), {"domainMetadata": {"domain": "d1", "configuration": "{}", "removed": False}}],
        [rm("c", 1 * DAY), add("a"), {"txn": {"appId": "x", "version": 2}}, add("b")],
        [{"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}, {"txn": {"appId": "y", "version": 7}},
         {"domainMetadata": {"domain": "d1", "configuration": "{\"v\":2}", "removed": False}}],
    ]
    for v, acts in enumerate(commits):
        with open(os.path.join(log, "%020d.json" % v), "w") as f:
            f.write("\n".join(json.dumps(a) for a in acts) + "\n")
    return d


def test_oracle_checkpoint_known_answer(tmp_path):
    d = _handmade(str(tmp_path))
    rows, n_adds = ock.checkpoint_actions(d, now_ms=11 * DAY)       # keep removes after day 9
    kinds = [k for k, _ in rows]
    # newest commit first: v3 protocol (first seen), txn y, domain d1 (v3 wins);
    # v2: remove c (day 1: expired), add a (re-added after its v1 remove), txn x v2, add b (kept: the
    # v0 add b is then a duplicate); v1: remove a (day 10: kept), add c (deleted in v2), domain d1
    # (seen); v0: protocol (seen), metaData (first), add a / b (already returned), txn x (seen)
    assert kinds == ["protocol", "txn", "domainMetadata", "add", "txn", "add", "remove", "metaData"]
    assert rows[1][1][:2] == ("y", 7) and rows[2][1][1] == "{\"v\":2}" and rows[4][1][:2] == ("x", 2)
    assert [r[1][0] for r in rows if r[0] == "add"] == ["a", "b"] and n_adds == 2
    assert rows[6][1][0] == "a"


# ---- the reference's own answers: CreateCheckpointSuite.scala (kernel-defaults tests) -------------------
SUITE_NOW = 1_700_000_000_000


def _write_commits(d, commits):
    log = os.path.join(d, "_delta_log")
    os.makedirs(log)
    for v, acts in enumerate(commits):
        with open(os.path.join(log, "%020d.json" % v), "w") as f:
            f.write("\n".join(json.dumps(a) for a in acts) + "\n")
    return d


def _suite_meta(retention=None):
    conf = {"delta.deletedFileRetentionDuration": retention} if retention else {}
    return {"metaData": {"id": "t", "format": {"provider": "parquet", "options": {}},
                         "schemaString": json.dumps({"type": "struct", "fields": [
                             {"name": "c1", "type": "integer", "nullable": True, "metadata": {}}]}),
                         "partitionColumns": [], "configuration": conf, "createdTime": 1}}


def _suite_add(p):
    return {"add": {"path": p, "partitionValues": {}, "size": 0, "modificationTime": 0, "dataChange": True}}


def _suite_remove(p, ts):
    return {"remove": {"path": p, "deletionTimestamp": ts, "dataChange": True}}


def suite_tombstone_log(d, retention):
    """The log of CreateCheckpointSuite.scala:224-296 ("checkpoint contains all not expired
    tombstones"), as commits relative to a fixed now: addFiles (each commit also updates the metadata
    with the retention setting), then removes of file8 (ts 1), file7 (-8 days), file6 (-3 days),
    file5 (-1 s), addFiles file10-18, removes of file3 (-9 days) and file2 (-1 day); checkpoint at 7."""
    day = 24 * 60 * 60 * 1000
    return _write_commits(d, [
        [{"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}, _suite_meta(retention)] +
        [_suite_add("file%d" % i) for i in range(1, 10)],
        [_suite_remove("file8", 1)],
        [_suite_remove("file7", SUITE_NOW - 8 * day)],
        [_suite_remove("file6", SUITE_NOW - 3 * day)],
        [_suite_remove("file5", SUITE_NOW - 1000)],
        [_suite_meta(retention)] + [_suite_add("file%d" % i) for i in range(10, 19)],
        [_suite_remove("file3", SUITE_NOW - 9 * day)],
        [_suite_remove("file2", SUITE_NOW - 1 * day)],
    ])


# the tombstones the suite asserts per retention setting (:276-290)
SUITE_TOMBSTONES = {None: {"file6", "file5", "file2"}, "2 days": {"file5", "file2"}, "0 days": set()}


def suite_txn_log(d):
    """CreateCheckpointSuite.scala:178-222 ("commits with set transactions"): idempotent appends of
    appId1 (versions 0, 2, 3), a delete, appId2 (7, 25), appId3 (7908), a plain append, appId4."""
    txn = lambda a, v: {"txn": {"appId": a, "version": v, "lastUpdated": 1}}   # noqa: E731
    return _write_commits(d, [
        [{"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}, _suite_meta(), _suite_add("p0"), txn("appId1", 0)],
        [_suite_add("p1"), txn("appId1", 2)],
        [_suite_add("p2"), txn("appId1", 3)],
        [_suite_remove("p0", SUITE_NOW)],
        [_suite_add("p4"), txn("appId2", 7)],
        [_suite_add("p5"), txn("appId2", 25)],
        [_suite_add("p6"), txn("appId3", 7908)],
        [_suite_add("p7")],
        [_suite_add("p8"), txn("appId4", 12312312)],
    ])


SUITE_TXNS = {"appId1": 3, "appId2": 25, "appId3": 7908, "appId4": 12312312}


@pytest.mark.parametrize("retention", [None, "2 days", "0 days"])
def test_oracle_suite_tombstones(tmp_path, retention):
    """The oracle writer keeps exactly the tombstones CreateCheckpointSuite asserts."""
    d = suite_tombstone_log(str(tmp_path), retention)
    rows, _ = ock.checkpoint_actions(d, now_ms=SUITE_NOW)
    assert {r[1][0] for r in rows if r[0] == "remove"} == SUITE_TOMBSTONES[retention]
    assert sum(r[0] == "add" for r in rows) == 18 - 6


def test_oracle_suite_txns(tmp_path):
    d = suite_txn_log(str(tmp_path))
    rows, _ = ock.checkpoint_actions(d, now_ms=SUITE_NOW)
    assert {r[1][0]: r[1][1] for r in rows if r[0] == "txn"} == SUITE_TXNS
    assert sum(r[0] == "txn" for r in rows) == 4 and sum(r[0] == "protocol" for r in rows) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("retention", [None, "2 days", "0 days"])
def test_gpu_suite_tombstones(tmp_path, retention):
    """Table.checkpoint on the GPU over the suite's log writes exactly the asserted tombstones (the
    file read back with pyarrow), and the whole file equals the oracle's rows."""
    from delta_amd import kernel as K
    d = suite_tombstone_log(str(tmp_path), retention)
    want = ock.checkpoint_actions(d, now_ms=SUITE_NOW)[0]        # (before the checkpoint exists)
    eng = K.GpuEngine()
    v, n_adds = K.Table.forPath(eng, d).checkpoint(eng, now_ms=SUITE_NOW)
    assert v == 7 and n_adds == 18 - 6            # file1..file18 less the six removed
    got = ock.read_checkpoint(os.path.join(d, "_delta_log", "%020d.checkpoint.parquet" % v))
    assert {r[1][0] for r in got if r[0] == "remove"} == SUITE_TOMBSTONES[retention]
    assert got == want
    eng.close()


@pytest.mark.gpu
def test_gpu_suite_txns(tmp_path):
    from delta_amd import kernel as K
    d = suite_txn_log(str(tmp_path))
    want = ock.checkpoint_actions(d, now_ms=SUITE_NOW)[0]
    eng = K.GpuEngine()
    v, _ = K.Table.forPath(eng, d).checkpoint(eng, now_ms=SUITE_NOW)
    got = ock.read_checkpoint(os.path.join(d, "_delta_log", "%020d.checkpoint.parquet" % v))
    assert {r[1][0]: r[1][1] for r in got if r[0] == "txn"} == SUITE_TXNS
    assert [r[0] for r in got].count("protocol") == 1
    assert got == want
    eng.close()


def _now_keep_half(ckpt_version, n_commits):
    # synth removes carry deletionTimestamp 1.7e12 + version: keep those of the newer half
    return 1_700_000_000_000 + ckpt_version + n_commits // 2 + 604_800_000


CASES = {
    "classic-dv": dict(n_adds=6_000, n_commits=8, dv_frac=0.2, ckpt_removes=40),
    "multipart-stats": dict(n_adds=9_000, n_parts=3, n_commits=6, with_stats=True, pv_keys=2),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_checkpoint_write(tmp_path, name):
    from delta_amd import kernel as K
    from delta_amd import synth
    from tests.parity_util import assert_same, oracle_scan, product_scan
    d = str(tmp_path)
    spec = synth.TableSpec(seed=synth.SEED + 3, extra={"protocol": {"minWriterVersion": 2, "minReaderVersion": 1,
                                                                     "readerFeatures": None,
                                                                     "writerFeatures": None}}, **CASES[name])
    info = synth.write_table(d, spec)
    # a txn and a domainMetadata line in the newest commit, an older txn in the first
    log = os.path.join(d, "_delta_log")
    with open(os.path.join(log, "%020d.json" % info["version"]), "a") as f:
        f.write(_line(txn={"appId": "app", "version": 9, "lastUpdated": 5}) + "\n")
        f.write(_line(domainMetadata={"domain": "dom", "configuration": "{}", "removed": False}) + "\n")
    with open(os.path.join(log, "%020d.json" % (spec.ckpt_version + 1)), "a") as f:
        f.write(_line(txn={"appId": "app", "version": 1}) + "\n")
    now = _now_keep_half(spec.ckpt_version, spec.n_commits)
    before = oracle_scan(d)
    want, want_adds = ock.checkpoint_actions(d, now)
    eng = K.GpuEngine()
    v, n_adds = K.Table.forPath(eng, d).checkpoint(eng, now_ms=now)
    assert v == info["version"] and n_adds == want_adds
    # read back with pyarrow (an independent Parquet reader): rows in order, and the schema's
    # repetition / nesting as the reference declares it
    got = ock.read_checkpoint(os.path.join(log, "%020d.checkpoint.parquet" % v))
    import pyarrow.parquet as pq
    from tests.test_checkpoint_schema import EXPECTED
    pf = pq.ParquetFile(os.path.join(log, "%020d.checkpoint.parquet" % v))
    sch = pf.schema_arrow
    assert sch.names == ["txn", "add", "remove", "metaData", "protocol", "domainMetadata"]
    for top in ("add", "remove", "metaData", "protocol", "txn", "domainMetadata"):
        t = sch.field(top).type
        assert [(t.field(i).name, t.field(i).nullable) for i in range(t.num_fields)] == EXPECTED[top], top
    assert pf.metadata.row_group(pf.metadata.num_row_groups - 1).column(0).compression == "SNAPPY"
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a == b, (i, a, b)
    assert json.load(open(os.path.join(log, "_last_checkpoint"))) == {"version": v, "size": n_adds}
    # the table now starts from the new checkpoint: same scan files, oracle and product
    after_o = oracle_scan(d)
    assert sorted(after_o[1]) == sorted(before[1])
    assert_same(product_scan(d), after_o)
    with pytest.raises(K.DkError, match="already exists"):
        K.Table.forPath(eng, d).checkpoint(eng, now_ms=now)


@pytest.mark.gpu
def test_gpu_checkpoint_unsupported_writer_feature(tmp_path):
    from delta_amd import kernel as K
    from delta_amd import synth
    d = str(tmp_path)
    synth.write_table(d, synth.TableSpec(n_adds=1_000, n_commits=2))     # writerFeatures deletionVectors, ...
    eng = K.GpuEngine()
    with pytest.raises(K.DkError, match="writer table feature \"deletionVectors\""):
        K.Table.forPath(eng, d).checkpoint(eng)
