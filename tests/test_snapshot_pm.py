"""Snapshot-load P&M pass (LogReplay.loadTableProtocolAndMetadata, internal/replay/LogReplay.java:
220-314): the product's protocol / metadata must equal the oracle's on every golden table, and on a
synthetic checkpoint-only table where the first non-null rows sit deep inside the checkpoint."""
import os
import re

import pytest

from tests.golden_util import TABLES

NAMES = sorted(os.listdir(TABLES))


def _product_pm(root):
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    try:
        snap = K.Table.forPath(eng, root).getLatestSnapshot(eng)
        return snap.protocol, snap.metadata, snap._validated
    finally:
        eng.close()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_pm_golden(name):
    from oracle import ref
    prot, meta, _ = ref.load_protocol_metadata(os.path.join(TABLES, name))
    assert prot["minReaderVersion"] >= 1 and prot["minWriterVersion"] >= 1
    assert meta["id"] and meta["schemaString"].startswith("{") and meta["format"]["provider"] == "parquet"
    assert isinstance(meta["configuration"], dict) and isinstance(meta["partitionColumns"], list)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_pm_golden(name):
    from oracle import ref
    root = os.path.join(TABLES, name)
    assert _product_pm(root) == ref.load_protocol_metadata(root)


def _checkpoint_only(d, parts, move_pm_to=None):
    """Synthetic table whose commits are all covered by the checkpoint (JSONs deleted): P&M must
    come from the checkpoint. move_pm_to=(i, j) rewrites part 1 with the protocol row at i and the
    metaData row at j (small pages, so the rows sit deep inside the column chunks)."""
    import numpy as np
    import pyarrow.parquet as pq
    from delta_amd import synth
    synth.write_table(d, synth.TableSpec(n_adds=40_000, n_commits=0, pv_keys=2, n_parts=parts))
    log = os.path.join(d, "_delta_log")
    for f in os.listdir(log):
        if f.endswith(".json"):
            os.remove(os.path.join(log, f))
    if move_pm_to:
        first = sorted(f for f in os.listdir(log) if f.endswith(".parquet"))[0]
        t = pq.read_table(os.path.join(log, first))
        n = t.num_rows
        order = list(range(2, n))
        i, j = move_pm_to
        for pos, src in sorted([(i, 0), (j, 1)]):
            order.insert(pos, src)
        t = t.take(np.array(order))
        pq.write_table(t, os.path.join(log, first), data_page_size=4096, use_dictionary=False)


@pytest.mark.gpu
@pytest.mark.parametrize("parts,move", [(1, None), (3, None), (1, (25_001, 13_007)), (2, (19_999, 20_000))])
def test_gpu_pm_checkpoint_only(tmp_path, parts, move):
    from oracle import ref
    d = str(tmp_path)
    _checkpoint_only(d, parts, move)
    got = _product_pm(d)
    assert got == ref.load_protocol_metadata(d)
    assert got[1]["partitionColumns"] == ["date"]
    assert got[0]["readerFeatures"] == ["deletionVectors", "v2Checkpoint"]
    assert got[1]["configuration"] == {"delta.enableDeletionVectors": "true"}


def test_oracle_pm_moved_rows(tmp_path):
    from oracle import ref
    d = str(tmp_path)
    _checkpoint_only(d, 1, (25_001, 13_007))
    prot, meta, _ = ref.load_protocol_metadata(d)
    assert (prot["minReaderVersion"], prot["minWriterVersion"]) == (3, 7) and meta["partitionColumns"] == ["date"]
    assert prot["readerFeatures"] == ["deletionVectors", "v2Checkpoint"]
    assert meta["format"] == {"provider": "parquet", "options": {}} and meta["createdTime"] == 1_700_000_000_000


def _pm_table(d, protocol, configuration=None):
    """A one-commit table with the given protocol / metaData configuration."""
    import json
    log = os.path.join(d, "_delta_log")
    os.makedirs(log)
    meta = {"id": "t", "format": {"provider": "parquet", "options": {}},
            "schemaString": json.dumps({"type": "struct", "fields": [
                {"name": "a", "type": "long", "nullable": True, "metadata": {}}]}),
            "partitionColumns": [], "configuration": configuration or {}, "createdTime": 1}
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        f.write(json.dumps({"protocol": protocol}) + "\n" + json.dumps({"metaData": meta}) + "\n")
        f.write(json.dumps({"add": {"path": "a.parquet", "partitionValues": {}, "size": 1, "modificationTime": 1,
                                    "dataChange": True}}) + "\n")
    return d


# TableFeatures.validateReadSupportedTable (TableFeatures.java:76-98): (protocol, configuration,
# expected error fragment or None)
VALIDATION_CASES = [
    ({"minReaderVersion": 1, "minWriterVersion": 2}, None, None),
    ({"minReaderVersion": 2, "minWriterVersion": 5}, {"delta.columnMapping.mode": "Name"}, None),
    ({"minReaderVersion": 2, "minWriterVersion": 5}, {"delta.columnMapping.mode": "bogus"},
     "Invalid value for table property 'delta.columnMapping.mode'"),
    ({"minReaderVersion": 3, "minWriterVersion": 7, "readerFeatures": ["deletionVectors", "v2Checkpoint"],
      "writerFeatures": ["deletionVectors"]}, None, None),
    ({"minReaderVersion": 3, "minWriterVersion": 7, "readerFeatures": ["deletionVectors", "fancyFeature"],
      "writerFeatures": []}, None, "requires reader table features [fancyFeature]"),
    ({"minReaderVersion": 3, "minWriterVersion": 7, "readerFeatures": ["columnMapping"], "writerFeatures": []},
     {"delta.columnMapping.mode": "oops"}, "Invalid value for table property"),
    ({"minReaderVersion": 4, "minWriterVersion": 7}, None, "requires reader version 4"),
]


@pytest.mark.parametrize("case", range(len(VALIDATION_CASES)))
def test_oracle_read_support(tmp_path, case):
    from oracle import ref
    prot, conf, err = VALIDATION_CASES[case]
    d = _pm_table(str(tmp_path / "t"), prot, conf)
    if err is None:
        p, m, _ = ref.load_protocol_metadata(d)
        assert p["minReaderVersion"] == prot["minReaderVersion"]
        assert p["readerFeatures"] == prot.get("readerFeatures", [])
    else:
        with pytest.raises(ref.OracleError, match=re.escape(err)):
            ref.load_protocol_metadata(d)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(VALIDATION_CASES)))
def test_gpu_read_support(tmp_path, case):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    from oracle import ref
    prot, conf, err = VALIDATION_CASES[case]
    d = _pm_table(str(tmp_path / "t"), prot, conf)
    if err is None:
        assert _product_pm(d) == ref.load_protocol_metadata(d)
    else:
        eng = K.GpuEngine()
        with pytest.raises(DkError, match=re.escape(err)):
            K.Table.forPath(eng, d).getLatestSnapshot(eng)
        eng.close()


# ---- checksum files and the order of the P&M finds (LogReplay.java:130-150, 260-302, 384-426) ----
BAD = {"minReaderVersion": 3, "minWriterVersion": 7, "readerFeatures": ["fancyFeature"], "writerFeatures": []}
GOOD = {"minReaderVersion": 1, "minWriterVersion": 2}


def _meta(i):
    import json
    return {"id": "t%d" % i, "format": {"provider": "parquet", "options": {}},
            "schemaString": json.dumps({"type": "struct", "fields": []}), "partitionColumns": [],
            "configuration": {}, "createdTime": i}


def _commits(d, actions_per_commit, crcs=()):
    """Commits 0..n-1 with the given actions; crcs: (version, protocol, metadata, n_lines)."""
    import json
    log = os.path.join(d, "_delta_log")
    os.makedirs(log)
    for v, acts in enumerate(actions_per_commit):
        with open(os.path.join(log, "%020d.json" % v), "w") as f:
            f.write("".join(json.dumps(a) + "\n" for a in acts) or json.dumps({"commitInfo": {}}) + "\n")
    for v, p, m, lines in crcs:
        with open(os.path.join(log, "%020d.crc" % v), "w") as f:
            f.write("\n".join([json.dumps({"protocol": p, "metadata": m, "numFiles": 0})] * lines) + "\n")
    return d


# (commits, crcs, expected error fragment or None)
CRC_CASES = {
    # a checksum file at the snapshot version answers alone: no log read, no validation
    "crc-at-version": ([[{"protocol": GOOD}, {"metaData": _meta(0)}], [{"protocol": BAD}]],
                       [(1, BAD, _meta(9), 1)], None),
    # an older checksum file is the hint: the newer commit's metadata wins, the hint's protocol fills in
    "crc-hint": ([[{"protocol": GOOD}, {"metaData": _meta(0)}], [{"protocol": GOOD}], [{"metaData": _meta(2)}]],
                 [(1, BAD, _meta(1), 1)], None),
    # a checksum file with two rows is not a checksum file: the log decides (and validates)
    "crc-two-rows": ([[{"protocol": BAD}, {"metaData": _meta(0)}], []], [(1, GOOD, _meta(9), 2)],
                     "requires reader table features [fancyFeature]"),
    # metadata in a newer commit than the protocol: found first, so the reference never validates
    "meta-newer-than-protocol": ([[{"protocol": BAD}], [{"metaData": _meta(1)}]], [], None),
    # protocol newer than the metadata: validated when the metadata arrives
    "protocol-newer": ([[{"metaData": _meta(0)}], [{"protocol": BAD}]], [], "fancyFeature"),
}


@pytest.mark.parametrize("name", sorted(CRC_CASES))
def test_oracle_crc_and_order(tmp_path, name):
    from oracle import ref
    commits, crcs, err = CRC_CASES[name]
    d = _commits(str(tmp_path / "t"), commits, crcs)
    if err:
        with pytest.raises(ref.OracleError, match=re.escape(err)):
            ref.load_protocol_metadata(d)
        return
    p, m, validated = ref.load_protocol_metadata(d)
    if name == "crc-at-version":
        assert p == ref._pm_json_protocol(BAD) and m["id"] == "t9" and not validated
    if name == "crc-hint":
        assert p == ref._pm_json_protocol(BAD) and m["id"] == "t2" and not validated
    if name == "meta-newer-than-protocol":
        assert p["readerFeatures"] == ["fancyFeature"] and m["id"] == "t1" and not validated


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CRC_CASES))
def test_gpu_crc_and_order(tmp_path, name):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    from oracle import ref
    commits, crcs, err = CRC_CASES[name]
    d = _commits(str(tmp_path / "t"), commits, crcs)
    if err:
        eng = K.GpuEngine()
        with pytest.raises(DkError, match=re.escape(err)):
            K.Table.forPath(eng, d).getLatestSnapshot(eng)
        eng.close()
    else:
        assert _product_pm(d) == ref.load_protocol_metadata(d)


@pytest.mark.gpu
def test_gpu_crc_on_synthetic_checkpoint(tmp_path):
    """A Spark-style checksum at the snapshot version: the snapshot loads from it, the scan is
    unchanged."""
    from delta_amd import kernel as K
    from delta_amd import synth
    from oracle import ref
    d = str(tmp_path)
    info = synth.write_table(d, synth.TableSpec(n_adds=5_000, n_commits=3))
    synth.write_crc(d, info["version"])
    got = _product_pm(d)
    assert got == ref.load_protocol_metadata(d) and got[2] is False
