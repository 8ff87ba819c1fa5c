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
        return snap.protocol, snap.metadata
    finally:
        eng.close()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_pm_golden(name):
    from oracle import ref
    prot, meta = ref.load_protocol_metadata(os.path.join(TABLES, name))
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
    prot, meta = ref.load_protocol_metadata(d)
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
        p, m = ref.load_protocol_metadata(d)
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
