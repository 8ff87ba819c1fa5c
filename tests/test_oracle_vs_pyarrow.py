"""Pins the C oracle's Parquet decode against pyarrow (an independent Parquet implementation) on
synthetic checkpoints covering every encoding / page / codec combination the path reads
(SURVEY.md App. D)."""
import itertools

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from delta_amd import synth
from oracle import ref

CASES = [
    dict(compression="none", data_page_version="1.0", use_dictionary=True),
    dict(compression="snappy", data_page_version="1.0", use_dictionary=True),
    dict(compression="none", data_page_version="2.0", use_dictionary=False),
    dict(compression="snappy", data_page_version="2.0", use_dictionary=True),
    dict(compression="none", data_page_version="1.0", delta_binary_packed=True),
    dict(compression="snappy", data_page_version="2.0", delta_binary_packed=True),
]


def _arrow_leaf(table, dotted):
    parts = dotted.split(".")
    col = table.column(parts[0]).combine_chunks()
    return col, parts[1:]


def _expected_rows(table, dotted):
    """Python values per row for a leaf, None when any ancestor or the leaf is null."""
    out = []
    for row in table.column(dotted.split(".")[0]).to_pylist():
        v = row
        parts = dotted.split(".")[1:]
        for p in parts:
            if v is None:
                break
            if p == "key_value":
                break
            v = v.get(p) if isinstance(v, dict) else None
        out.append(v)
    return out


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}={v}" for k, v in c.items()))
def test_decode_matches_pyarrow(tmp_path, case):
    spec = synth.TableSpec(n_adds=30_000, pv_keys=2, dv_frac=0.3, with_stats=True, ckpt_removes=50,
                           max_rows_per_page=7_000, n_commits=0, **case)
    info = synth.write_table(str(tmp_path), spec)
    fn = info["checkpoint_files"][0]
    t = pq.read_table(fn)
    pf = ref.ParquetFile.open(fn)
    assert pf.num_rows == t.num_rows
    n = t.num_rows
    add = t.column("add").to_pylist()
    # scalar leaves
    for leaf, dt in [("add.size", np.int64), ("add.modificationTime", np.int64),
                     ("add.deletionVector.offset", np.int32), ("add.deletionVector.cardinality", np.int64)]:
        c = pf.read(leaf)
        exp = _expected_rows(t, leaf)
        got = [None if c.row_def[i] < c.max_def else c.fixed[i * c.width:(i + 1) * c.width].view(dt)[0].item()
               for i in range(n)]
        assert got == exp, leaf
    for leaf in ["add.path", "add.deletionVector.pathOrInlineDv", "add.stats", "remove.path"]:
        c = pf.read(leaf)
        exp = _expected_rows(t, leaf)
        got = [None if c.row_def[i] < c.max_def else c.string(i).decode() for i in range(n)]
        assert got == exp, leaf
    c = pf.read("add.dataChange")
    assert [None if c.row_def[i] < 2 else bool(c.fixed[i]) for i in range(n)] == _expected_rows(t, "add.dataChange")
    # map leaves
    k = pf.read("add.partitionValues.key_value.key")
    v = pf.read("add.partitionValues.key_value.value")
    assert k.n_rows == n
    for i in range(n):
        exp = None if add[i] is None else add[i]["partitionValues"]
        if k.row_def[i] < 2:
            assert exp is None
            continue
        got = []
        for j in range(k.row_offs[i], k.row_offs[i + 1]):
            got.append((k.chars[k.offs[j]:k.offs[j + 1]].tobytes().decode(),
                        None if v.entry_def[j] < v.max_def else v.chars[v.offs[j]:v.offs[j + 1]].tobytes().decode()))
        assert got == list(exp), i
    # list leaf (protocol.readerFeatures) and missing columns
    rf = pf.read("protocol.readerFeatures.list.element")
    assert rf.n_rows == n and rf.row_def[0] >= 3
    assert [rf.chars[rf.offs[j]:rf.offs[j + 1]].tobytes() for j in range(rf.row_offs[0], rf.row_offs[1])] == \
        [b"deletionVectors", b"v2Checkpoint"]
    assert pf.read("add.no_such_column") is None
