"""GPU error paths: the scan fails the way the reference does, and the engine stays usable.

* an illegal java.net.URI in a checkpoint add path and in a commit-tail add path
  (LogReplayUtils.pathToUri, LogReplayUtils.java:83-89: new URI(path) -> RuntimeException wrapping
  java.net.URISyntaxException);
* a corrupt page header, a damaged snappy block and a GZIP column chunk
  (ParquetFileReader.java:82,142: KernelEngineException "Error reading Parquet file: <path>").
After each failure a clean table is scanned with the same engine and must match the oracle.
"""
import json
import os

import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from delta_amd import synth
from tests.parity_util import assert_same, oracle_scan, product_scan

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def clean_table(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("clean"))
    synth.write_table(d, synth.TableSpec(n_adds=4_000, n_commits=3, compression="snappy"))
    return d


def _still_usable(engine, clean_table):
    assert_same(product_scan(clean_table, engine=engine), oracle_scan(clean_table))


def _table(d, **kw):
    spec = dict(n_adds=4_000, n_commits=3)
    spec.update(kw)
    synth.write_table(d, synth.TableSpec(**spec))
    return os.path.join(d, "_delta_log", "%020d.checkpoint.parquet" % 10)


def _rewrite_checkpoint(path, fn, **write_kw):
    t = pq.read_table(path)
    t = fn(t)
    kw = dict(compression="none", use_dictionary=False, write_statistics=True)
    kw.update(write_kw)
    pq.write_table(t, path, **kw)


def _scan_error(engine, root):
    from delta_amd._lib import DkError
    with pytest.raises(DkError) as ei:
        product_scan(root, engine=engine)
    return str(ei.value)


def test_illegal_uri_checkpoint_row(tmp_path, engine, clean_table):
    ck = _table(str(tmp_path))

    def bad_path(t):
        add = t.column("add").combine_chunks()
        paths = add.field("path").to_pylist()
        paths[1234] = "date=2024-01-01/bad path {x}.parquet"   # space and braces: illegal in a URI
        fields = [add.field(i) if add.type[i].name != "path" else pa.array(paths, pa.string())
                  for i in range(add.type.num_fields)]
        new_add = pa.StructArray.from_arrays(fields, fields=list(add.type), mask=add.is_null())
        return t.set_column(t.schema.get_field_index("add"), "add", new_add)
    _rewrite_checkpoint(ck, bad_path)
    msg = _scan_error(engine, str(tmp_path))
    assert "java.net.URISyntaxException" in msg and "checkpoint row" in msg, msg
    _still_usable(engine, clean_table)


def test_illegal_uri_tail_row(tmp_path, engine, clean_table):
    _table(str(tmp_path))
    log = os.path.join(str(tmp_path), "_delta_log")
    last = max(int(f[:20]) for f in os.listdir(log) if f.endswith(".json"))
    with open(os.path.join(log, "%020d.json" % (last + 1)), "w") as f:
        f.write(json.dumps({"add": {"path": "date=2024-01-01/a b.parquet", "partitionValues": {"date": "2024-01-01"},
                                    "size": 1, "modificationTime": 2, "dataChange": True}}) + "\n")
    msg = _scan_error(engine, str(tmp_path))
    assert "java.net.URISyntaxException" in msg and "a b.parquet" in msg, msg
    _still_usable(engine, clean_table)


def _first_data_page_offset(path, leaf="add.path"):
    md = pq.ParquetFile(path).metadata
    for i in range(md.num_columns):
        c = md.row_group(0).column(i)
        if c.path_in_schema == leaf:
            return c.data_page_offset
    raise KeyError(leaf)


def test_corrupt_page_header(tmp_path, engine, clean_table):
    ck = _table(str(tmp_path), use_dictionary=False)
    off = _first_data_page_offset(ck)
    with open(ck, "r+b") as f:
        f.seek(off)
        f.write(b"\xff" * 12)
    msg = _scan_error(engine, str(tmp_path))
    assert msg.startswith("Error reading Parquet file: ") and ck in msg, msg
    _still_usable(engine, clean_table)


def test_damaged_snappy_block(tmp_path, engine, clean_table):
    ck = _table(str(tmp_path), use_dictionary=False, compression="snappy")
    pf = pq.ParquetFile(ck)
    col = next(pf.metadata.row_group(0).column(i) for i in range(pf.metadata.num_columns)
               if pf.metadata.row_group(0).column(i).path_in_schema == "add.path")
    body_mid = col.data_page_offset + col.total_compressed_size // 2
    with open(ck, "r+b") as f:
        f.seek(body_mid)
        f.write(b"\x00" * 256)       # 1-byte literals from here on: the block no longer has its length
    msg = _scan_error(engine, str(tmp_path))
    assert msg.startswith("Error reading Parquet file: ") and ck in msg, msg
    _still_usable(engine, clean_table)


def test_gzip_chunk(tmp_path, engine, clean_table):
    _table(str(tmp_path), compression="gzip")
    msg = _scan_error(engine, str(tmp_path))
    assert msg.startswith("Error reading Parquet file: ") and "compression codec" in msg, msg
    _still_usable(engine, clean_table)
