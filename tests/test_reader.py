"""Streaming ParquetHandler reader (dk_reader_*, include/dkgpu.h) against the oracle.

Reference contract (ParquetHandler.java:59-68, ParquetFileReader.java:54-147, ParquetSchemaUtils.java:
92-138): batches of at most parquet.reader.batch-size rows, files in input order and rows in file
order, a batch never spans two files, an all-null column for a missing leaf, field-id then name then
case-insensitive matching, the row-index metadata column, row groups pruned by the predicate, and an
iterator that can be closed early. Every batch column is compared, concatenated per file, with the
oracle decoder's column (oracle/dk_ref.c via oracle/ref.py) bit for bit.
"""
import threading

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from delta_amd import kernel as K
from delta_amd import synth
from delta_amd._lib import DkError, dk_rg_filter
from delta_amd.partitions import RF_COL, RF_GT, RF_LIT, RL, pack_row_group_filter
from oracle import fieldids, ref

LEAVES = K.ADD_LEAVES + K.REMOVE_LEAVES


def _concat(batches, leaf):
    """Per-file concatenation of BatchColumns into the dk_column layout (int64 offsets from 0)."""
    cols = [b.columns[leaf] for b in batches]
    c0 = cols[0]
    out = dict(present=c0.present, row_def=np.concatenate([c.row_def for c in cols]))
    if not c0.present:
        return out
    if c0.max_rep > 0:
        ro, base = [np.zeros(1, np.int64)], 0
        for c in cols:
            ro.append(c.row_offs[1:] + base)
            base += int(c.row_offs[-1])
        out["row_offs"] = np.concatenate(ro)
        out["entry_def"] = np.concatenate([c.entry_def for c in cols])
    out["validity"] = np.concatenate([c.validity for c in cols])
    if c0.phys == 6:
        of, base = [np.zeros(1, np.int64)], 0
        for c in cols:
            of.append(c.offs[1:] + base)
            base += int(c.offs[-1])
        out["offs"] = np.concatenate(of)
        out["chars"] = np.concatenate([c.chars for c in cols])
    else:
        out["fixed"] = np.concatenate([c.fixed for c in cols])
    return out


def _assert_leaf(got, want, leaf):
    if want is None:
        assert not got["present"] or not got["row_def"].any(), leaf
        return
    assert got["present"], leaf
    np.testing.assert_array_equal(got["row_def"], want.row_def, err_msg=leaf)
    defs = want.entry_def if want.max_rep > 0 else want.row_def
    np.testing.assert_array_equal(got["validity"], defs == want.max_def, err_msg=leaf + " validity")
    if want.max_rep > 0:
        np.testing.assert_array_equal(got["row_offs"], want.row_offs, err_msg=leaf)
        np.testing.assert_array_equal(got["entry_def"], want.entry_def, err_msg=leaf)
    if want.phys == 6:
        np.testing.assert_array_equal(got["offs"], want.offs, err_msg=leaf)
        np.testing.assert_array_equal(got["chars"], want.chars, err_msg=leaf)
    else:
        np.testing.assert_array_equal(got["fixed"], want.fixed, err_msg=leaf)


def _check_files(paths, leaves, batches, batch_size, oracle_cols):
    by_file = {}
    last_file = -1
    for b in batches:
        assert 0 < b.n_rows <= batch_size
        assert b.file >= last_file                   # input-file order, never revisiting a file
        last_file = b.file
        by_file.setdefault(b.file, []).append(b)
    for fi, path in enumerate(paths):
        bs = by_file.get(fi, [])
        assert all(b.n_rows == batch_size for b in bs[:-1])
        want = oracle_cols(fi, path)
        for leaf in leaves:
            _assert_leaf(_concat(bs, leaf), want[leaf], leaf)


def _oracle(path, leaves):
    pf = ref.ParquetFile.open(path)
    return {leaf: pf.read(leaf) for leaf in leaves}


@pytest.mark.gpu
@pytest.mark.parametrize("spec,batch,window", [
    (dict(pv_keys=2, dv_frac=0.3, ckpt_removes=300, max_rows_per_page=3000), 1000, 3000),
    (dict(compression="snappy", n_parts=3, data_page_version="2.0", use_dictionary=False), 1024, 0),
    (dict(delta_binary_packed=True, with_stats=True, row_group_size=7000, variable_paths=True), 777, 5439),
])
def test_reader_matches_oracle(tmp_path, spec, batch, window):
    info = synth.write_table(str(tmp_path), synth.TableSpec(n_adds=20_000, n_commits=2, **spec))
    paths = info["checkpoint_files"]
    leaves = LEAVES + (["add.stats"] if spec.get("with_stats") else []) + ["add.noSuchLeaf"]
    eng = K.GpuEngine(parquet_batch_size=batch)
    with eng.readParquetFiles(paths, leaves, window_rows=window) as rd:
        batches = list(rd)
    _check_files(paths, leaves, batches, batch, lambda fi, p: _oracle(p, leaves))
    assert sum(b.n_rows for b in batches) == sum(ref.ParquetFile.open(p).num_rows for p in paths)


def _sorted_file(path, n=10_000, rg=1000):
    size = np.arange(n, dtype=np.int64) * 3
    t = pa.table({"add": pa.StructArray.from_arrays(
        [pa.array(["p%05d" % i for i in range(n)]), pa.array(size)], names=["path", "size"])})
    pq.write_table(t, path, row_group_size=rg)
    return size


@pytest.mark.gpu
def test_reader_row_index_and_row_group_pruning(tmp_path):
    p = str(tmp_path / "f.parquet")
    size = _sorted_file(p)
    # add.size > 16000: row groups 0..4 (max 14997) are pruned by their statistics, groups 5.. stay
    flt = pack_row_group_filter((["add.size"], [(RF_COL, 0, 0), (RF_LIT, RL["long"], 16000), (RF_GT, 0, 0)], b""),
                                dk_rg_filter)
    eng = K.GpuEngine(parquet_batch_size=512)
    with eng.readParquetFiles([p], ["add.path", "add.size", K.ROW_INDEX_COLUMN], predicate=flt,
                              window_rows=1536) as rd:
        batches = list(rd)
    ri = np.concatenate([b.row_index for b in batches])
    np.testing.assert_array_equal(ri, np.arange(5000, 10_000))        # file row indices, not reader rows
    got = np.concatenate([b.columns["add.size"].fixed for b in batches]).view("<i8")
    np.testing.assert_array_equal(got, size[5000:])                   # whole row groups: no row filtering
    # without a predicate the row index is simply 0..n-1
    with eng.readParquetFiles([p], [K.ROW_INDEX_COLUMN, "add.path"]) as rd:
        ri = np.concatenate([b.row_index for b in rd])
    np.testing.assert_array_equal(ri, np.arange(10_000))


@pytest.mark.gpu
def test_reader_early_close_and_late_release(tmp_path):
    p = str(tmp_path / "f.parquet")
    _sorted_file(p)
    eng = K.GpuEngine(parquet_batch_size=100)
    rd = eng.readParquetFiles([p, p], ["add.path", "add.size"], window_rows=300)
    raw = [rd.next_raw() for _ in range(5)]            # spans two windows
    rd.close()                                         # before exhaustion, batches still held
    first = raw[0].contents
    c = K.BatchColumn(first.cols[0], first.n_rows, "add.path")
    assert c.string(0) == b"p00000" and c.string(99) == b"p00099"
    last = K.BatchColumn(raw[4].contents.cols[1], raw[4].contents.n_rows, "add.size")
    assert last.fixed.view("<i8")[0] == 400 * 3
    for r in raw:
        K.ParquetReader.release(r)
    # a fresh reader over the same engine still works
    with eng.readParquetFiles([p], ["add.size"]) as rd2:
        assert sum(b.n_rows for b in rd2) == 10_000


def _ids_file(path, dup=False):
    def f(name, typ, fid):
        return pa.field(name, typ, metadata={b"PARQUET:field_id": str(fid).encode()})
    add = pa.struct([f("p_renamed", pa.string(), 10), f("SIZE", pa.int64(), 11 if not dup else 10),
                     f("size", pa.int64(), 12)])
    schema = pa.schema([f("add_x", add, 1)])
    n = 3000
    t = pa.table({"add_x": pa.StructArray.from_arrays(
        [pa.array(["f%d" % i for i in range(n)]), pa.array(np.arange(n, dtype=np.int64)),
         pa.array(np.arange(n, dtype=np.int64) * 7)], fields=list(add))}, schema=schema)
    pq.write_table(t, path, row_group_size=1000)


@pytest.mark.gpu
def test_reader_field_ids(tmp_path):
    p = str(tmp_path / "ids.parquet")
    _ids_file(p)
    eng = K.GpuEngine(parquet_batch_size=1000)
    # Kernel fields "add"(id 1).{"path"(id 10), "size" (no id), "Size"(id 11)}; "gone" (id 99, no name match)
    leaves = ["add.path", "add.size", "add.Size", "add.gone"]
    ids = {"add.path": [1, 10], "add.size": [1], "add.Size": [1, 11], "add.gone": [1, 99]}
    with eng.readParquetFiles([p], leaves, field_ids=ids) as rd:
        batches = list(rd)
    pf = ref.ParquetFile.open(p)
    for leaf in leaves:
        file_leaf = fieldids.resolve(p, leaf, ids[leaf])
        want = pf.read(file_leaf) if file_leaf else None
        _assert_leaf(_concat(batches, leaf), want, leaf)
    # the resolutions the reference makes: by id, exact name, id again; no match -> all null
    assert fieldids.resolve(p, "add.path", [1, 10]) == "add_x.p_renamed"
    assert fieldids.resolve(p, "add.size", [1]) == "add_x.size"
    assert fieldids.resolve(p, "add.Size", [1, 11]) == "add_x.SIZE"
    assert fieldids.resolve(p, "add.gone", [1, 99]) is None
    # without ids the names decide: "add" matches no top-level column
    with eng.readParquetFiles([p], ["add.path"]) as rd:
        assert not any(b.columns["add.path"].present for b in rd)


@pytest.mark.gpu
def test_reader_duplicate_field_ids_fail(tmp_path):
    p = str(tmp_path / "dup.parquet")
    _ids_file(p, dup=True)
    eng = K.GpuEngine()
    with pytest.raises(DkError, match="multiple columns .* same field id"):
        eng.readParquetFiles([p], ["add.size"], field_ids={"add.size": [1]})
    with pytest.raises(fieldids.DuplicateFieldId):
        fieldids.resolve(p, "add.size", [1])


@pytest.mark.gpu
def test_reader_threads_share_engine(tmp_path):
    info = synth.write_table(str(tmp_path), synth.TableSpec(n_adds=30_000, n_parts=4, n_commits=1,
                                                            compression="snappy"))
    paths = info["checkpoint_files"]
    eng = K.GpuEngine(parquet_batch_size=1024)
    out, errs = {}, []

    def work(i):
        try:
            with eng.readParquetFiles([paths[i]], ["add.path", "add.size"]) as rd:
                out[i] = list(rd)
        except Exception as e:        # surfaced below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(paths))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for i, p in enumerate(paths):
        want = _oracle(p, ["add.path", "add.size"])
        for leaf in ("add.path", "add.size"):
            _assert_leaf(_concat(out[i], leaf), want[leaf], leaf)


def test_oracle_field_id_resolution(tmp_path):
    """CPU: the oracle's ParquetSchemaUtils restatement on a file with ids, renames and case variants."""
    p = str(tmp_path / "ids.parquet")
    _ids_file(p)
    assert fieldids.resolve(p, "add_x.p_renamed") == "add_x.p_renamed"
    assert fieldids.resolve(p, "ADD_X.P_RENAMED") == "add_x.p_renamed"      # case-insensitive
    assert fieldids.resolve(p, "add_x.size") == "add_x.size"                # exact name beats case
    assert fieldids.resolve(p, "x.y", [1, 12]) == "add_x.size"              # ids beat names
    assert fieldids.resolve(p, "add_x.nope") is None
    d = str(tmp_path / "dup.parquet")
    _ids_file(d, dup=True)
    with pytest.raises(fieldids.DuplicateFieldId):
        fieldids.resolve(d, "add_x.size")           # the id map is built even when no id is asked
