"""Deterministic synthetic Delta tables (checkpoint Parquet + JSON commit tail).

Test and benchmark input tooling, not product code. Writes tables whose `_delta_log` has the layout
Delta Kernel reads:

* a checkpoint at version ``ckpt_version`` — classic single-part
  (``%020d.checkpoint.parquet``) or multi-part (``%020d.checkpoint.%010d.%010d.parquet``,
  ``kernel-api/.../internal/util/FileNames.java:191-201``) — with the Spark checkpoint column
  layout (optional ``add``/``remove``/``metaData``/``protocol`` structs, map<string,string>
  partitionValues as ``key_value`` repeated groups);
* ``n_commits`` newline-delimited JSON commits after it, mixing new adds, removes of checkpoint
  files, re-adds of removed paths and duplicate adds;
* ``_last_checkpoint``.

Paths follow ``<part>/part-<i%1000:05d>-<uuid4>.c000.snappy.parquet`` with ``<part>`` =
``date=2024-MM-DD``, seed 20250218 by default.
"""
from __future__ import annotations

import dataclasses
import json
import os
import sys
from dataclasses import dataclass, field

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

SEED = 20250218
HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
Z85 = np.frombuffer(
    b"0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#",
    dtype=np.uint8)

STR = pa.string()
MAP_SS = pa.map_(pa.string(), pa.string())
DV_TYPE = pa.struct([
    ("storageType", STR), ("pathOrInlineDv", STR), ("offset", pa.int32()),
    ("sizeInBytes", pa.int32()), ("cardinality", pa.int64()), ("maxRowIndex", pa.int64())])
STATS_PARSED_TYPE = pa.struct([
    ("numRecords", pa.int64()),
    ("minValues", pa.struct([("id", pa.int64()), ("name", STR)])),
    ("maxValues", pa.struct([("id", pa.int64()), ("name", STR)])),
    ("nullCount", pa.struct([("id", pa.int64()), ("name", pa.int64())]))])


@dataclass
class TableSpec:
    n_adds: int = 100_000
    n_parts: int = 1
    ckpt_version: int = 10
    n_commits: int = 10
    adds_per_commit: int = 50
    removes_per_commit: int = 50
    readd_frac: float = 0.1          # fraction of commit adds that re-add a removed path
    dup_frac: float = 0.05           # fraction of commit adds that duplicate an earlier commit add
    ckpt_removes: int = 0            # tombstone rows stored in the checkpoint (ignored by replay)
    pv_keys: int = 1                 # 1: {date}, 2: {date, region}
    with_stats: bool = False
    with_stats_parsed: bool = False
    dv_frac: float = 0.0
    compression: str = "none"
    data_page_version: str = "1.0"
    use_dictionary: bool = True
    delta_binary_packed: bool = False
    row_group_size: int = 1 << 20
    max_rows_per_page: int = 20_000  # parquet-mr 1.12 page row-count limit
    write_page_index: bool = True
    hot_frac: float = 0.0            # C5 skew: fraction of paths under one hot partition
    v2_sidecars: int = 0             # > 0: V2 checkpoint = manifest + this many sidecars
    v2_manifest: str = "parquet"     # V2 manifest format: "parquet" or "json"
    v2_json_adds: int = 0            # JSON manifest: this many add rows inline (+ a few removes, which
                                     # the reader ignores); the first commit removes a quarter of them
                                     # and re-adds another quarter
    variable_paths: bool = False     # add random suffixes / escapes so lengths vary
    seed: int = SEED
    extra: dict = field(default_factory=dict)


def _uuid4(rng, n):
    b = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    b[:, 6] = (b[:, 6] & 0x0F) | 0x40
    b[:, 8] = (b[:, 8] & 0x3F) | 0x80
    hx = np.empty((n, 32), dtype=np.uint8)
    hx[:, 0::2] = HEX[b >> 4]
    hx[:, 1::2] = HEX[b & 15]
    out = np.full((n, 36), ord("-"), dtype=np.uint8)
    out[:, 0:8] = hx[:, 0:8]
    out[:, 9:13] = hx[:, 8:12]
    out[:, 14:18] = hx[:, 12:16]
    out[:, 19:23] = hx[:, 16:20]
    out[:, 24:36] = hx[:, 20:32]
    return out


def _digits(vals, width):
    out = np.empty((len(vals), width), dtype=np.uint8)
    v = np.asarray(vals, dtype=np.int64).copy()
    for i in range(width - 1, -1, -1):
        out[:, i] = 48 + (v % 10)
        v //= 10
    return out


_MDAYS = np.array([31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31])


def _dates(day_idx):
    """day index 0..365 in 2024 -> (n, 10) 'YYYY-MM-DD' bytes."""
    cum = np.concatenate([[0], np.cumsum(_MDAYS)])
    month = np.searchsorted(cum, day_idx, side="right") - 1
    day = day_idx - cum[month] + 1
    out = np.empty((len(day_idx), 10), dtype=np.uint8)
    out[:, 0:4] = np.frombuffer(b"2024", dtype=np.uint8)
    out[:, 4] = ord("-")
    out[:, 5:7] = _digits(month + 1, 2)
    out[:, 7] = ord("-")
    out[:, 8:10] = _digits(day, 2)
    return out


def _strings_from_matrix(mat):
    n, w = mat.shape
    offs = np.arange(n + 1, dtype=np.int32) * w
    return pa.StringArray.from_buffers(n, pa.py_buffer(offs.tobytes()),
                                       pa.py_buffer(np.ascontiguousarray(mat).tobytes()))


def _strings_from_list(lst):
    return pa.array(lst, type=pa.string())


def gen_paths(rng, n, start_index, spec: TableSpec):
    """Returns (list-free) arrow string array of paths + the date-index per path."""
    n_days = 366
    day = rng.integers(0, n_days, size=n)
    if spec.hot_frac > 0:
        hot = rng.random(n) < spec.hot_frac
        day[hot] = 77
    prefix = np.frombuffer(b"date=", dtype=np.uint8)
    mat = np.empty((n, 83), dtype=np.uint8)
    mat[:, 0:5] = prefix
    mat[:, 5:15] = _dates(day)
    mat[:, 15:21] = np.frombuffer(b"/part-", dtype=np.uint8)
    mat[:, 21:26] = _digits((np.arange(n) + start_index) % 1000, 5)
    mat[:, 26] = ord("-")
    mat[:, 27:63] = _uuid4(rng, n)
    mat[:, 63:83] = np.frombuffer(b".c000.snappy.parquet", dtype=np.uint8)
    if not spec.variable_paths:
        return _strings_from_matrix(mat), day
    # variable lengths: random extra segment, occasional escapes (still valid java.net.URI input)
    base = [bytes(r).decode() for r in mat]
    extra = rng.integers(0, 40, size=n)
    kinds = rng.integers(0, 10, size=n)
    out = []
    for i, p in enumerate(base):
        k = kinds[i]
        if k == 0:
            p = p.replace(".c000", "-" + "x" * int(extra[i]) + ".c000")
        elif k == 1:
            p = "s3://Bucket-A/tbl/" + p
        elif k == 2:
            p = p.replace("date=", "dt%3A=%2f")
        elif k == 3:
            p = "file:/tmp/t%20x/" + p
        out.append(p)
    return _strings_from_list(out), day


def _pv_array(day, spec: TableSpec, rng):
    n = len(day)
    dates = _dates(np.asarray(day))
    if spec.pv_keys == 1:
        keys = _strings_from_matrix(np.tile(np.frombuffer(b"date", dtype=np.uint8), (n, 1)))
        vals = _strings_from_matrix(dates)
        offs = np.arange(n + 1, dtype=np.int32)
    else:
        regions = np.array([b"us-east", b"eu-west", b"ap-south"])
        r = rng.integers(0, 3, size=n)
        k = []
        v = []
        # interleave date/region per row
        kmat = np.empty((2 * n, 6), dtype=np.uint8)
        kmat[0::2] = np.frombuffer(b"date\0\0", dtype=np.uint8)
        kmat[1::2] = np.frombuffer(b"region", dtype=np.uint8)
        klen = np.empty(2 * n, dtype=np.int32)
        klen[0::2] = 4
        klen[1::2] = 6
        vmat = np.zeros((2 * n, 10), dtype=np.uint8)
        vmat[0::2] = dates
        vlen = np.empty(2 * n, dtype=np.int32)
        vlen[0::2] = 10
        for j, reg in enumerate(regions):
            m = np.where(r == j)[0]
            vmat[2 * m + 1, :len(reg)] = np.frombuffer(reg, dtype=np.uint8)
            vlen[2 * m + 1] = len(reg)
        keys = _ragged(kmat, klen)
        vals = _ragged(vmat, vlen)
        offs = np.arange(n + 1, dtype=np.int32) * 2
        del k, v
    return pa.MapArray.from_arrays(pa.array(offs), keys, vals)


def _ragged(mat, lens):
    n = mat.shape[0]
    offs = np.zeros(n + 1, dtype=np.int32)
    np.cumsum(lens, out=offs[1:])
    mask = np.arange(mat.shape[1])[None, :] < lens[:, None]
    data = mat[mask]
    return pa.StringArray.from_buffers(n, pa.py_buffer(offs.tobytes()), pa.py_buffer(data.tobytes()))


def _dv_array(rng, n, frac):
    present = rng.random(n) < frac
    m = int(present.sum())
    z = Z85[rng.integers(0, len(Z85), size=(m, 20))]
    st = _strings_from_matrix(np.full((m, 1), ord("u"), dtype=np.uint8))
    pid = _strings_from_matrix(z)
    off = pa.array(np.ones(m, dtype=np.int32))
    size = pa.array(rng.integers(30, 4000, size=m).astype(np.int32))
    card = pa.array(rng.integers(1, 1000, size=m).astype(np.int64))
    mri = pa.array([None] * m, type=pa.int64())
    dense = pa.StructArray.from_arrays([st, pid, off, size, card, mri],
                                       fields=list(DV_TYPE))
    return _spread(dense, present), present


def _spread(dense_arr, present):
    """Expand a dense array of len sum(present) into len(present) with nulls where ~present."""
    n = len(present)
    idx = np.full(n, -1, dtype=np.int64)
    idx[present] = np.arange(int(present.sum()))
    take_idx = pa.array(np.where(present, idx, 0))
    out = dense_arr.take(take_idx)
    mask = pa.array(~present)
    return _with_nulls(out, mask)


def _with_nulls(arr, mask):
    if isinstance(arr.type, pa.StructType):
        return pa.StructArray.from_arrays([arr.field(i) for i in range(arr.type.num_fields)],
                                          fields=list(arr.type), mask=mask)
    return pa.compute.if_else(mask, pa.scalar(None, type=arr.type), arr)


def _stats_json(ids_min, ids_max, names_min, names_max, nrec):
    return [
        '{"numRecords":%d,"minValues":{"id":%d,"name":"%s"},"maxValues":{"id":%d,"name":"%s"},'
        '"nullCount":{"id":0,"name":0}}' % (nrec[i], ids_min[i], names_min[i], ids_max[i], names_max[i])
        for i in range(len(nrec))]


def _add_struct(rng, n, start_index, spec: TableSpec, data_change: bool, paths=None, day=None):
    if paths is None:
        paths, day = gen_paths(rng, n, start_index, spec)
    pv = _pv_array(day, spec, rng)
    size = pa.array(rng.integers(1 << 20, 1 << 28, size=n, dtype=np.int64))
    mtime = pa.array(1_700_000_000_000 + rng.integers(0, 1_000_000_000, size=n, dtype=np.int64))
    dc = pa.array(np.full(n, data_change))
    tags = pa.nulls(n, type=MAP_SS)
    if spec.dv_frac > 0:
        dv, _ = _dv_array(rng, n, spec.dv_frac)
    else:
        dv = pa.nulls(n, type=DV_TYPE)
    brid = pa.nulls(n, type=pa.int64())
    drcv = pa.nulls(n, type=pa.int64())
    arrays = [paths, pv, size, mtime, dc, tags, dv, brid, drcv]
    fields = [("path", STR), ("partitionValues", MAP_SS), ("size", pa.int64()),
              ("modificationTime", pa.int64()), ("dataChange", pa.bool_()), ("tags", MAP_SS),
              ("deletionVector", DV_TYPE), ("baseRowId", pa.int64()),
              ("defaultRowCommitVersion", pa.int64())]
    if spec.with_stats or spec.with_stats_parsed:
        # 8-digit values (no leading zeros: stats must be valid JSON for Jackson)
        idmin = rng.integers(10_000_000, 50_000_000, size=n)
        idmax = idmin + rng.integers(0, 1_000_000, size=n)
        nrec = rng.integers(10_000_000, 100_000_000, size=n)
        nmat = np.empty((n, 7), dtype=np.uint8)
        nmat[:, 0] = ord("n")
        nmat[:, 1:] = _digits(rng.integers(0, 500_000, size=n), 6)
    if spec.with_stats:
        # {"numRecords":N,"minValues":{"id":A,"name":"nXXXXXX"},"maxValues":{...},"nullCount":{...}}
        parts = [b'{"numRecords":', None, b',"minValues":{"id":', None, b',"name":"', nmat,
                 b'"},"maxValues":{"id":', None, b',"name":"', nmat, b'"},"nullCount":{"id":0,"name":0}}']
        nums = {1: nrec, 3: idmin, 7: idmax}
        cols = []
        for i, p in enumerate(parts):
            if isinstance(p, bytes):
                cols.append(np.tile(np.frombuffer(p, dtype=np.uint8), (n, 1)))
            elif p is None:
                cols.append(_digits(nums[i], 8))
            else:
                cols.append(p)
        stats = _strings_from_matrix(np.concatenate(cols, axis=1))
        arrays.append(stats)
        fields.append(("stats", STR))
    if spec.with_stats_parsed:
        nm = _strings_from_matrix(nmat)
        sp = pa.StructArray.from_arrays([
            pa.array(nrec.astype(np.int64)),
            pa.StructArray.from_arrays([pa.array(idmin.astype(np.int64)), nm], names=["id", "name"]),
            pa.StructArray.from_arrays([pa.array(idmax.astype(np.int64)), nm], names=["id", "name"]),
            pa.StructArray.from_arrays([pa.array(np.zeros(n, np.int64)), pa.array(np.zeros(n, np.int64))],
                                       names=["id", "name"])], fields=list(STATS_PARSED_TYPE))
        arrays.append(sp)
        fields.append(("stats_parsed", STATS_PARSED_TYPE))
    return pa.StructArray.from_arrays(arrays, fields=[pa.field(a, t) for a, t in fields])


def _remove_type():
    return pa.struct([("path", STR), ("deletionTimestamp", pa.int64()), ("dataChange", pa.bool_()),
                      ("extendedFileMetadata", pa.bool_()), ("partitionValues", MAP_SS),
                      ("size", pa.int64()), ("deletionVector", DV_TYPE), ("baseRowId", pa.int64()),
                      ("defaultRowCommitVersion", pa.int64())])


METADATA_TYPE = pa.struct([
    ("id", STR), ("name", STR), ("description", STR),
    ("format", pa.struct([("provider", STR), ("options", MAP_SS)])),
    ("schemaString", STR), ("partitionColumns", pa.list_(STR)), ("configuration", MAP_SS),
    ("createdTime", pa.int64())])
PROTOCOL_TYPE = pa.struct([
    ("minReaderVersion", pa.int32()), ("minWriterVersion", pa.int32()),
    ("readerFeatures", pa.list_(STR)), ("writerFeatures", pa.list_(STR))])

SCHEMA_STRING = json.dumps({"type": "struct", "fields": [
    {"name": "id", "type": "long", "nullable": True, "metadata": {}},
    {"name": "name", "type": "string", "nullable": True, "metadata": {}},
    {"name": "date", "type": "string", "nullable": True, "metadata": {}}]}, separators=(",", ":"))


def _pm_rows(spec: TableSpec):
    proto = {"minReaderVersion": 3, "minWriterVersion": 7,
             "readerFeatures": ["deletionVectors", "v2Checkpoint"],
             "writerFeatures": ["deletionVectors", "v2Checkpoint"]}
    proto.update(spec.extra.get("protocol") or {})
    meta = {"id": "6f7a3d1e-2b0c-4c1e-9c4a-5a8e7d9b0c11", "name": None, "description": None,
            "format": {"provider": "parquet", "options": []},
            "schemaString": SCHEMA_STRING, "partitionColumns": ["date"],
            "configuration": [("delta.enableDeletionVectors", "true")],
            "createdTime": 1_700_000_000_000}
    return proto, meta


def _part_sizes(spec: TableSpec):
    n = spec.n_adds
    return [n // spec.n_parts + (1 if i < n % spec.n_parts else 0) for i in range(spec.n_parts)]


def _part_rng(spec: TableSpec, pi):
    """Each checkpoint part draws from its own stream, so parts can be generated in parallel and
    the table is the same whatever the worker count."""
    return np.random.Generator(np.random.PCG64([spec.seed, 1 + pi]))


def build_part_table(spec: TableSpec, pi, cnt, start, rng):
    """Arrow table of checkpoint part ``pi``: [protocol, metaData] rows (part 0 only) + ``cnt`` adds +
    ``ckpt_removes`` tombstones (part 0 only). Returns (table, add path array)."""
    proto, meta = _pm_rows(spec)
    adds = _add_struct(rng, cnt, start, spec, data_change=False)
    n_pm = 2 if pi == 0 else 0
    n_rm = spec.ckpt_removes if pi == 0 else 0
    total = n_pm + cnt + n_rm
    # row layout: [protocol, metaData] + adds + removes
    add_col = pa.concat_arrays([pa.nulls(n_pm, type=adds.type), adds,
                                pa.nulls(n_rm, type=adds.type)]) if (n_pm or n_rm) else adds
    rm_type = _remove_type()
    if n_rm:
        rpaths, rday = gen_paths(rng, n_rm, 10_000_000 + start, spec)
        rm = pa.StructArray.from_arrays([
            rpaths, pa.array(np.full(n_rm, 1_699_000_000_000, np.int64)), pa.array(np.ones(n_rm, bool)),
            pa.array(np.ones(n_rm, bool)), _pv_array(rday, spec, rng),
            pa.array(rng.integers(1 << 20, 1 << 28, size=n_rm, dtype=np.int64)),
            pa.nulls(n_rm, type=DV_TYPE), pa.nulls(n_rm, type=pa.int64()),
            pa.nulls(n_rm, type=pa.int64())], fields=list(rm_type))
        rm_col = pa.concat_arrays([pa.nulls(n_pm + cnt, type=rm_type), rm])
    else:
        rm_col = pa.nulls(total, type=rm_type)
    if n_pm:
        meta_col = pa.concat_arrays([pa.array([None, meta], type=METADATA_TYPE),
                                     pa.nulls(total - 2, type=METADATA_TYPE)])
        proto_col = pa.concat_arrays([pa.array([proto, None], type=PROTOCOL_TYPE),
                                      pa.nulls(total - 2, type=PROTOCOL_TYPE)])
    else:
        meta_col = pa.nulls(total, type=METADATA_TYPE)
        proto_col = pa.nulls(total, type=PROTOCOL_TYPE)
    t = pa.table({"add": add_col, "remove": rm_col, "metaData": meta_col, "protocol": proto_col})
    return t, adds.field("path")


def _part_job(job):
    """Build and write one checkpoint part (or V2 sidecar). Returns (part, {local add row: path} for
    the rows the commit tail picks, file size, (protocol row, metaData row) for a V2 part 0)."""
    spec, pi, cnt, start, path, picks, sidecar = job
    t, paths = build_part_table(spec, pi, cnt, start, _part_rng(spec, pi))
    pm = None
    if sidecar:
        if pi == 0:
            pm = (t.column("protocol")[0].as_py(), t.column("metaData")[1].as_py())
            t = t.slice(2)
        t = t.select(["add", "remove"])
    _write_parquet(t, path, spec)
    picked = {int(i): paths[int(i)].as_py() for i in picks}
    return pi, picked, os.path.getsize(path), pm


def _run_part_jobs(spec: TableSpec, jobs):
    """Parts of large tables are built in forked worker processes (call this before the process
    touches the GPU); small ones in-process. DK_SYNTH_WORKERS caps the worker count."""
    workers = min(len(jobs), int(os.environ.get("DK_SYNTH_WORKERS", "16")), os.cpu_count() or 1)
    progress = spec.extra.get("progress")
    if spec.n_adds < 2_000_000 or workers <= 1:
        out = []
        for j in jobs:
            out.append(_part_job(j))
            if progress:
                print("[synth] part %d/%d written" % (len(out), len(jobs)), file=sys.stderr, flush=True)
        return out
    import concurrent.futures as cf
    import multiprocessing as mp
    out = []
    with cf.ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("fork")) as ex:
        for r in ex.map(_part_job, jobs):
            out.append(r)
            if progress and (len(out) % 8 == 0 or len(out) == len(jobs)):
                print("[synth] part %d/%d written" % (len(out), len(jobs)), file=sys.stderr, flush=True)
    return out


def _write_parquet(table, path, spec: TableSpec):
    kw = dict(compression=spec.compression, data_page_version=spec.data_page_version,
              write_page_index=spec.write_page_index, row_group_size=spec.row_group_size,
              max_rows_per_page=spec.max_rows_per_page, write_statistics=True)
    if spec.delta_binary_packed:
        kw["use_dictionary"] = False
        kw["column_encoding"] = {c: "DELTA_BINARY_PACKED" for c in (
            "add.size", "add.modificationTime")}
    else:
        kw["use_dictionary"] = spec.use_dictionary
    pq.write_table(table, path, **kw)


def _json_add(path, day, size, mtime, dv=None, stats=None, pv_keys=1, region=None):
    d = {"path": path, "partitionValues": {"date": day}, "size": int(size),
         "modificationTime": int(mtime), "dataChange": True}
    if pv_keys == 2:
        d["partitionValues"]["region"] = region or "us-east"
    if stats is not None:
        d["stats"] = stats
    if dv is not None:
        d["deletionVector"] = dv
    return {"add": d}


def _json_remove(path, day, ts, dv=None):
    d = {"path": path, "deletionTimestamp": int(ts), "dataChange": True,
         "extendedFileMetadata": True, "partitionValues": {"date": day}, "size": 1234}
    if dv is not None:
        d["deletionVector"] = dv
    return {"remove": d}


CKPT_META_TYPE = pa.struct([("version", pa.int64()), ("tags", pa.map_(pa.string(), pa.string()))])
SIDECAR_TYPE = pa.struct([("path", pa.string()), ("sizeInBytes", pa.int64()), ("modificationTime", pa.int64()),
                          ("tags", pa.map_(pa.string(), pa.string()))])


def _uuid(rng):
    h = "".join("%02x" % b for b in rng.integers(0, 256, 16))
    return "%s-%s-%s-%s-%s" % (h[:8], h[8:12], h[12:16], h[16:20], h[20:])


def _write_v2_manifest(log, v, sidecars, pm, rng, spec: TableSpec):
    """V2 checkpoint (PROTOCOL.md "V2 Spec"): sidecars under _delta_log/_sidecars/ hold the add /
    remove rows (one per part, P&M rows dropped); the manifest ``<v>.checkpoint.<uuid>.parquet``
    (or ``.json``) holds protocol, metaData, checkpointMetadata and one sidecar row per file."""
    proto_row, meta_row = pm
    sc_rows = [{"path": name, "sizeInBytes": size, "modificationTime": 1_714_496_113_961, "tags": None}
               for name, size in sidecars]
    if spec.v2_manifest == "json":
        mfn = os.path.join(log, "%020d.checkpoint.%s.json" % (v, _uuid(rng)))
        # line order of the reference's GOLD/v2-checkpoint-json manifest
        lines = [{"checkpointMetadata": {"version": v}}]
        lines += [{"sidecar": {k: r[k] for k in ("path", "sizeInBytes", "modificationTime")}} for r in sc_rows]
        lines += [{"protocol": proto_row}, {"metaData": _meta_json(meta_row)}]
        if spec.v2_json_adds > 0:
            arr, day = gen_paths(rng, spec.v2_json_adds, 9_000_000, spec)
            spec.extra["manifest_adds"] = paths = arr.to_pylist()
            for i, pth in enumerate(paths):
                lines.append(_json_add(pth, "2024-01-01", 1000 + i, 1_700_000_000_000 + i, pv_keys=spec.pv_keys,
                                       stats='{"numRecords":1}' if i % 3 else None))
                if i % 7 == 3:      # a checkpoint remove: never a tombstone
                    lines.append(_json_remove(pth + ".old", "2024-01-01", 1_700_000_000_000))
        with open(mfn, "w") as f:
            f.write("\n".join(json.dumps(x) for x in lines) + "\n")
        return mfn
    n = 3 + len(sc_rows)
    t0, _ = build_part_table(dataclasses.replace(spec, ckpt_removes=0), 1, 0, 0, _part_rng(spec, 0))
    add_t, rm_t = t0.schema.field("add").type, t0.schema.field("remove").type
    man = pa.table({
        "add": pa.nulls(n, type=add_t), "remove": pa.nulls(n, type=rm_t),
        "metaData": pa.array([None, meta_row, None] + [None] * len(sc_rows), type=METADATA_TYPE),
        "protocol": pa.array([proto_row, None, None] + [None] * len(sc_rows), type=PROTOCOL_TYPE),
        "checkpointMetadata": pa.array([None, None, {"version": v, "tags": None}] + [None] * len(sc_rows),
                                       type=CKPT_META_TYPE),
        "sidecar": pa.array([None, None, None] + sc_rows, type=SIDECAR_TYPE)})
    mfn = os.path.join(log, "%020d.checkpoint.%s.parquet" % (v, _uuid(rng)))
    _write_parquet(man, mfn, spec)
    return mfn


def _meta_json(meta_row):
    """metaData row as a commit-JSON object (map columns come back from arrow as key/value pairs)."""
    m = dict(meta_row)
    fmt = dict(m.get("format") or {})
    fmt["options"] = dict(fmt.get("options") or [])
    m["format"] = fmt
    m["configuration"] = dict(m.get("configuration") or [])
    return {k: v for k, v in m.items() if v is not None}


def write_crc(root: str, version: int, spec: TableSpec = None, protocol=None, metadata=None, extra=None):
    """A Spark-style checksum file <version>.crc (one JSON object: table size, file counts, the
    protocol and the metadata -- the fields ChecksumReader / CRCInfo read) in root/_delta_log."""
    proto, meta = _pm_rows(spec or TableSpec())
    obj = {"tableSizeBytes": 0, "numFiles": 0, "numMetadata": 1, "numProtocol": 1,
           "protocol": protocol if protocol is not None else proto,
           "metadata": metadata if metadata is not None else _meta_json(meta)}
    obj.update(extra or {})
    path = os.path.join(root, "_delta_log", "%020d.crc" % version)
    with open(path, "w") as f:
        f.write(json.dumps(obj) + "\n")
    return path


def write_table(root: str, spec: TableSpec):
    """Write the synthetic table under ``root``. Returns a dict describing what was written."""
    rng = np.random.Generator(np.random.PCG64([spec.seed, 0]))     # commit tail, file names
    log = os.path.join(root, "_delta_log")
    os.makedirs(log, exist_ok=True)
    v = spec.ckpt_version
    per = _part_sizes(spec)
    starts = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    n_ck = int(starts[-1])
    # checkpoint rows the commit tail removes, drawn up front so each part hands back only those
    n_pool = spec.n_commits * spec.removes_per_commit
    pool = rng.integers(0, n_ck, size=n_pool) if n_ck else np.zeros(0, np.int64)
    owner = np.searchsorted(starts, pool, side="right") - 1
    sidecar = spec.v2_sidecars > 0
    jobs = []
    for pi, cnt in enumerate(per):
        if sidecar:
            side = os.path.join(log, "_sidecars")
            os.makedirs(side, exist_ok=True)
            path = os.path.join(side, "%020d.checkpoint.%010d.%010d.%s.parquet" % (v, pi + 1, spec.n_parts, _uuid(rng)))
        elif spec.n_parts == 1:
            path = os.path.join(log, "%020d.checkpoint.parquet" % v)
        else:
            path = os.path.join(log, "%020d.checkpoint.%010d.%010d.parquet" % (v, pi + 1, spec.n_parts))
        picks = np.unique(pool[owner == pi] - starts[pi])
        jobs.append((spec, pi, cnt, int(starts[pi]), path, picks, sidecar))
    results = sorted(_run_part_jobs(spec, jobs), key=lambda r: r[0])
    picked = {}
    for pi, pk, _, _ in results:
        for i, p in pk.items():
            picked[int(starts[pi]) + i] = p
    files = [j[4] for j in jobs]
    n_rows_total = n_ck + 2 + spec.ckpt_removes
    if sidecar:
        pm = results[0][3]
        man = _write_v2_manifest(log, v, [(os.path.basename(j[4]), r[2]) for j, r in zip(jobs, results)], pm, rng, spec)
        files = [man] + files
    lc = {"version": v, "size": int(n_rows_total)}
    if spec.n_parts > 1 and not sidecar:
        lc["parts"] = spec.n_parts
    with open(os.path.join(log, "_last_checkpoint"), "w") as f:
        f.write(json.dumps(lc))

    # ---- JSON commit tail ----
    new_serial = 0
    pool_i = 0
    added_in_tail = []      # paths added by commits (candidates for duplicates / removal)
    removed = []            # paths removed by commits (candidates for re-add)
    for c in range(spec.n_commits):
        ver = v + 1 + c
        lines = [json.dumps({"commitInfo": {"timestamp": 1_700_000_000_000 + ver,
                                            "operation": "WRITE"}})]
        if c == 0 and spec.extra.get("manifest_adds"):
            ma = spec.extra["manifest_adds"]
            q = max(1, len(ma) // 4)
            lines += [json.dumps(_json_remove(pth, "2024-01-01", 1_700_000_000_000 + ver)) for pth in ma[:q]]
            lines += [json.dumps(_json_add(pth, "2024-01-01", 77, 1_700_000_000_000 + ver, pv_keys=spec.pv_keys))
                      for pth in ma[q:2 * q]]
        # removes
        for _ in range(spec.removes_per_commit):
            pick = rng.random()
            if (pick < 0.5 or not added_in_tail) and pool_i < n_pool:
                p = picked[int(pool[pool_i])]
                pool_i += 1
            elif added_in_tail:
                p = added_in_tail[int(rng.integers(0, len(added_in_tail)))]
            else:
                continue
            removed.append(p)
            lines.append(json.dumps(_json_remove(p, "2024-01-01", 1_700_000_000_000 + ver)))
        # adds
        n_readd = int(round(spec.adds_per_commit * spec.readd_frac))
        n_dup = int(round(spec.adds_per_commit * spec.dup_frac))
        n_new = spec.adds_per_commit - n_readd - n_dup
        adds = []
        for _ in range(n_readd):
            if removed:
                adds.append(removed[int(rng.integers(0, len(removed)))])
        for _ in range(n_dup):
            if added_in_tail:
                adds.append(added_in_tail[int(rng.integers(0, len(added_in_tail)))])
        if n_new > 0:
            arr, day = gen_paths(rng, n_new, 5_000_000 + new_serial, spec)
            new_serial += n_new
            adds.extend(arr.to_pylist())
        for p in adds:
            dv = None
            if spec.dv_frac > 0 and rng.random() < spec.dv_frac:
                dv = {"storageType": "u",
                      "pathOrInlineDv": bytes(Z85[rng.integers(0, len(Z85), 20)]).decode(),
                      "offset": 1, "sizeInBytes": int(rng.integers(30, 4000)),
                      "cardinality": int(rng.integers(1, 1000))}
            stats = None
            if spec.with_stats and rng.random() >= 0.05:      # ~5% of commit adds carry no stats
                lo = int(rng.integers(0, 50_000_000))
                stats = ('{"numRecords":10,"minValues":{"id":%d,"name":"a"},"maxValues":'
                         '{"id":%d,"name":"z"},"nullCount":{"id":%d,"name":0}}'
                         % (lo, lo + 100, int(rng.integers(0, 3))))
            lines.append(json.dumps(_json_add(p, "2024-01-01", rng.integers(1 << 20, 1 << 28),
                                              1_700_000_000_000 + ver, dv=dv, stats=stats,
                                              pv_keys=spec.pv_keys)))
            added_in_tail.append(p)
        with open(os.path.join(log, "%020d.json" % ver), "w") as f:
            f.write("\n".join(lines) + "\n")
    return {"checkpoint_files": files, "version": v + spec.n_commits,
            "checkpoint_rows": n_ck}


# ---------------------------------------------------------------- typed add.stats_parsed tables
TYPED_STATS_COLUMNS = (("l", "long"), ("i", "integer"), ("d", "date"), ("ts", "timestamp"), ("tz", "timestamp_ntz"),
                       ("s", "string"), ("dc", "decimal(12,2)"), ("dd", "decimal(6,1)"), ("f", "float"),
                       ("g", "double"))
_TS_ALPHABET = ["a", "b", "c", "x", "y", "z", "é", "中", "\"", "\\", "\U0001f600"]


def _typed_value(rng, name, n_ts):
    """One stats value of column ``name``: (JSON text fragment, typed Python value), or None (no stat)."""
    import datetime
    import decimal
    if rng.random() < 0.05:
        return None
    if name == "l" or name.startswith("x"):
        v = int(rng.integers(-10 ** 6, 10 ** 6)) * 1_000_003 if name == "l" else int(rng.integers(-200, 200))
        return str(v), v
    if name == "i":
        v = int(rng.integers(-(1 << 31), 1 << 31))
        return str(v), v
    if name == "d":
        v = int(rng.integers(-3000, 20000))
        return '"%s"' % (datetime.date(1970, 1, 1) + datetime.timedelta(days=v)).isoformat(), v
    if name in ("ts", "tz"):
        ms = int(rng.integers(-10 ** 11, 2 * 10 ** 12))
        t = datetime.datetime(1970, 1, 1) + datetime.timedelta(milliseconds=ms)
        text = t.strftime("%Y-%m-%dT%H:%M:%S.") + "%03d" % (t.microsecond // 1000) + ("Z" if name == "ts" else "")
        return '"%s"' % text, ms * (1 if n_ts == "ms" else 1000)
    if name == "s":
        k = int(rng.integers(0, 7))
        v = "".join(_TS_ALPHABET[int(j)] for j in rng.integers(0, len(_TS_ALPHABET), size=k))
        return json.dumps(v, ensure_ascii=bool(rng.integers(0, 2))), v
    if name in ("dc", "dd"):
        scale, lim = (2, 10 ** 11) if name == "dc" else (1, 99_999)
        u = int(rng.integers(-lim, lim + 1))
        d = decimal.Decimal(u).scaleb(-scale)
        return str(d), d
    # float / double: specials (NaN / Infinity as JSON strings, -0.0 as a number) and plain values
    c = rng.random()
    if c < 0.04:
        v = float("nan")
    elif c < 0.07:
        v = float("inf")
    elif c < 0.10:
        v = float("-inf")
    elif c < 0.15:
        v = -0.0
    elif c < 0.20:
        v = 0.0
    else:
        v = float(rng.normal() * 1000.0)
        if name == "f":
            v = float(np.float32(v))
    if v != v:
        return '"NaN"', v
    if v in (float("inf"), float("-inf")):
        return '"%s"' % ("Infinity" if v > 0 else "-Infinity"), v
    return repr(v), v


def write_typed_stats_table(root, n=3000, seed=7, ts_unit="us", n_tail=40, extra_long=0):
    """A table whose checkpoint adds carry add.stats (Delta's JSON) and add.stats_parsed (Spark's
    from_json(stats): the same values, typed) for every stats type of TYPED_STATS_COLUMNS: long, int,
    date, timestamp / timestamp_ntz (INT64 ``ts_unit`` "us" or "ms", or INT96 for "int96"), string
    (with escapes and multi-byte UTF-8), decimal as INT64 / INT32, float, double (NaN, +-Infinity,
    -0.0, which Kernel reads from "-0.0" as +0.0). Some rows have JSON stats and a null stats_parsed,
    some a null JSON and typed stats (the reference reads only the JSON: kept), some neither. A
    commit after the checkpoint adds ``n_tail`` files with JSON stats and removes a few. Returns
    {column: [typed min values]} for building predicates. extra_long: that many more long columns
    x0, x1, ... with small values (wide filters)."""
    import decimal
    rng = np.random.default_rng(seed)
    log = os.path.join(root, "_delta_log")
    os.makedirs(log, exist_ok=True)
    columns = list(TYPED_STATS_COLUMNS) + [("x%d" % k, "long") for k in range(extra_long)]
    names = [c for c, _ in columns]
    unit = "us" if ts_unit == "int96" else ts_unit
    typ = {"l": pa.int64(), "i": pa.int32(), "d": pa.date32(), "ts": pa.timestamp(unit, tz="UTC"),
           "tz": pa.timestamp(unit), "s": STR, "dc": pa.decimal128(12, 2), "dd": pa.decimal128(6, 1),
           "f": pa.float32(), "g": pa.float64()}
    typ.update({"x%d" % k: pa.int64() for k in range(extra_long)})
    vals_t = pa.struct([(c, typ[c]) for c in names])
    nc_t = pa.struct([(c, pa.int64()) for c in names])
    sp_t = pa.struct([("numRecords", pa.int64()), ("minValues", vals_t), ("maxValues", vals_t), ("nullCount", nc_t)])
    schema = {"type": "struct", "fields": [{"name": c, "type": t, "nullable": True, "metadata": {}}
                                           for c, t in columns]}
    proto = {"minReaderVersion": 1, "minWriterVersion": 2}
    meta = {"id": "typed-stats", "format": {"provider": "parquet", "options": {}},
            "schemaString": json.dumps(schema), "partitionColumns": [], "configuration": {}, "createdTime": 0}
    mins = {c: [] for c in names}

    def stats_row():
        nrec = int(rng.integers(1, 1000))
        js, parsed = {}, {"numRecords": nrec, "minValues": {}, "maxValues": {}, "nullCount": {}}
        for side in ("minValues", "maxValues"):
            parts = []
            for c in names:
                tv = _typed_value(rng, c, unit)
                parsed[side][c] = None if tv is None else tv[1]
                if tv is not None:
                    parts.append('"%s":%s' % (c, tv[0]))
                    if side == "minValues":
                        mins[c].append(tv[1])
            js[side] = "{" + ",".join(parts) + "}"
        ncs = {c: int(rng.integers(0, 3)) for c in names}
        parsed["nullCount"] = ncs
        text = '{"numRecords":%d,"minValues":%s,"maxValues":%s,"nullCount":{%s}}' % (
            nrec, js["minValues"], js["maxValues"], ",".join('"%s":%d' % (c, ncs[c]) for c in names))
        return text, parsed

    adds, stats, sps = [], [], []
    for k in range(n):
        text, parsed = stats_row()
        if k % 53 == 5:
            text = None
        if k % 59 == 7:
            parsed = None
        if k % 61 == 9:
            text = parsed = None
        adds.append("f%05d.parquet" % k)
        stats.append(text)
        sps.append(parsed)
    add_t = pa.struct([("path", STR), ("partitionValues", MAP_SS), ("size", pa.int64()),
                       ("modificationTime", pa.int64()), ("dataChange", pa.bool_()), ("stats", STR),
                       ("stats_parsed", sp_t)])
    rows = [{"path": p, "partitionValues": [], "size": 1000 + i, "modificationTime": 1_700_000_000_000,
             "dataChange": False, "stats": st, "stats_parsed": sp} for i, (p, st, sp) in enumerate(zip(adds, stats, sps))]
    total = n + 2
    add_col = pa.concat_arrays([pa.nulls(2, type=add_t), pa.array(rows, type=add_t)])
    t = pa.table({"protocol": pa.array([proto, None] + [None] * n, type=PROTOCOL_TYPE),
                  "metaData": pa.array([None, dict(meta, format={"provider": "parquet", "options": []},
                                                   configuration=[])] + [None] * n, type=METADATA_TYPE),
                  "add": add_col, "remove": pa.nulls(total, type=_remove_type())})
    pq.write_table(t, os.path.join(log, "%020d.checkpoint.parquet" % 0), compression="snappy",
                   row_group_size=1024, store_decimal_as_integer=True,
                   use_deprecated_int96_timestamps=ts_unit == "int96")
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        f.write(json.dumps({"protocol": proto}) + "\n" + json.dumps({"metaData": meta}) + "\n")
        for p, st in zip(adds, stats):
            a = {"path": p, "partitionValues": {}, "size": 1, "modificationTime": 0, "dataChange": True}
            if st is not None:
                a["stats"] = st
            f.write(json.dumps({"add": a}) + "\n")
    with open(os.path.join(log, "_last_checkpoint"), "w") as f:
        f.write(json.dumps({"version": 0, "size": total}) + "\n")
    with open(os.path.join(log, "%020d.json" % 1), "w") as f:
        for k in range(n_tail):
            a = {"path": "t%05d.parquet" % k, "partitionValues": {}, "size": 1, "modificationTime": 0,
                 "dataChange": True, "stats": stats_row()[0]}
            f.write(json.dumps({"add": a}) + "\n")
        for k in range(0, n, max(1, n // 20)):
            f.write(json.dumps({"remove": {"path": adds[k], "deletionTimestamp": 1, "dataChange": True}}) + "\n")
    del decimal
    return mins
