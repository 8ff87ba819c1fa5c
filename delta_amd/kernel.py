"""Python mirror of the Delta Kernel read surface over libdkgpu (the role JNI plays for Java).

Reference surface (paths under /root/reference/kernel/kernel-api/src/main/java/io/delta/kernel/):
  Table.forPath / getLatestSnapshot          Table.java:56-58,76; internal/TableImpl.java:65-103
  SnapshotManager.getLogSegmentForVersion    internal/snapshot/SnapshotManager.java:311-566
  LogSegment.allLogFilesReversed             internal/snapshot/LogSegment.java:166-178
  Snapshot.getScanBuilder / ScanBuilder.build   Snapshot.java:69; internal/ScanBuilderImpl.java:77-86
  Scan.getScanFiles -> FilteredColumnarBatch Scan.java:101; internal/ScanImpl.java:120-186
  ScanMetrics counters                       internal/metrics/ScanMetrics.java:28-40

Log-segment selection is Kernel host logic the GPU engine does not replace; it is
restated here because the JVM is absent. Decode, key building and reconciliation all run in
libdkgpu on the GPU; nothing here computes a selection.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import re
import time
import weakref
from dataclasses import dataclass, field

import numpy as np

from ._lib import (MAX_LEAF_DEPTH, Column, DkError, check, dk_batch, dk_column, dk_config, dk_dv_descriptor,
                   dk_read_options, dk_rg_filter, lib)

ADD_LEAVES = ["add.path", "add.partitionValues.key_value.key", "add.partitionValues.key_value.value",
              "add.size", "add.modificationTime", "add.dataChange",
              "add.deletionVector.storageType", "add.deletionVector.pathOrInlineDv",
              "add.deletionVector.offset", "add.deletionVector.sizeInBytes",
              "add.deletionVector.cardinality", "add.tags.key_value.key", "add.tags.key_value.value",
              "add.baseRowId", "add.defaultRowCommitVersion"]
STATS_LEAF = "add.stats"
REMOVE_LEAVES = ["remove.path", "remove.deletionVector.storageType", "remove.deletionVector.pathOrInlineDv",
                 "remove.deletionVector.offset", "remove.deletionVector.sizeInBytes",
                 "remove.deletionVector.cardinality"]
PM_LEAVES = ["protocol.minReaderVersion", "protocol.minWriterVersion",
             "protocol.readerFeatures.list.element", "protocol.writerFeatures.list.element",
             "metaData.id", "metaData.name", "metaData.description", "metaData.format.provider",
             "metaData.format.options.key_value.key", "metaData.format.options.key_value.value",
             "metaData.schemaString", "metaData.partitionColumns.list.element",
             "metaData.configuration.key_value.key", "metaData.configuration.key_value.value",
             "metaData.createdTime"]
SIDECAR_LEAVES = ["sidecar.path", "sidecar.sizeInBytes", "sidecar.modificationTime"]

TIMING = 1


def scan_groups(n_files):
    """Groups of checkpoint files for a grouped getScanFiles run (dk_replay_run_grouped): about 8
    files per group, at most 8 groups; DK_SCAN_GROUPS overrides (0: one ungrouped run)."""
    env = os.environ.get("DK_SCAN_GROUPS")
    if env is not None:
        return max(0, min(int(env), n_files))
    return 0 if n_files <= 1 else min(8, max(2, n_files // 8))


def _cstrs(items):
    arr = (C.c_char_p * len(items))()
    arr[:] = [s.encode() if isinstance(s, str) else s for s in items]
    return arr


class GpuEngine:
    """Engine (engine/Engine.java:30-64) backed by one MI355X."""

    def __init__(self, parquet_batch_size=1024, json_batch_size=1024, device=0, timing=False):
        self.cfg = dk_config(parquet_batch_size, json_batch_size, device, TIMING if timing else 0)
        self._h = C.c_void_p()
        check(lib().dk_engine_create(C.byref(self.cfg), C.byref(self._h)))

    create = classmethod(lambda cls, **kw: cls(**kw))

    @property
    def json_batch_size(self):
        return self.cfg.json_batch_size

    def close(self):
        if self._h:
            lib().dk_engine_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ParquetHandler.readParquetFiles (engine/ParquetHandler.java:64-68)
    def read_parquet_files(self, paths, leaves):
        return ParquetSet(self, paths, leaves)

    def readParquetFiles(self, paths, leaves, predicate=None, field_ids=None, window_rows=0):
        """ParquetHandler.readParquetFiles as a Kernel caller consumes it: an iterator of ColumnarBatch
        (<= parquet_batch_size rows, file by file, never spanning files), closable before exhaustion.
        leaves: projected leaf paths; ROW_INDEX_COLUMN among them requests the row-index metadata
        column. predicate: optional dk_rg_filter (row-group pruning, best effort). field_ids: optional
        {leaf: [id or -1 per dotted component]} (parquet.field.id of the Kernel fields)."""
        return ParquetReader(self, paths, leaves, predicate, field_ids, window_rows)


def prune_row_groups(path, packed_filter):
    """Row groups of `path` that survive the checkpoint predicate (dk_parquet_prune_row_groups)."""
    cap = 4096
    keep = (C.c_uint8 * cap)()
    n = C.c_int32()
    check(lib().dk_parquet_prune_row_groups(path.encode(), C.byref(packed_filter), keep, cap, C.byref(n)))
    if n.value > cap:
        raise DkError("%s has more than %d row groups" % (path, cap))
    return [g for g in range(n.value) if keep[g]]


def nonnull_row_groups(path, leaf):
    """keep flag per row group: False where footer statistics show `leaf` null in every row."""
    cap = 4096
    keep = (C.c_uint8 * cap)()
    n = C.c_int32()
    check(lib().dk_parquet_nonnull_row_groups(path.encode(), leaf.encode(), keep, cap, C.byref(n)))
    if n.value > cap:
        raise DkError("%s has more than %d row groups" % (path, cap))
    return [bool(keep[g]) for g in range(n.value)]


def row_group_rows(path):
    """Row counts of a Parquet file's row groups (footer only)."""
    cap = 4096
    rows = (C.c_int64 * cap)()
    n = C.c_int32()
    check(lib().dk_parquet_row_groups(path.encode(), rows, cap, C.byref(n)))
    if n.value > cap:
        raise DkError("%s has more than %d row groups" % (path, cap))
    return [int(rows[i]) for i in range(n.value)]


class ParquetSet:
    """A set of Parquet files decoded on the GPU (one batch per file; batches in input order)."""

    def __init__(self, engine: GpuEngine, paths, leaves, row_groups=None, groups=None, async_open=False):
        """row_groups: optional [(first, end)] row-group range per file (dk_parquet_open_rg);
        groups: optional list of row-group indices per file (dk_parquet_open_sel);
        async_open: return once the tables are read, the files being read, sized and decoded on a
        library thread meanwhile (dk_parquet_open_async; every call waits for what it needs)."""
        self.engine = engine
        self.paths = list(paths)
        self.leaves = list(leaves)
        self._h = C.c_void_p()
        self.async_open = bool(async_open and row_groups is None)
        if async_open and row_groups is None:
            cnt = lst = None
            if groups is not None:
                cnt = (C.c_int32 * max(1, len(groups)))(*[len(g) for g in groups])
                flat = [g for gs in groups for g in gs]
                lst = (C.c_int32 * max(1, len(flat)))(*flat)
            check(lib().dk_parquet_open_async(engine._h, _cstrs(self.paths), len(self.paths), _cstrs(self.leaves),
                                              len(self.leaves), cnt, lst, C.byref(self._h)))
        elif groups is not None:
            cnt = (C.c_int32 * max(1, len(groups)))(*[len(g) for g in groups])
            flat = [g for gs in groups for g in gs]
            lst = (C.c_int32 * max(1, len(flat)))(*flat)
            check(lib().dk_parquet_open_sel(engine._h, _cstrs(self.paths), len(self.paths), _cstrs(self.leaves),
                                            len(self.leaves), cnt, lst, C.byref(self._h)))
        elif row_groups is None:
            check(lib().dk_parquet_open(engine._h, _cstrs(self.paths), len(self.paths), _cstrs(self.leaves),
                                        len(self.leaves), C.byref(self._h)))
        else:
            lo = (C.c_int32 * max(1, len(row_groups)))(*[a for a, _ in row_groups])
            hi = (C.c_int32 * max(1, len(row_groups)))(*[b for _, b in row_groups])
            check(lib().dk_parquet_open_rg(engine._h, _cstrs(self.paths), len(self.paths), _cstrs(self.leaves),
                                           len(self.leaves), lo, hi, C.byref(self._h)))

    def decode(self):
        check(lib().dk_parquet_decode(self._h))
        check(lib().dk_parquet_sync(self._h))
        return self

    def num_rows(self, file_idx):
        return lib().dk_parquet_num_rows(self._h, file_idx)

    def row_offset(self, file_idx):
        """File row index of this set's first row of the file (non-zero for a row-group shard)."""
        return lib().dk_parquet_row_offset(self._h, file_idx)

    def column(self, file_idx, leaf, copy=True) -> Column:
        """copy=False: a view of the library's pinned mirror, valid until the next decode / close."""
        c = dk_column()
        check(lib().dk_parquet_column(self._h, file_idx, self.leaves.index(leaf), C.byref(c)))
        return Column(c, leaf, copy)

    def first_row(self, file_idx, leaf, min_def=1):
        """Index of the first row whose definition level is >= min_def, or -1 (device scan)."""
        r = C.c_int64()
        check(lib().dk_parquet_first_row(self._h, file_idx, self.leaves.index(leaf), min_def, C.byref(r)))
        return r.value

    def column_rows(self, file_idx, leaf, row0, n) -> Column:
        """Rows [row0, row0 + n) of a decoded column, offsets rebased to the slice."""
        c = dk_column()
        check(lib().dk_parquet_column_rows(self._h, file_idx, self.leaves.index(leaf), row0, n, C.byref(c)))
        return Column(c, leaf)

    def columns(self, file_idx):
        """leaf -> Column, or None when the file lacks the leaf (all-null, NonExistentColumnReader)."""
        out = {}
        for leaf in self.leaves:
            c = self.column(file_idx, leaf)
            out[leaf] = c if c.present else None
        return out

    def traffic(self):
        r, w = C.c_int64(), C.c_int64()
        check(lib().dk_parquet_traffic(self._h, C.byref(r), C.byref(w)))
        return r.value, w.value

    def kernel_traffic(self, kernel):
        """Algorithmic (read, written) bytes of one launch of a decode kernel."""
        r, w = C.c_int64(), C.c_int64()
        check(lib().dk_parquet_kernel_traffic(self._h, kernel.encode(), C.byref(r), C.byref(w)))
        return r.value, w.value

    def close(self):
        if self._h:
            lib().dk_parquet_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


ROW_INDEX_COLUMN = "_metadata.row_index"     # StructField.METADATA_ROW_INDEX_COLUMN_NAME


def _np_view(ptr, n, dtype):
    if not ptr or n <= 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,))


class BatchColumn:
    """One leaf of a ColumnarBatch, copied out of the batch's pinned buffers. Offsets are rebased to the
    batch (row_offs / offs start at 0), so the layout equals a dk_column slice of the same rows."""

    def __init__(self, c, n_rows, path):
        self.path = path
        self.present = bool(c.present)
        self.n_rows = n_rows
        self.phys, self.width, self.max_def, self.max_rep, self.rep_def = c.phys, c.width, c.max_def, c.max_rep, c.rep_def
        self.row_def = _np_view(c.row_def, n_rows, np.uint8).copy()
        self.row_offs = self.entry_def = self.fixed = self.offs = self.chars = self.validity = None
        if not self.present:
            return
        v0, nv = c.value_offset, c.n_values
        if c.max_rep > 0:
            ro = _np_view(c.row_offs, n_rows + 1, np.int32).astype(np.int64)
            self.row_offs = ro - ro[0]
            self.entry_def = _np_view(c.entry_def, v0 + nv, np.uint8)[v0:].copy()
        bits = _np_view(c.validity, (v0 + nv + 7) // 8, np.uint8)
        self.validity = np.unpackbits(bits, bitorder="little")[v0:v0 + nv].astype(bool)
        if c.phys == 6:
            o = _np_view(c.offs, v0 + nv + 1, np.int32)[v0:].astype(np.int64)
            self.chars = _np_view(c.chars, int(o[-1]) if nv >= 0 else 0, np.uint8)[o[0]:o[-1]].copy() \
                if o[-1] > o[0] else np.zeros(0, np.uint8)
            self.offs = o - o[0]
        else:
            self.fixed = _np_view(c.fixed, (v0 + nv) * c.width, np.uint8)[v0 * c.width:].copy()

    def string(self, i):
        return bytes(self.chars[self.offs[i]:self.offs[i + 1]])


class ColumnarBatch:
    """A batch from ParquetReader: columns by leaf path (requested order), plus the row index."""

    def __init__(self, b: dk_batch, leaves, want_row_index):
        self.file = b.file
        self.n_rows = b.n_rows
        self.columns = {leaf: BatchColumn(b.cols[i], b.n_rows, leaf) for i, leaf in enumerate(leaves)}
        self.row_index = _np_view(b.row_index, b.n_rows, np.int64).copy() if want_row_index else None


class ParquetReader:
    """Iterator over dk_reader batches; close() early is safe (ScanImpl.java:376-392)."""

    def __init__(self, engine, paths, leaves, predicate=None, field_ids=None, window_rows=0):
        self.paths = list(paths)
        self.want_row_index = ROW_INDEX_COLUMN in leaves
        self.leaves = [x for x in leaves if x != ROW_INDEX_COLUMN]
        opt = dk_read_options()
        self._ids = None
        if field_ids:
            ids = np.full(len(self.leaves) * MAX_LEAF_DEPTH, -1, np.int32)
            for i, leaf in enumerate(self.leaves):
                for d, v in enumerate((field_ids.get(leaf) or [])[:MAX_LEAF_DEPTH]):
                    ids[i * MAX_LEAF_DEPTH + d] = -1 if v is None else v
            self._ids = ids
            opt.field_ids = ids.ctypes.data
        self._pred = predicate
        opt.predicate = C.cast(C.byref(predicate), C.c_void_p) if predicate is not None else None
        opt.row_index = 1 if self.want_row_index else 0
        opt.window_rows = window_rows
        self._h = C.c_void_p()
        check(lib().dk_reader_open(engine._h, _cstrs(self.paths), len(self.paths), _cstrs(self.leaves),
                                   len(self.leaves), C.byref(opt), C.byref(self._h)))

    def num_rows(self, file_idx):
        return lib().dk_reader_num_rows(self._h, file_idx)

    def next_raw(self):
        """The next dk_batch pointer (caller releases it with release()), or None at the end."""
        out = C.POINTER(dk_batch)()
        check(lib().dk_reader_next(self._h, C.byref(out)))
        return out if out else None

    @staticmethod
    def release(raw):
        lib().dk_batch_release(raw)

    def __iter__(self):
        return self

    def __next__(self):
        raw = self.next_raw()
        if raw is None:
            raise StopIteration
        try:
            return ColumnarBatch(raw.contents, self.leaves, self.want_row_index)
        finally:
            lib().dk_batch_release(raw)

    def close(self):
        if self._h:
            lib().dk_reader_close(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeletionVectors:
    """The DVs of a set of scan files, loaded into dense deleted-row bitmaps on the GPU
    (DeletionVectorUtils.loadNewDvAndBitmap, DeletionVectorUtils.java:27-37). descriptors: tuples
    (storageType, pathOrInlineDv, offset or None, sizeInBytes, cardinality)."""

    def __init__(self, engine, table_root, descriptors):
        self.n = len(descriptors)
        arr = (dk_dv_descriptor * max(1, self.n))()
        self._keep = []
        for i, (st, pd, off, size, card) in enumerate(descriptors):
            a, b = st.encode(), pd.encode()
            self._keep += [a, b]
            arr[i].storage_type, arr[i].path_or_inline = a, b
            arr[i].has_offset = 0 if off is None else 1
            arr[i].offset = off or 0
            arr[i].size_in_bytes, arr[i].cardinality = size, card
        self._h = C.c_void_p()
        check(lib().dk_dv_load(engine._h, table_root.encode(), arr, self.n, C.byref(self._h)))

    def num_bits(self, i):
        return lib().dk_dv_num_bits(self._h, i)

    def deleted(self, i):
        """Bool per row index (up to the largest deleted row): True = deleted."""
        nb = self.num_bits(i)
        buf = np.zeros(max(1, (nb + 7) // 8), np.uint8)
        check(lib().dk_dv_bitmap(self._h, i, buf.ctypes.data, buf.size, 0))
        return np.unpackbits(buf, bitorder="little")[:nb].astype(bool)

    def selection(self, i, row_index):
        """SelectionColumnVector: True where the row survives DV i."""
        ri = np.ascontiguousarray(row_index, dtype=np.int64)
        sel = np.zeros(max(1, ri.size), np.uint8)
        check(lib().dk_dv_selection(self._h, i, ri.ctypes.data, ri.size, sel.ctypes.data))
        return sel[:ri.size].astype(bool)

    def close(self):
        if self._h:
            lib().dk_dv_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _dv_of(data, r):
    """(storageType, pathOrInlineDv, offset, sizeInBytes, cardinality) of scan-file row r, or None."""
    st = data["add.deletionVector.storageType"]
    if st is None or not st.present or st.row_def[r] < st.max_def:
        return None
    off = data["add.deletionVector.offset"]
    has_off = off is not None and off.present and off.row_def[r] == off.max_def
    size = data["add.deletionVector.sizeInBytes"].fixed.view("<i4")[r]
    card = data["add.deletionVector.cardinality"].fixed.view("<i8")[r]
    return (st.string(r).decode(), data["add.deletionVector.pathOrInlineDv"].string(r).decode(),
            int(off.fixed.view("<i4")[r]) if has_off else None, int(size), int(card))


def read_scan_data(engine, scan, leaves):
    """Scan.transformPhysicalData over every selected scan file (Scan.java:147-230): each data file
    is read with the row-index metadata column (readParquetFiles) and, when the scan file carries a
    deletion vector, filtered by it (SelectionColumnVector). Yields (add.path, ColumnarBatch,
    selection or None)."""
    from urllib.parse import unquote
    root = scan.table_root()
    files = []
    for b in scan.getScanFiles(engine):
        for r in b.selected_rows():
            files.append((b.data["add.path"].string(int(r)).decode(), _dv_of(b.data, int(r))))
    with_dv = [dv for _, dv in files if dv is not None]
    dvs = DeletionVectors(engine, root, with_dv) if with_dv else None
    k = 0
    for path, dv in files:
        full = path if re.match(r"^[A-Za-z][A-Za-z0-9+.-]*:", path) else root.rstrip("/") + "/" + unquote(path)
        local = full[5:] if full.startswith("file:") else full
        with engine.readParquetFiles([local], list(leaves) + [ROW_INDEX_COLUMN]) as rd:
            for batch in rd:
                sel = dvs.selection(k, batch.row_index) if dv is not None else None
                yield path, batch, sel
        if dv is not None:
            k += 1
    if dvs is not None:
        dvs.close()


class JsonTail:
    """Commit files parsed on the host (DefaultJsonHandler.readJsonFiles semantics), optionally
    followed by JSON-format checkpoint parts (a V2 checkpoint's JSON manifest): rows
    [ckpt_row0, rows) are those parts' rows, whose adds reconcile as checkpoint adds."""

    def __init__(self, engine: GpuEngine, commit_paths, versions, with_stats=False, checkpoint_paths=()):
        self._h = C.c_void_p()
        paths = list(commit_paths) + list(checkpoint_paths)
        versions = list(versions) + [0] * len(checkpoint_paths)
        vers = (C.c_int64 * max(1, len(versions)))(*versions)
        check(lib().dk_json_tail_parse_parts(engine._h, _cstrs(paths), vers, len(paths), len(checkpoint_paths),
                                             1 if with_stats else 0, C.byref(self._h)))
        self.rows = lib().dk_json_tail_rows(self._h)
        self.ckpt_row0 = lib().dk_json_tail_checkpoint_row0(self._h)

    def column(self, leaf) -> Column:
        c = dk_column()
        check(lib().dk_json_tail_column(self._h, leaf.encode(), C.byref(c)))
        return Column(c, leaf)

    def close(self):
        if self._h:
            lib().dk_json_tail_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------------------------------------
# Log segment (SnapshotManager / Checkpointer / LogSegment)
# ------------------------------------------------------------------------------------------------
_DELTA = re.compile(r"^(\d{20})\.json$")
_CLASSIC = re.compile(r"^(\d{20})\.checkpoint\.parquet$")
_MULTI = re.compile(r"^(\d{20})\.checkpoint\.(\d{10})\.(\d{10})\.parquet$")
_V2 = re.compile(r"^(\d{20})\.checkpoint\.([^.]+)\.(json|parquet)$")


@dataclass
class LogFile:
    path: str
    kind: str
    version: int
    part: int = 0
    num_parts: int = 0


@dataclass
class LogSegment:
    log_path: str
    version: int
    deltas: list
    checkpoints: list

    def all_files_reversed(self):
        return sorted(self.deltas + self.checkpoints, key=lambda f: os.path.basename(f.path), reverse=True)


def _classify(log, name):
    full = os.path.join(log, name)
    for rx, kind in ((_DELTA, "commit"), (_CLASSIC, "classic"), (_MULTI, "multipart"), (_V2, "v2")):
        m = rx.match(name)
        if m:
            if kind == "multipart":
                return LogFile(full, kind, int(m.group(1)), int(m.group(2)), int(m.group(3)))
            return LogFile(full, kind, int(m.group(1)))
    return None


def build_log_segment(table_root: str) -> LogSegment:
    log = os.path.join(table_root, "_delta_log")
    if not os.path.isdir(log):
        raise DkError("Table at path `%s` is not found" % table_root)
    start = -1
    lc = os.path.join(log, "_last_checkpoint")
    if os.path.exists(lc):
        try:
            with open(lc) as f:
                start = int(json.loads(f.readline())["version"])
        except Exception:
            start = -1          # corrupt hint: list everything (Checkpointer.readLastCheckpointFile)
    files = [f for f in (_classify(log, n) for n in os.listdir(log)) if f and f.version >= max(start, 0)]
    if not files and start >= 0:
        files = [f for f in (_classify(log, n) for n in os.listdir(log)) if f]
    groups = {}
    for f in files:
        if f.kind != "commit":
            groups.setdefault((f.version, f.kind, f.num_parts), []).append(f)
    complete = []
    for (v, kind, nparts), fs in groups.items():
        if kind == "multipart":
            if sorted(x.part for x in fs) == list(range(1, nparts + 1)):
                complete.append((v, kind, sorted(fs, key=lambda x: x.part)))
        else:
            complete.append((v, kind, fs[:1]))
    deltas = sorted([f for f in files if f.kind == "commit"], key=lambda f: f.version)
    if not deltas and not complete:
        raise DkError("No delta files found in the directory: " + log)
    rank = {"classic": 0, "multipart": 1, "v2": 2}
    ck = max(complete, key=lambda c: (c[0], rank[c[1]], len(c[2])), default=None)
    ckv = ck[0] if ck else -1
    tail = [d for d in deltas if d.version > ckv]
    for i, d in enumerate(tail):
        if d.version != ckv + 1 + i:
            raise DkError("Versions are not contiguous")
    if ck is None and (not tail or tail[0].version != 0):
        raise DkError("Cannot compute snapshot. Missing delta file version 0.")
    return LogSegment(log, tail[-1].version if tail else ckv, tail, list(ck[2]) if ck else [])


# ------------------------------------------------------------------------------------------------
# tableRoot
# ------------------------------------------------------------------------------------------------
# ASCII characters java.net.URI's multi-argument constructors leave unquoted in a path component
# (unreserved, punct, "/", "@"); '%' is always quoted.
_PATH_CHARS = frozenset("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_-!.~'()*,;:$&+=/@")


def table_root_uri(path: str) -> str:
    """The tableRoot string of a scan file for a local table.

    Table.forPath resolves the path with DefaultFileSystemClient.resolvePath
    (kernel-defaults/.../engine/DefaultFileSystemClient.java:82-86: the Hadoop Path qualified
    against the local file system, i.e. "file:" + the absolute path with "//" collapsed and the
    trailing "/" dropped, kernel-api/.../internal/fs/Path.java normalizePath); TableImpl keeps it as
    a Path (TableImpl.java:81-85) and ActiveAddFilesIterator emits dataPath.toUri().toString()
    (ActiveAddFilesIterator.java:251). Path builds its URI with the multi-argument java.net.URI
    constructor, which percent-encodes (UTF-8, upper-case hex) every ASCII character that is not
    legal in a path, '%' included, and every non-ASCII space or ISO control character."""
    import unicodedata
    p = os.path.abspath(path)
    out = []
    for ch in p:
        o = ord(ch)
        if o < 0x80:
            out.append(ch if ch in _PATH_CHARS else "%%%02X" % o)
        elif unicodedata.category(ch) in ("Zs", "Zl", "Zp") or o <= 0x9F:
            out.append("".join("%%%02X" % b for b in ch.encode("utf-8", "surrogatepass")))
        else:
            out.append(ch)
    return "file:" + "".join(out)


# ------------------------------------------------------------------------------------------------
# Checksum (.crc) files (ChecksumReader / CRCInfo)
# ------------------------------------------------------------------------------------------------
_CRC = re.compile(r"^(\d+)\.crc$")


def _read_checksum_file(path):
    """ChecksumReader.readChecksumFile (replay/ChecksumReader.java:98-127): exactly one JSON row
    with non-null protocol and metadata (CRCInfo.FULL_SCHEMA: "protocol", "metadata"), decoded with
    the P&M rules; anything else -- missing, empty, several rows, undecodable -- is no CRC."""
    from . import actions as A
    try:
        with open(path, "rb") as f:
            lines = f.read().decode("utf-8", "replace").splitlines()
        if len(lines) != 1:
            return None
        obj = json.loads(lines[0])
        p, m = obj.get("protocol"), obj.get("metadata")
        if p is None or m is None:
            return None
        return (int(os.path.basename(path).split(".")[0]), A.protocol_from_json(p), A.metadata_from_json(m))
    except Exception:
        return None


def read_crc_info(log_path, version, lower):
    """ChecksumReader.getCRCInfo (ChecksumReader.java:40-96): the checksum file at `version`, else the
    newest one in [lower, version] (listing from <lower>.crc)."""
    lower = min(lower, version)
    got = _read_checksum_file(os.path.join(log_path, "%020d.crc" % version))
    if got is not None or version == 0 or version == lower:
        return got
    start = "%020d.crc" % lower
    try:
        names = sorted(n for n in os.listdir(log_path) if n >= start)
    except OSError:
        return None
    crcs = []
    for n in names:
        m = _CRC.match(n)
        if not m:
            continue
        if int(m.group(1)) > version:
            break                                       # takeWhile(version <= target)
        crcs.append(n)
    return _read_checksum_file(os.path.join(log_path, crcs[-1])) if crcs else None


# ------------------------------------------------------------------------------------------------
# Table / Snapshot / Scan
# ------------------------------------------------------------------------------------------------
class Table:
    def __init__(self, path):
        self.path = os.path.abspath(path)

    @staticmethod
    def forPath(engine, path):
        return Table(path)

    def checkpoint(self, engine, version=None, now_ms=None):
        """Table.checkpoint (TableImpl.java:132-140 -> SnapshotManager.checkpoint): writes the classic
        checkpoint of the latest version and _last_checkpoint (delta_amd/checkpoint.py). Returns
        (version, number of add actions written)."""
        from .checkpoint import write_checkpoint
        latest = build_log_segment(self.path).version
        if version is not None and version != latest:
            raise DkError("checkpoint: this engine writes checkpoints of the latest version (%d), not %d"
                          % (latest, version))
        return write_checkpoint(engine, self.path, now_ms)

    def getLatestSnapshot(self, engine):
        t0 = time.perf_counter()
        seg = build_log_segment(self.path)
        snap = Snapshot(self, seg)
        snap.load_ms["log_segment"] = (time.perf_counter() - t0) * 1e3
        snap._json_batch_size = engine.json_batch_size
        snap._parquet_batch_size = engine.cfg.parquet_batch_size
        snap._load_protocol_metadata(engine)
        return snap


@dataclass
class ScanMetrics:
    addFilesSeen: int = 0
    addFilesSeenFromDeltaFiles: int = 0
    activeAddFiles: int = 0
    duplicateAddFiles: int = 0
    removeFilesSeenFromDeltaFiles: int = 0

    def as_tuple(self):
        return (self.addFilesSeen, self.addFilesSeenFromDeltaFiles, self.activeAddFiles,
                self.duplicateAddFiles, self.removeFilesSeenFromDeltaFiles)


class Snapshot:
    def __init__(self, table, seg):
        self.table = table
        self.log_segment = seg
        self.protocol = None
        self.metadata = None
        self.load_ms = {}   # snapshot-load phases (ms): log_segment, crc, commits_pm, checkpoint_pm
        self.crc_info = None
        self._validated = False   # TableFeatures.validateReadSupportedTable ran in the P&M pass
        self._manifest = None

    def getVersion(self):
        return self.log_segment.version

    def getScanBuilder(self):
        return ScanBuilder(self)

    def _json_manifest(self):
        """Actions of a V2 checkpoint's JSON manifest (ActionsIterator reads it with the JSON handler,
        ActionsIterator.java:306-315, and extracts its sidecar rows, :256-283). Host-parsed: one
        small file. Returns (sidecar paths in manifest order, protocol, metaData). Its add rows
        are checkpoint rows too: GpuScan parses the manifest after the commit tail
        (dk_json_tail_parse_parts) and reconciles them as checkpoint adds."""
        if self._manifest is None:
            side, proto, meta = [], None, None
            with open(self.log_segment.checkpoints[0].path, "rb") as f:
                for line in f.read().decode("utf-8", "replace").splitlines():
                    if not line.strip():
                        continue
                    obj = json.loads(line)
                    sc = obj.get("sidecar")
                    if sc is not None:
                        side.append(os.path.join(self.log_segment.log_path, "_sidecars", sc["path"]))
                    if proto is None and obj.get("protocol") is not None:
                        proto = obj["protocol"]
                    if meta is None and obj.get("metaData") is not None:
                        meta = obj["metaData"]
            self._manifest = (side, proto, meta)
        return self._manifest

    def _json_checkpoint_parts(self):
        """The checkpoint parts read with the JSON handler: a V2 checkpoint's JSON manifest."""
        cks = self.log_segment.checkpoints
        return [cks[0].path] if cks and cks[0].kind == "v2" and cks[0].path.endswith(".json") else []

    def _checkpoint_files(self, engine, with_pruning=False):
        """Checkpoint data files in replay order: multi-part parts descending (LogSegment
        ordering); V2 parquet manifest first, then its sidecars in manifest order; a V2 JSON
        manifest contributes only its sidecars. with_pruning: also whether the checkpoint predicate
        can prune each file's row groups -- multi-part parts and sidecars get it as is; a classic
        or V2 top-level file gets OR(predicate, sidecar IS NOT NULL), which never converts to a
        parquet-mr filter (ActionsIterator.java:175-226, 336-351)."""
        files = self._checkpoint_file_list(engine)
        if not with_pruning:
            return files
        cks = self.log_segment.checkpoints
        if not cks:
            return files, []
        if cks[0].kind == "v2":
            top = 0 if cks[0].path.endswith(".json") else 1
            return files, [i >= top for i in range(len(files))]
        return files, [cks[0].kind == "multipart"] * len(files)

    def _checkpoint_file_list(self, engine):
        cks = self.log_segment.checkpoints
        if not cks:
            return []
        if cks[0].kind == "v2":
            man = cks[0].path
            if man.endswith(".json"):
                return list(self._json_manifest()[0])
            ps = ParquetSet(engine, [man], SIDECAR_LEAVES).decode()
            sp = ps.column(0, "sidecar.path")
            side = []
            if sp.present:
                for r in range(sp.n_rows):
                    if sp.row_def[r] >= sp.max_def:
                        side.append(os.path.join(self.log_segment.log_path, "_sidecars", sp.string(r).decode()))
            ps.close()
            return [man] + side
        return [f.path for f in sorted(cks, key=lambda f: os.path.basename(f.path), reverse=True)]

    def _load_protocol_metadata(self, engine):
        """LogReplay's snapshot-load pass (internal/replay/LogReplay.java:130-150, 220-314, 384-426).

        1. maybeGetNewerSnapshotHintAndCurrentCrcInfo: a fresh Table has no snapshot hint, so the
           newest checksum file in [max(checkpoint version, version - 100, 0), version] becomes the
           hint (ChecksumReader.getCRCInfo, replay/ChecksumReader.java:40-96). A hint at the
           snapshot version ends the pass with its Protocol and Metadata (nothing else is read and,
           as in the reference, nothing is validated).
        2. Otherwise files newest first: commits (scanned on host threads, dk_log_pm_scan), then the
           checkpoint (decoded on the GPU). Per batch the protocol is looked for first, then the
           metadata; the table is validated (TableFeatures.validateReadSupportedTable) only when the
           metadata turns up while the protocol is already known (:270-283). After the commit at
           hint version + 1 the hint fills whatever is still missing (:292-302)."""
        from . import actions as A
        seg = self.log_segment
        v = seg.version
        t0 = time.perf_counter()
        ck_v = seg.checkpoints[0].version if seg.checkpoints else 0
        crc = read_crc_info(seg.log_path, v, max(ck_v, v - 100, 0))
        self.load_ms["crc"] = (time.perf_counter() - t0) * 1e3
        self.crc_info = crc
        if crc is not None and crc[0] == v:
            self.protocol, self.metadata = crc[1], crc[2]
            return
        self._validated = False
        t0 = time.perf_counter()
        try:
            done = self._pm_from_commits(hint=crc)
        finally:
            self.load_ms["commits_pm"] = (time.perf_counter() - t0) * 1e3
        if not done and (self.protocol is None or self.metadata is None):
            t0 = time.perf_counter()
            try:
                self._pm_from_checkpoint(engine)
            finally:
                self.load_ms["checkpoint_pm"] = (time.perf_counter() - t0) * 1e3
        if self.protocol is None:
            raise DkError("No protocol found at version %d" % self.getVersion())
        if self.metadata is None:
            raise DkError("No metadata found at version %d" % self.getVersion())

    def _found(self, protocol=None, metadata=None):
        """One batch's finds, in the reference's order: protocol first, then metadata; validate when
        the metadata arrives with the protocol already known. Returns True once both are known."""
        from . import actions as A
        if self.protocol is None and protocol is not None:
            self.protocol = protocol
            if self.metadata is not None:
                return True
        if self.metadata is None and metadata is not None:
            self.metadata = metadata
            if self.protocol is not None:
                # dataPath.toString(): the qualified path, unescaped (internal/fs/Path.java:328-350)
                A.validate_read_supported(self.protocol, "file:" + self.table.path, self.metadata)
                self._validated = True
                return True
        return False

    def _pm_from_commits(self, hint=None):
        """Commit files newest first; returns True when the pass is complete (both found, or the
        hint filled the rest)."""
        from . import actions as A
        deltas = list(reversed(self.log_segment.deltas))
        if hint is not None:                 # only commits newer than the hint are read
            deltas = [d for d in deltas if d.version > hint[0]]
        n = len(deltas)
        if n:
            arr = lambda t: (t * n)()
            pl, po, pn, ml, mo, mn = (arr(C.c_int64) for _ in range(6))
            scanned = C.c_int32()
            check(lib().dk_log_pm_scan(_cstrs([d.path for d in deltas]), n, pl, po, pn, ml, mo, mn, C.byref(scanned)))
            J = self._json_batch_size
            for i in range(scanned.value):
                def action(off, ln, key):
                    # decoded in libdkgpu with DefaultJsonRow's rules (dk_json_pm_decode), handed
                    # back re-serialised with exactly the schema's fields
                    path = deltas[i].path.encode()
                    which = 0 if key == "protocol" else 1
                    n = C.c_int64()
                    buf = C.create_string_buffer(2 * int(ln) + 256)
                    rc = lib().dk_json_pm_decode(path, off, ln, which, buf, len(buf), C.byref(n))
                    if rc == 2:
                        buf = C.create_string_buffer(int(n.value) + 16)
                        rc = lib().dk_json_pm_decode(path, off, ln, which, buf, len(buf), C.byref(n))
                    check(rc)
                    return json.loads(buf.raw[:n.value].decode("utf-8"))
                # batches of J lines per commit file (DefaultJsonHandler): in line order
                events = sorted([(pl[i] // J, 0, "p")] * (pl[i] >= 0) + [(ml[i] // J, 1, "m")] * (ml[i] >= 0))
                b = 0
                while b < len(events):
                    batch = [e for e in events if e[0] == events[b][0]]
                    prot = meta = None
                    for _, _, k in batch:
                        if k == "p" and self.protocol is None:
                            prot = A.protocol_from_json(action(po[i], pn[i], "protocol"))
                        if k == "m" and self.metadata is None:
                            meta = A.metadata_from_json(action(mo[i], mn[i], "metaData"))
                    if self._found(prot, meta):
                        return True
                    b += len(batch)
                if hint is not None and deltas[i].version == hint[0] + 1:
                    return self._from_hint(hint)
        if hint is not None:
            return self._from_hint(hint)
        return False

    def _from_hint(self, hint):
        if self.protocol is None:
            self.protocol = hint[1]
        if self.metadata is None:
            self.metadata = hint[2]
        return True

    def _pm_from_checkpoint(self, engine):
        from . import actions as A
        cks = self.log_segment.checkpoints
        if cks and cks[0].kind == "v2" and cks[0].path.endswith(".json"):
            _, proto, meta = self._json_manifest()
            if self._found(A.protocol_from_json(proto) if self.protocol is None and proto is not None else None,
                           A.metadata_from_json(meta) if self.metadata is None and meta is not None else None):
                return
            files = self._checkpoint_files(engine) if (self.protocol is None or self.metadata is None) else []
        else:
            files = self._checkpoint_files(engine) if cks else []
        if files and (self.protocol is None or self.metadata is None):
            # only row groups whose footer statistics allow a non-null protocol / metaData row
            # (an all-null row group cannot hold the first one); files with none are not read
            t_a = time.perf_counter()
            want = [lf for lf, need in (("protocol.minReaderVersion", self.protocol is None),
                                        ("metaData.id", self.metadata is None)) if need]
            groups = []
            for f in files:
                keep = None
                for lf in want:
                    k = nonnull_row_groups(f, lf)
                    keep = k if keep is None else [a or b for a, b in zip(keep, k)]
                groups.append([g for g, k in enumerate(keep) if k])
            files = [f for f, g in zip(files, groups) if g]
            groups = [g for g in groups if g]
            if not files:
                return
            t_b = time.perf_counter()
            ps = ParquetSet(engine, files, PM_LEAVES, groups=groups).decode()
            t_c = time.perf_counter()
            B = self._parquet_batch_size
            for fi in range(len(files)):
                # the first non-null protocol / metaData row of the file, found on the device; only
                # that row's values come back to the host; batches of B rows in row order (counted
                # over the row groups decoded here).
                rp = ps.first_row(fi, "protocol.minReaderVersion") if self.protocol is None else -1
                rm = ps.first_row(fi, "metaData.id") if self.metadata is None else -1
                prot = _protocol_row(ps, fi, rp) if rp >= 0 else None
                meta = _metadata_row(ps, fi, rm) if rm >= 0 else None
                if prot is not None and meta is not None and rp // B != rm // B:
                    first, second = ((prot, None), (None, meta)) if rp < rm else ((None, meta), (prot, None))
                    done = self._found(*first) or self._found(*second)
                else:
                    done = self._found(prot, meta)
                if done:
                    break
            t_d = time.perf_counter()
            ps.close()
            # (where a cold load goes: footers, the open + device decode, the rows found and decoded)
            self.load_ms.update(checkpoint_pm_footers=(t_b - t_a) * 1e3, checkpoint_pm_decode=(t_c - t_b) * 1e3,
                                checkpoint_pm_rows=(t_d - t_c) * 1e3)


def _row(ps, fi, leaf, r):
    c = ps.column_rows(fi, leaf, r, 1)
    return c if c.present else None


def _str_row(ps, fi, leaf, r):
    c = _row(ps, fi, leaf, r)
    return None if c is None or c.row_def[0] < c.max_def else c.string(0).decode("utf-8", "replace")


def _int_row(ps, fi, leaf, r, dtype):
    c = _row(ps, fi, leaf, r)
    return None if c is None or c.row_def[0] < c.max_def else int(c.fixed.view(dtype)[0])


def _list_row(ps, fi, leaf, r):
    c = _row(ps, fi, leaf, r)
    return _list_at(c, 0)


def _map_row(ps, fi, kleaf, vleaf, r):
    kc, vc = _row(ps, fi, kleaf, r), _row(ps, fi, vleaf, r)
    if kc is None or kc.row_def[0] < kc.rep_def - 1:
        return None
    a, b = int(kc.row_offs[0]), int(kc.row_offs[1])
    out = {}
    for i in range(a, b):
        v = None if vc is None or vc.entry_def[i] < vc.max_def else vc.string(i).decode("utf-8", "replace")
        out[kc.string(i).decode("utf-8", "replace")] = v
    return out


def _protocol_row(ps, fi, r):
    """Protocol.fromColumnVector (actions/Protocol.java:33-47) on checkpoint row r."""
    from .actions import KernelException
    rv = _int_row(ps, fi, "protocol.minReaderVersion", r, np.int32)
    wv = _int_row(ps, fi, "protocol.minWriterVersion", r, np.int32)
    if rv is None or wv is None:
        raise KernelException("protocol action with a null minReaderVersion / minWriterVersion")
    return {"minReaderVersion": rv, "minWriterVersion": wv,
            "readerFeatures": _list_row(ps, fi, "protocol.readerFeatures.list.element", r) or [],
            "writerFeatures": _list_row(ps, fi, "protocol.writerFeatures.list.element", r) or []}


def _metadata_row(ps, fi, r):
    """Metadata.fromColumnVector (actions/Metadata.java:35-55) on checkpoint row r."""
    from .actions import KernelException
    md = {"id": _str_row(ps, fi, "metaData.id", r),
          "name": _str_row(ps, fi, "metaData.name", r),
          "description": _str_row(ps, fi, "metaData.description", r),
          "format": {"provider": _str_row(ps, fi, "metaData.format.provider", r),
                     "options": _map_row(ps, fi, "metaData.format.options.key_value.key",
                                         "metaData.format.options.key_value.value", r) or {}},
          "schemaString": _str_row(ps, fi, "metaData.schemaString", r),
          "partitionColumns": _list_row(ps, fi, "metaData.partitionColumns.list.element", r),
          "createdTime": _int_row(ps, fi, "metaData.createdTime", r, np.int64),
          "configuration": _map_row(ps, fi, "metaData.configuration.key_value.key",
                                    "metaData.configuration.key_value.value", r)}
    for key in ("id", "schemaString", "partitionColumns", "configuration"):
        if md[key] is None:
            raise KernelException("Field `%s` in `metaData` is not nullable, but it is null" % key)
    return md


def _list_at(col, r):
    """list<string> value of row r of a decoded list leaf (None when the list is null)."""
    if col is None or not col.present or col.row_def[r] < col.rep_def - 1:
        return None
    a, b = int(col.row_offs[r]), int(col.row_offs[r + 1])
    return [col.string(i).decode() if col.entry_def[i] >= col.max_def else None for i in range(a, b)]


class ScanBuilder:
    def __init__(self, snapshot):
        self.snapshot = snapshot
        self.read_stats = False
        self.shard = None
        self.predicate = None

    def withFilter(self, predicate):
        """ScanBuilderImpl.withFilter (internal/ScanBuilderImpl.java:61-67). The partition part of the
        filter becomes a GPU partition-pruning program (delta_amd/partitions.py), the data part a GPU
        data-skipping program (K11, delta_amd/skipping.py)."""
        if self.predicate is not None:
            raise ValueError("There already exists a filter in current builder")
        self.predicate = predicate
        return self

    def withStats(self, flag=True):
        self.read_stats = flag
        return self

    def withReadSchema(self, schema_json):
        """ScanBuilderImpl.withReadSchema (ScanBuilderImpl.java:70-74): the logical schema the scan
        state reports (Kernel StructType JSON); the scan files are the same."""
        self.read_schema = schema_json
        return self

    def withShard(self, world, rank, exchange=None, owner=None):
        """Reconcile only this rank's checkpoint row groups (delta_amd/shard.py). exchange: None (the
        probe runs against this rank's own copy of the commit-tail key table), or a callable that
        drives the hash(path)-owner exchange for this rank (shard.exchange_hash_owner over
        torch.distributed, or an in-process loopback), called with the scan's ExchangeSide after
        every run. owner: the owner-partitioned reconciliation over a library communicator
        (shard.OwnerComm: RCCL, callbacks or in-process ranks): this rank parses only its share of
        the commit files, and the key table of the keys it owns answers every rank's rows for them;
        the whole protocol runs in dk_replay_owner_run."""
        self.shard = (int(world), int(rank))
        self.exchange = exchange
        self.owner = owner
        if exchange is not None and owner is not None:
            raise ValueError("withShard: one exchange mode at a time")
        return self

    def build(self):
        sc = GpuScan(self.snapshot, self.read_stats, self.shard, self.predicate)
        sc.read_schema = getattr(self, "read_schema", None)
        sc.exchange = getattr(self, "exchange", None)
        # owner mode: an explicit owner communicator (also at world 1: one RCCL rank through the ABI)
        sc.owner = getattr(self, "owner", None) if self.shard else None
        return sc


def _own_column(c):
    """A Column whose arrays are its own (copies of a zero-copy view's)."""
    import copy
    o = copy.copy(c)
    for a in ("row_def", "row_offs", "entry_def", "fixed", "offs", "chars"):
        v = getattr(c, a, None)
        if isinstance(v, np.ndarray):
            setattr(o, a, v.copy())
    return o


class LazyColumns(dict):
    """leaf -> Column of one batch, copied from HBM on first access (the batch's vectors are
    device-resident with a host mirror on demand); a leaf the file lacks reads as
    None (all-null, NonExistentColumnReader)."""

    def __init__(self, leaves, fetch):
        super().__init__()
        self._leaves = list(leaves)
        self._fetch = fetch

    def __missing__(self, leaf):
        if leaf not in self._leaves:
            raise KeyError(leaf)
        c = self._fetch(leaf)
        c = c if c.present else None
        self[leaf] = c
        return c

    def get(self, leaf, default=None):
        return self[leaf] if leaf in self._leaves else default

    def __contains__(self, leaf):
        return leaf in self._leaves

    def keys(self):
        return list(self._leaves)

    def __iter__(self):
        return iter(self._leaves)

    def __len__(self):
        return len(self._leaves)

    def items(self):
        return [(k, self[k]) for k in self._leaves]

    def values(self):
        return [self[k] for k in self._leaves]


@dataclass
class FilteredColumnarBatch:
    """data: leaf -> Column (add.* leaves) plus the constant tableRoot; selection: bool per row or
    None when every row is selected (KA/data/FilteredColumnarBatch.java:37-111)."""
    data: dict
    table_root: str
    size: int
    selection: np.ndarray | None
    source: str = ""
    file_index: int = -1          # replay-order checkpoint file index; -1 = commit tail
    row_offset: int = 0           # file row of this batch's first row (row-group shards)
    commit_index: int = -1        # owner mode: the commit file's replay-order index (tail batches)

    def selected_rows(self):
        if self.selection is None:
            return np.arange(self.size)
        return np.nonzero(self.selection)[0]


class GpuScan:
    """Scan whose getScanFiles runs decode + reconciliation in libdkgpu (SURVEY.md §8(b) plugin
    point 2)."""

    # leaves mirrored to host memory per decoded group (dk_replay_prefetch_leaf)
    PREFETCH_LEAVES = ("add.size",)

    def __init__(self, snapshot, read_stats=False, shard=None, predicate=None):
        self.snapshot = snapshot
        self.shard = shard
        self.predicate = predicate
        self.skipping = None          # (planner node, compiled Program) when a data-skipping filter applies
        self._deferred_error = None
        self.partition = None
        self.partition_filter, self.data_filter = None, None
        if predicate is not None:
            from . import skipping as sk
            md = snapshot.metadata or {}
            parts = md.get("partitionColumns") or []
            self.partition_filter, self.data_filter = sk.split_filters(predicate, parts)
            self.partition = None     # compiled partition-pruning program (dk_part_compile)
            if self.partition_filter is not None:
                from . import partitions as pp
                from . import programs
                try:
                    self.partition = programs.compile_partition(
                        self.partition_filter, pp.partition_fields(md["schemaString"], parts))
                except (sk.UnsupportedExpression, pp.UnsupportedPartitionFilter) as e:
                    # the reference fails when the scan files are read, never at build(); a filter
                    # this engine cannot compile fails there too, loudly
                    self._deferred_error = e
            if self.data_filter is not None:
                leaves = sk.data_schema_leaves(md["schemaString"], parts)
                node = sk.construct(self.data_filter, leaves)
                if node is not None:
                    try:
                        sk.check_types(node, leaves)
                    except sk.UnsupportedExpression as e:
                        self._deferred_error = e      # the reference fails when the scan files are read
                    else:
                        from . import programs
                        try:
                            self.skipping = (node, programs.compile_skipping(node, leaves))
                        except sk.UnsupportedExpression as e:
                            self._deferred_error = e  # (the compiler's own type check)
        # ScanImpl.getScanFiles: shouldReadStats = hasDataSkippingFilter || includeStats (:128-130)
        self.read_stats = read_stats or self.skipping is not None
        self.metrics = ScanMetrics()
        self.tail_metrics = ScanMetrics()
        self.ckpt_metrics = ScanMetrics()
        self.replay = None
        self.prepare_ms = {}
        self._handed = weakref.WeakValueDictionary()   # zero-copy checkpoint batches handed out (_detach_batches)

    def table_root(self):
        """tableRoot = dataPath.toUri().toString() (ActiveAddFilesIterator.java:251)."""
        return table_root_uri(self.snapshot.table.path)

    def getScanState(self, engine):
        """Scan.getScanState (ScanImpl.java:189-218, ScanStateRow.java:35-44) as a dict: the table's
        configuration, the logical read schema, its physical equivalent under the column mapping
        mode, the physical data read schema (no partition columns; `_metadata.row_index` when
        deletionVectors is a reader feature), partition columns, protocol versions and tablePath;
        schemas as the reference's JSON text (delta_amd/schema.py)."""
        from . import schema
        return schema.scan_state(self.snapshot.metadata or {}, self.snapshot.protocol or {}, self.table_root(),
                                 read_schema=getattr(self, "read_schema", None))

    def prepare(self, engine):
        """Host-side setup: parse the commit tail, open checkpoint files, upload to HBM."""
        if self._deferred_error is not None:
            raise self._deferred_error
        t0 = time.perf_counter()
        seg = self.snapshot.log_segment
        commits = list(reversed(seg.deltas))
        # the commit tail is parsed (host threads, GIL released in the library) while the checkpoint
        # files are opened below; its errors still surface first, as in the reference's replay order
        import threading
        tail_box = {}

        owner = getattr(self, "owner", None)
        parts = self.snapshot._json_checkpoint_parts()
        if owner is not None:
            # owner mode: this rank parses the commit files j = rank (mod world) of the replay order
            # (newest first) and, on rank 0, the JSON manifest; their batch steps are renumbered in
            # the global replay order once the ranks' batch counts are known (owner.global_steps)
            world, rank = self.shard
            self.tail_commits = [j for j in range(len(commits)) if j % world == rank]
            self.tail_parts = list(range(len(commits), len(commits) + len(parts))) if rank == 0 else []
            mine = [commits[j] for j in self.tail_commits]
            parts = parts if rank == 0 else []
        else:
            mine = commits

        n_files_all = len(commits) + len(self.snapshot._json_checkpoint_parts())

        def parse_tail():
            # the tail, then the replay's commit-tail half (action table + key-table inputs)
            t = time.perf_counter()
            try:
                try:
                    tail = JsonTail(engine, [d.path for d in mine], [d.version for d in mine], self.read_stats,
                                    checkpoint_paths=parts)
                except BaseException:
                    if owner is not None:   # the peers wait in global_steps: they raise with this rank
                        tail_box["voted"] = "failed"
                        owner.global_steps(np.zeros(n_files_all, np.int64), failed=True)
                    raise
                tail_box["tail"] = tail
                if owner is not None:
                    files = self.tail_commits + self.tail_parts
                    steps = (C.c_int32 * max(1, len(files)))()
                    check(lib().dk_json_tail_file_steps(tail._h, steps))
                    local = np.zeros(n_files_all, np.int64)
                    for k, j in enumerate(files):
                        local[j] = steps[k]
                    tail_box["voted"] = "failed"        # (until the vote has gone through)
                    total = np.asarray(owner.global_steps(local), dtype=np.int64)
                    tail_box["voted"] = "ok"
                    step0 = np.concatenate([[0], np.cumsum(total)])
                    if step0[-1] >= (1 << 31) - 1:
                        raise DkError("owner mode: more than 2^31 commit-tail batches")
                    base = (C.c_int32 * max(1, len(files)))(*[int(step0[j]) for j in files])
                    check(lib().dk_json_tail_rebase_steps(tail._h, base))
                    row0 = (C.c_int64 * (len(files) + 1))()
                    check(lib().dk_json_tail_file_row0(tail._h, row0))
                    self.tail_file_rows = [(files[k], int(row0[k]), int(row0[k + 1])) for k in range(len(files))]
                tail_box["ms"] = (time.perf_counter() - t) * 1e3
                t = time.perf_counter()
                rh = C.c_void_p()
                check(lib().dk_replay_create(engine._h, tail._h, None, C.byref(rh)))
                tail_box["rh"] = rh
                tail_box["create_ms"] = (time.perf_counter() - t) * 1e3
            except BaseException as e:          # re-raised on the calling thread
                tail_box["error"] = e

        def owner_failed():
            """This rank is about to raise from prepare: make sure its peers raise too instead of
            waiting for it in a collective (global_steps, or the exchange's first vote)."""
            if owner is None or tail_box.get("voted") == "failed":
                return                      # (a failed vote: every rank raised at global_steps)
            if not tail_box.get("voted"):
                owner.global_steps(np.zeros(n_files_all, np.int64), failed=True)
            else:
                owner.abort()               # global_steps went through: the exchange's first vote

        tail_thread = threading.Thread(target=parse_tail, daemon=True)
        started = []

        def start_tail():
            if not started:
                started.append(1)
                tail_thread.start()
        try:
            self._prepare_checkpoint(engine, t0, start_tail)
            start_tail()
        except BaseException as e:
            if started:                             # the tail's errors come first in replay order
                tail_thread.join()
                self.tail = tail_box.get("tail")    # freed by close()
                self._rh = tail_box.get("rh")
            try:
                owner_failed()
            finally:
                if "error" in tail_box:
                    raise tail_box["error"]
                raise e
        tail_thread.join()
        if "tail" in tail_box:
            self.tail = tail_box["tail"]
        if "rh" in tail_box:
            self._rh = tail_box["rh"]
        if "error" in tail_box:
            owner_failed()
            raise tail_box["error"]
        self.prepare_ms["commit_tail"] = tail_box["ms"]
        self.prepare_ms["replay_create_tail"] = tail_box["create_ms"]
        try:
            t3 = time.perf_counter()
            if self.ckpt is not None:
                check(lib().dk_replay_attach_checkpoint(self._rh, self.ckpt._h))
            self.prepare_ms["replay_attach"] = (time.perf_counter() - t3) * 1e3
            if getattr(self, "exchange", None) is not None and self.shard and self.shard[0] > 1:
                check(lib().dk_replay_set_exchange(self._rh, self.shard[0], self.shard[1]))
            if getattr(self, "owner", None) is not None:
                check(lib().dk_replay_set_owner(self._rh, self.shard[0], self.shard[1]))
            if self.partition is not None:
                check(lib().dk_replay_set_partition_filter(self._rh, self.partition.handle))
            if self.skipping is not None:
                check(lib().dk_replay_set_skipping(self._rh, self.skipping[1].handle))
        except BaseException:
            owner_failed()
            raise
        return self

    def _prepare_checkpoint(self, engine, t1, start_tail=lambda: None):
        """Plan the checkpoint files (row-group pruning, shards) and open them (host read + H2D +
        the device sizing passes). start_tail() starts the commit tail's parse beside the open: before
        a synchronous open, after an asynchronous one has returned (it returns once the footers and
        page headers are read; those and the tail's parse are CPU-bound on the same cores, and the
        open's first H2D copies are on the critical path: 173 -> 166 ms at C3, profiles/r04/tail_after_open;
        DK_TAIL_AFTER_OPEN=0 starts it first in both cases)."""
        self.prepare_ms = {}
        all_files, prunable = self.snapshot._checkpoint_files(engine, with_pruning=True)
        # row groups read per file: all, minus those the checkpoint predicate (the partition filter
        # on add.partitionValues_parsed) proves empty in multi-part parts and sidecars
        groups = [None] * len(all_files)
        if self.partition_filter is not None and any(prunable):
            from . import partitions as pp
            md = self.snapshot.metadata or {}
            prog = pp.row_group_filter(self.partition_filter,
                                       pp.partition_fields(md["schemaString"], md.get("partitionColumns") or []))
            packed = pp.pack_row_group_filter(prog, dk_rg_filter)
            for i, f in enumerate(all_files):
                if prunable[i]:
                    groups[i] = prune_row_groups(f, packed)
        if self.shard or any(g is not None for g in groups):
            # shards: this rank's contiguous run of the surviving row groups (delta_amd/shard.py)
            rows = [row_group_rows(f) for f in all_files]
            groups = [list(range(len(r))) if g is None else g for g, r in zip(groups, rows)]
            if self.shard:
                from .shard import plan_units
                units = plan_units([[rows[fi][g] for g in gs] for fi, gs in enumerate(groups)], *self.shard)
                self.ckpt_index = [f for f, _, _ in units]
                sel = [groups[f][a:b] for f, a, b in units]
            else:                                   # a fully pruned file yields no batch at all
                self.ckpt_index = [i for i, g in enumerate(groups) if g]
                sel = [groups[i] for i in self.ckpt_index]
        else:
            self.ckpt_index = list(range(len(all_files)))
            sel = None
        self.ckpt_files = [all_files[i] for i in self.ckpt_index]
        # the checkpoint's remove columns are not read: ActiveAddFilesIterator ignores every remove of a
        # checkpoint batch (ActiveAddFilesIterator.java:158-183, `if (!isFromCheckpoint)`) and only its
        # add rows reach the scan files, so the fused engine pushes that into the projection (the
        # commit tail's removes are parsed by the JSON tail parser)
        leaves = ADD_LEAVES + ([STATS_LEAF] if self.read_stats else [])
        if self.skipping is not None:
            # the typed add.stats_parsed leaves of the program's stats paths: the engine evaluates
            # skipping over them where a checkpoint file carries them with a type that holds the stat
            # (dk_replay_set_skipping), the add.stats JSON standing in for the rows they cannot
            leaves = leaves + ["add.stats_parsed." + ".".join(p) for p in self.skipping[1].paths]
        t2 = time.perf_counter()
        # a plain scan (no shard, skipping or partition filter) opens the checkpoint asynchronously: the
        # grouped getScanFiles hands out the first files' batches while the later files still land
        # (DK_ASYNC_OPEN=0: the synchronous open)
        # (data skipping, partition pruning and row-group predicates too: C4 308-310 ms against 321-327
        # synchronous, profiles/r04/c4_async_ab; DK_ASYNC_FILTERED=0 keeps them synchronous)
        # sharded scans (a rank's row-group runs) open asynchronously too: in owner mode the commit
        # tail's exchange overlaps the open, and the row exchanges wait for the decode (dk_replay_run)
        filtered = self.skipping is not None or self.partition is not None or self.predicate is not None
        plain = (not filtered or os.environ.get("DK_ASYNC_FILTERED", "1") != "0") and \
            (scan_groups(len(self.ckpt_files or [])) or self.shard) and os.environ.get("DK_ASYNC_OPEN", "1") != "0"
        late = bool(plain) and bool(self.ckpt_files) and os.environ.get("DK_TAIL_AFTER_OPEN", "1") != "0"
        if not late:
            start_tail()
        self.ckpt = ParquetSet(engine, self.ckpt_files, leaves, groups=sel, async_open=bool(plain)) \
            if self.ckpt_files else None
        start_tail()
        t3 = time.perf_counter()
        self.prepare_ms.update({"plan_files": (t2 - t1) * 1e3, "checkpoint_open": (t3 - t2) * 1e3})
        if self.ckpt is not None and not self.ckpt.async_open:
            self._open_phases()

    def _open_phases(self):
        """The checkpoint open's phases (an asynchronous open's once it has finished)."""
        om = (C.c_double * 7)()
        check(lib().dk_parquet_open_ms(self.ckpt._h, om))
        self.prepare_ms.update({"open_read_h2d": om[0], "open_metadata": om[1], "open_prepare": om[2],
                                "prep_h2d_headers": om[3], "prep_host_pages": om[4], "prep_device_sizing": om[5],
                                "prep_host_tiles_alloc": om[6]})

    def getRemainingFilter(self):
        """ScanImpl.getRemainingFilter (:221-223): the data filter, which skipping never fully
        applies."""
        return self.data_filter

    def run(self):
        """The device step: commit-tail keys + table, checkpoint decode, probe, selection (with an
        exchange: decode + routing, the exchange, then the probe of the rows the owners flagged)."""
        if getattr(self, "owner", None) is not None:
            # the commit-tail exchange, dk_replay_run and the row exchanges, all in the library
            # (dk_replay_owner_run over the owner's dk_comm)
            self.owner.run_scan(self)
            return
        check(lib().dk_replay_run(self._rh))
        if getattr(self, "exchange", None) is not None and self.shard and self.shard[0] > 1:
            from .shard import ExchangeSide
            self.exchange(ExchangeSide(self))

    def sync(self):
        check(lib().dk_replay_sync(self._rh))
        cnt = (C.c_int64 * 5)()
        check(lib().dk_replay_counters(self._rh, cnt))
        self.metrics = ScanMetrics(*[int(x) for x in cnt])
        tail, ck = (C.c_int64 * 5)(), (C.c_int64 * 5)()
        check(lib().dk_replay_counters_split(self._rh, tail, ck))
        self.tail_metrics = ScanMetrics(*[int(x) for x in tail])
        self.ckpt_metrics = ScanMetrics(*[int(x) for x in ck])

    def selection_bits(self, fi, device=False):
        """Packed selection of checkpoint file fi of this scan (LSB first): a numpy array, or a
        torch uint8 tensor on this GPU filled by the device (for RCCL) when device=True."""
        n = self.ckpt.num_rows(fi)
        nb = (n + 7) // 8
        if device:
            import torch
            t = torch.empty(max(1, nb), dtype=torch.uint8, device="cuda")
            check(lib().dk_replay_ckpt_selection_bits(self._rh, fi, C.c_void_p(t.data_ptr()), n, 1))
            return t[:nb]
        out = np.zeros(max(1, nb), dtype=np.uint8)
        check(lib().dk_replay_ckpt_selection_bits(self._rh, fi, out.ctypes.data, n, 0))
        return out[:nb]

    def kernel_stats(self):
        out = {}
        for i in range(32):
            name, avg, cnt = C.c_char_p(), C.c_double(), C.c_int64()
            if lib().dk_replay_kernel_stats(self._rh, i, C.byref(name), C.byref(avg), C.byref(cnt)) != 0:
                continue
            if cnt.value:
                out[name.value.decode()] = (avg.value, cnt.value)
        return out

    def getScanFiles(self, engine):
        if self.replay is None:
            self.prepare(engine)
            self.replay = True
        else:
            self._detach_batches()          # the rerun reuses the pinned blocks earlier batches view
        t0 = time.perf_counter()
        groups = scan_groups(len(self.ckpt_files or []))
        owner = getattr(self, "owner", None)
        exchanging = owner is not None or (getattr(self, "exchange", None) is not None and self.shard and self.shard[0] > 1)
        if owner is not None and self.ckpt is not None:
            # owner mode: add.size goes to host memory right after the decode, beside the exchanges.
            # A failure here must still reach the peers (they are about to vote in the owner run):
            # this rank answers the run's first vote with its error bit (owner.abort)
            try:
                for leaf in self.PREFETCH_LEAVES:
                    if leaf in self.ckpt.leaves:
                        check(lib().dk_replay_prefetch_leaf(self._rh, leaf.encode()))
                if os.environ.get("DK_INJECT_PREFETCH_FAULT") == str(self.shard[1]):
                    raise DkError("injected prefetch failure (DK_INJECT_PREFETCH_FAULT)")
            except BaseException:
                owner.abort()
                raise
        if groups and not exchanging:
            # grouped: batches go out as their group of files is decoded and probed; the counters are
            # final once the iterator is exhausted (ScanImpl's metrics are read after it, too)
            # add.size (split planning reads it from every scan file) goes to host memory as each
            # group finishes decoding, not at the consumer's first touch
            for leaf in self.PREFETCH_LEAVES:
                if leaf in self.ckpt.leaves:
                    check(lib().dk_replay_prefetch_leaf(self._rh, leaf.encode()))
            check(lib().dk_replay_run_grouped(self._rh, groups))
            check(lib().dk_replay_wait_file(self._rh, -1))
            self.prepare_ms["device_run"] = (time.perf_counter() - t0) * 1e3
            return self._batches(grouped=True)
        self.run()
        self.sync()
        self.prepare_ms["device_run"] = (time.perf_counter() - t0) * 1e3
        return self._batches()

    def _batches(self, grouped=False):
        root = self.table_root()
        leaves = ADD_LEAVES + ([STATS_LEAF] if self.read_stats else [])
        if self.tail.rows and getattr(self, "owner", None) is not None:
            # owner mode: this rank's commit files, one batch each, tagged with their replay-order
            # index (commit_index) so that the ranks' batches merge in the reference's order
            sel = np.zeros(self.tail.rows, dtype=np.uint8)
            check(lib().dk_replay_json_selection(self._rh, sel.ctypes.data, self.tail.rows))
            n_commits = len(self.snapshot.log_segment.deltas)
            for j, a, b in self.tail_file_rows:
                if b <= a:
                    continue
                cols = LazyColumns(leaves, lambda leaf, a=a, b=b: self.tail.column(leaf).slice_rows(a, b))
                if j < n_commits:
                    fb = FilteredColumnarBatch(cols, root, b - a, sel[a:b].view(bool), "json-tail")
                else:                       # the V2 JSON manifest's rows (rank 0): first checkpoint batch
                    fb = FilteredColumnarBatch(cols, root, b - a, sel[a:b].view(bool),
                                               self.snapshot._json_checkpoint_parts()[0], -1, 0)
                fb.commit_index = j
                self._handed[id(fb)] = fb
                yield fb
        elif self.tail.rows:
            sel = np.zeros(self.tail.rows, dtype=np.uint8)
            check(lib().dk_replay_json_selection(self._rh, sel.ctypes.data, self.tail.rows))
            r0 = int(self.tail.ckpt_row0)
            if r0 > 0:
                cols = LazyColumns(leaves, self.tail.column)
                fb = FilteredColumnarBatch(cols, root, r0, sel[:r0].view(bool), "json-tail")
                self._handed[id(fb)] = fb
                yield fb
            if r0 < self.tail.rows:
                # a V2 JSON manifest's rows: the first checkpoint batch (ActionsIterator reads the
                # manifest before its sidecars)
                cols = LazyColumns(leaves, lambda leaf: self.tail.column(leaf).slice_rows(r0, self.tail.rows))
                fb = FilteredColumnarBatch(cols, root, int(self.tail.rows - r0), sel[r0:].view(bool),
                                           self.snapshot._json_checkpoint_parts()[0], -1, 0)
                self._handed[id(fb)] = fb
                yield fb
        # checkpoint batches: zero-copy views of the library's pinned selection bytes and column
        # mirrors (every file's selection comes to the host in one round of copies; a leaf's first
        # access queues its copy for every later file), valid until the scan is closed
        for fi, path in enumerate(self.ckpt_files or []):
            if grouped:
                check(lib().dk_replay_wait_file(self._rh, fi))
            n = self.ckpt.num_rows(fi)
            ptr = C.c_void_p()
            check(lib().dk_replay_ckpt_selection_host(self._rh, fi, C.byref(ptr)))
            sel = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_bool)), shape=(n,)) if n else np.zeros(0, bool)
            cols = LazyColumns(leaves, lambda leaf, fi=fi: self.ckpt.column(fi, leaf, copy=False))
            fb = FilteredColumnarBatch(cols, root, int(n), sel, path, self.ckpt_index[fi],
                                       int(self.ckpt.row_offset(fi)))
            self._handed[id(fb)] = fb
            yield fb
        if grouped:
            self.sync()                     # the counters (and any error the waits did not see)
            if self.ckpt is not None and self.ckpt.async_open:
                self._open_phases()

    def _detach_batches(self):
        """Checkpoint batches handed out by getScanFiles view the library's pinned selection and
        column mirrors (zero-copy). Before a rerun or close recycles those blocks, every batch still
        referenced gets its own copies of its selection and of every leaf, so that it stays valid
        after the iterator and the scan are closed, as the reference's batches do."""
        live = list(getattr(self, "_handed", {}).values())
        self._handed = weakref.WeakValueDictionary()
        for b in live:
            if b.selection is not None:
                b.selection = np.array(b.selection, copy=True)
            for leaf in b.data.keys():
                got = dict.get(b.data, leaf)
                if got is None and dict.__contains__(b.data, leaf):
                    continue                                  # fetched: absent from the file
                if got is None:
                    c = b.data._fetch(leaf)                   # not read yet: read it now
                    got = c if c.present else None
                dict.__setitem__(b.data, leaf, None if got is None else _own_column(got))
            b.data._fetch = None

    def close(self):
        t0 = time.perf_counter()
        if getattr(self, "_handed", None):
            self._detach_batches()
        t1 = time.perf_counter()
        if getattr(self, "_rh", None):
            lib().dk_replay_free(self._rh)
            self._rh = None
        t2 = time.perf_counter()
        for o in ("ckpt", "tail"):
            x = getattr(self, o, None)
            if x is not None:
                x.close()
        t3 = time.perf_counter()
        # where close() spends its time (bench.py's DK_CONSUME_PROFILE block)
        self.close_ms = dict(close_detach=(t1 - t0) * 1e3, close_replay=(t2 - t1) * 1e3, close_inputs=(t3 - t2) * 1e3)
