"""Checkpoint writing: Table.checkpoint -> SnapshotManager.checkpoint over CreateCheckpointIterator.

Reference (paths under /root/reference/kernel/kernel-api/src/main/java/io/delta/kernel/internal/):
  SnapshotManager.checkpoint                snapshot/SnapshotManager.java:151-200
  SnapshotImpl.getCreateCheckpointIterator  SnapshotImpl.java:170-174 (retention = now - TOMBSTONE_RETENTION)
  CreateCheckpointIterator                  replay/CreateCheckpointIterator.java:63-416
  TableFeatures.validateWriteSupportedTable TableFeatures.java:33-45,110-160,270-277
  SingleAction.CHECKPOINT_SCHEMA            actions/SingleAction.java:30-37 (+ AddFile / RemoveFile /
                                            Metadata / Protocol / SetTransaction / DomainMetadata FULL_SCHEMA)
  Checkpointer.writeLastCheckpointFile      checkpoints/Checkpointer.java:185-203

What runs where:
  * the add selection -- the latest-version-wins reconciliation of every add in the log segment
    against the commit tail's tombstones and earlier adds (processAdds, :234-254) -- is the GPU replay
    of Scan.getScanFiles (decode + keys + probe in libdkgpu), which applies exactly that rule;
  * commit-tail removes are kept while deletionTimestamp > now - delta.deletedFileRetentionDuration
    (processRemoves, :210-232); checkpoint removes are never rewritten;
  * protocol / metaData / txn (per appId) / domainMetadata (per domain): the first seen in reverse
    log order (:256-330);
  * rows come out in the iterator's order (commits newest first, then the checkpoint, row order);
  * the Parquet file is encoded on the device (dk_ckpt_writer_*, the ParquetHandler.writeParquetFileAtomically
    role, DefaultParquetHandler.java:115-163) and written atomically (a temporary file linked into
    place, failing when the checkpoint exists), then _last_checkpoint {version, size = adds kept}.
"""
from __future__ import annotations

import json
import os
import re
import time

import numpy as np

from ._lib import DkError

SUPPORTED_WRITER_FEATURES = frozenset(["appendOnly", "inCommitTimestamp", "columnMapping", "typeWidening-preview",
                                       "typeWidening", "domainMetadata", "rowTracking"])     # TableFeatures.java:33-45


class CheckpointAlreadyExistsException(DkError):
    pass


def validate_write_supported(protocol, metadata, table_path):
    """TableFeatures.validateWriteSupportedTable (TableFeatures.java:110-160)."""
    from .actions import KernelException
    schema = json.loads(metadata["schemaString"])

    def no_invariants():
        if any("delta.invariants" in (f.get("metadata") or {}) for f in schema.get("fields", [])):
            raise KernelException("This version of Delta Kernel does not support writing to tables with "
                                  "column invariants.")

    wv = protocol["minWriterVersion"]
    if wv == 1:
        return
    if wv == 2:
        no_invariants()
        return
    if wv == 7:
        feats = protocol.get("writerFeatures") or []
        for f in feats:
            if f == "invariants":
                no_invariants()
            elif f not in SUPPORTED_WRITER_FEATURES:
                raise KernelException("Unsupported Delta writer feature: table `%s` requires writer table feature "
                                      "\"%s\" which is unsupported by this version of Delta Kernel." % (table_path, f))
        if "rowTracking" in feats and "domainMetadata" not in feats:
            raise KernelException("Feature 'rowTracking' is supported and depends on feature 'domainMetadata', "
                                  "but 'domainMetadata' is unsupported")
        return
    raise KernelException("Unsupported Delta writer protocol: table `%s` requires writer version %d which is "
                          "unsupported by this version of Delta Kernel." % (table_path, wv))


_UNIT_MS = {"microsecond": 1e-3, "millisecond": 1, "second": 1000, "minute": 60_000, "hour": 3_600_000,
            "day": 86_400_000, "week": 604_800_000}


def interval_ms(text):
    """IntervalParserUtils.safeParseIntervalAsMillis for '[interval] <n> <unit>[s] ...' (the forms
    delta.deletedFileRetentionDuration takes; months / years are not fixed lengths and refused)."""
    s = text.strip().lower()
    if not s.startswith("interval "):
        s = "interval " + s
    parts = s.split()[1:]
    if not parts or len(parts) % 2:
        raise DkError("Error parsing '%s' to interval" % text)
    total = 0.0
    for i in range(0, len(parts), 2):
        n, unit = parts[i], parts[i + 1].rstrip("s")
        if unit not in _UNIT_MS or not re.fullmatch(r"[+-]?\d+(\.\d+)?", n):
            raise DkError("Error parsing '%s' to interval" % text)
        total += float(n) * _UNIT_MS[unit]
    return int(total)


_ADD_KEYS = ("path", "partitionValues", "size", "modificationTime", "dataChange", "stats", "tags", "deletionVector",
             "baseRowId", "defaultRowCommitVersion")
_RM_KEYS = ("path", "deletionTimestamp", "dataChange", "extendedFileMetadata", "partitionValues", "size", "stats",
            "tags", "deletionVector", "baseRowId", "defaultRowCommitVersion")
_DV_KEYS = ("storageType", "pathOrInlineDv", "offset", "sizeInBytes", "cardinality")


def _pick(obj, keys):
    if obj is None:
        return None
    out = {k: obj.get(k) for k in keys}
    if out.get("deletionVector") is not None:
        out["deletionVector"] = {k: out["deletionVector"].get(k) for k in _DV_KEYS}
    for m in ("partitionValues", "tags"):
        if isinstance(out.get(m), dict):
            out[m] = list(out[m].items())
    return out


# ---- decoded checkpoint columns -> python values ------------------------------------------------
def _s(c, r, maxdef=None):
    if c is None or not c.present or c.row_def[r] < (c.max_def if maxdef is None else maxdef):
        return None
    return c.string(r).decode("utf-8", "replace")


def _f(c, r, dtype):
    if c is None or not c.present or c.row_def[r] < c.max_def:
        return None
    w = np.dtype(dtype).itemsize
    return c.fixed[r * w:(r + 1) * w].view(dtype)[0].item()


def _m(kc, vc, r):
    if kc is None or not kc.present or kc.row_def[r] < kc.rep_def - 1:
        return None
    out = []
    for j in range(int(kc.row_offs[r]), int(kc.row_offs[r + 1])):
        k = bytes(kc.chars[kc.offs[j]:kc.offs[j + 1]]).decode("utf-8", "replace")
        v = None
        if vc is not None and vc.present and vc.entry_def[j] == vc.max_def:
            v = bytes(vc.chars[vc.offs[j]:vc.offs[j + 1]]).decode("utf-8", "replace")
        out.append((k, v))
    return out


def _add_from_cols(d, r):
    g = d.get
    dv = None
    st = g("add.deletionVector.storageType")
    # the deletionVector struct is defined iff the level reaches the struct's own (optional add = 1,
    # optional deletionVector = 2), whether storageType itself is optional (max_def 3) or required
    # (max_def 2, DeletionVectorDescriptor.READ_SCHEMA marks it non-nullable); RowColumnReader
    # starts the struct exactly then (RowColumnReader.java:65-173)
    if st is not None and st.present and st.row_def[r] >= 2:
        dv = {"storageType": _s(st, r), "pathOrInlineDv": _s(g("add.deletionVector.pathOrInlineDv"), r),
              "offset": _f(g("add.deletionVector.offset"), r, np.int32),
              "sizeInBytes": _f(g("add.deletionVector.sizeInBytes"), r, np.int32),
              "cardinality": _f(g("add.deletionVector.cardinality"), r, np.int64)}
    dc = g("add.dataChange")
    return {"path": _s(g("add.path"), r),
            "partitionValues": _m(g("add.partitionValues.key_value.key"), g("add.partitionValues.key_value.value"), r),
            "size": _f(g("add.size"), r, np.int64), "modificationTime": _f(g("add.modificationTime"), r, np.int64),
            "dataChange": None if dc is None or dc.row_def[r] < dc.max_def else bool(dc.fixed[r]),
            "stats": _s(g("add.stats"), r), "tags": _m(g("add.tags.key_value.key"), g("add.tags.key_value.value"), r),
            "deletionVector": dv, "baseRowId": _f(g("add.baseRowId"), r, np.int64),
            "defaultRowCommitVersion": _f(g("add.defaultRowCommitVersion"), r, np.int64)}


def _checkpoint_other_rows(engine, files):
    """Per old checkpoint file (replay order): {row: (action, value)} for its protocol / metaData /
    txn / domainMetadata rows (decoded on the GPU; protocol and metaData values are the snapshot's)."""
    from .kernel import ParquetSet
    leaves = ["protocol.minReaderVersion", "metaData.id", "txn.appId", "txn.version", "txn.lastUpdated",
              "domainMetadata.domain", "domainMetadata.configuration", "domainMetadata.removed"]
    out = []
    if not files:
        return out
    ps = ParquetSet(engine, files, leaves).decode()
    try:
        for fi in range(len(files)):
            cols = ps.columns(fi)
            rows = {}
            pc, mc, a, dmn = cols["protocol.minReaderVersion"], cols["metaData.id"], cols["txn.appId"], \
                cols["domainMetadata.domain"]
            for r in range(ps.num_rows(fi)):
                if pc is not None and pc.row_def[r] >= 1:
                    rows[r] = ("protocol", None)
                elif mc is not None and mc.row_def[r] >= 1:
                    rows[r] = ("metaData", None)
                elif a is not None and a.row_def[r] >= 1:
                    rows[r] = ("txn", {"appId": _s(a, r), "version": _f(cols["txn.version"], r, np.int64),
                                       "lastUpdated": _f(cols["txn.lastUpdated"], r, np.int64)})
                elif dmn is not None and dmn.row_def[r] >= 1:
                    rm = cols["domainMetadata.removed"]
                    rows[r] = ("domainMetadata", {"domain": _s(dmn, r),
                                                  "configuration": _s(cols["domainMetadata.configuration"], r),
                                                  "removed": None if rm is None or rm.row_def[r] < rm.max_def
                                                  else bool(rm.fixed[r])})
            out.append(rows)
    finally:
        ps.close()
    return out


def checkpoint_actions(engine, snapshot, now_ms=None, sink=None):
    """CreateCheckpointIterator's output: the selected rows of every batch, batches in reverse log
    order and rows in batch order, as (action name, value dict) pairs; plus the number of add
    actions kept (getNumberOfAddActions).

    sink (the GPU encoder): instead of materialising the old checkpoint's surviving adds, every
    maximal run of checkpoint rows between two other actions is handed over as
    sink(("ckpt", scan, file, row0, row1)) -- the device gathers those rows by the replay's
    selection -- with the rows before it flushed first as sink(("rows", [(action, value)...]))."""
    md = snapshot.metadata
    retention = interval_ms((md.get("configuration") or {}).get("delta.deletedFileRetentionDuration",
                                                                 "interval 1 week"))
    now_ms = int(time.time() * 1000) if now_ms is None else now_ms
    min_retention = now_ms - retention
    scan = snapshot.getScanBuilder().withStats(True).build()
    out = []
    n_adds = 0
    seen = {"protocol": set(), "metaData": set(), "txn": set(), "domainMetadata": set()}

    def first(kind, key):
        if key in seen[kind]:
            return False
        seen[kind].add(key)
        return True

    try:
        batches = scan.getScanFiles(engine)
        n_commit_rows = int(scan.tail.ckpt_row0)          # (a V2 JSON manifest's rows follow them)
        tail = next(batches) if n_commit_rows else None
        # commit rows: the JSON lines in tail order (newest commit first); the add selection is the
        # GPU replay's, the rest follows processRemoves / processProtocol / ... row by row
        row = 0
        for d in reversed(snapshot.log_segment.deltas):
            with open(d.path, "rb") as f:
                raw = f.read()
            # one row per line as the tail parser splits them (BufferedReader.readLine: '\n', '\r'
            # or '\r\n' ends a line), so row indices line up with the tail selection; other
            # separators str.splitlines() would honour (U+2028, U+0085, ...) may sit inside JSON
            # strings
            text = raw.decode("utf-8", "replace")
            lines = re.split(r"\r\n|\r|\n", text)
            if lines and lines[-1] == "":
                lines.pop()
            for line in lines:
                obj = json.loads(line)
                r, row = row, row + 1
                if obj.get("remove") is not None:
                    rm = obj["remove"]
                    if int(rm.get("deletionTimestamp") or 0) > min_retention:
                        out.append(("remove", _pick(rm, _RM_KEYS)))
                elif obj.get("add") is not None:
                    if tail is not None and tail.selection[r]:
                        out.append(("add", _pick(obj["add"], _ADD_KEYS)))
                        n_adds += 1
                elif obj.get("protocol") is not None:
                    if first("protocol", 0):
                        out.append(("protocol", snapshot.protocol))
                elif obj.get("metaData") is not None:
                    if first("metaData", 0):
                        out.append(("metaData", snapshot.metadata))
                elif obj.get("txn") is not None:
                    t = obj["txn"]
                    if first("txn", t.get("appId")):
                        out.append(("txn", {"appId": t.get("appId"), "version": t.get("version"),
                                            "lastUpdated": t.get("lastUpdated")}))
                elif obj.get("domainMetadata") is not None:
                    dm = obj["domainMetadata"]
                    if first("domainMetadata", dm.get("domain")):
                        out.append(("domainMetadata", {k: dm.get(k) for k in ("domain", "configuration", "removed")}))
        if tail is not None and row != n_commit_rows:
            raise DkError("commit tail rows do not match the commit lines")
        # checkpoint rows in file order: adds the GPU replay kept; the first protocol / metaData /
        # txn per appId / domainMetadata per domain
        others = _checkpoint_other_rows(engine, list(scan.ckpt_files or []))
        for fi, b in enumerate(batches):
            oth = others[fi] if fi < len(others) else {}
            if sink is not None and b.file_index >= 0:
                # runs of rows between the other actions go to the device encoder whole
                r0 = 0
                for r in sorted(oth) + [b.size]:
                    if r > r0:
                        sink(("rows", out))
                        out = []
                        sink(("ckpt", scan, fi, r0, r))
                    if r < b.size:
                        kind, v = oth[r]
                        key = 0 if kind in ("protocol", "metaData") else (v["appId"] if kind == "txn" else v["domain"])
                        if first(kind, key):
                            out.append((kind, snapshot.protocol if kind == "protocol" else
                                        snapshot.metadata if kind == "metaData" else v))
                    r0 = r + 1
                n_adds += int(b.size if b.selection is None else np.count_nonzero(b.selection))
                continue
            sel = set(int(r) for r in b.selected_rows())
            for r in sorted(sel | set(oth)):
                if r in sel:
                    out.append(("add", _add_from_cols(b.data, r)))
                    n_adds += 1
                    continue
                kind, v = oth[r]
                key = 0 if kind in ("protocol", "metaData") else (v["appId"] if kind == "txn" else v["domain"])
                if first(kind, key):
                    out.append((kind, snapshot.protocol if kind == "protocol" else
                                snapshot.metadata if kind == "metaData" else v))
        if sink is not None:
            sink(("rows", out))
            out = []
    finally:
        scan.close()
    return out, n_adds


def _json_value(kind, v):
    """A checkpoint row's value as the JSON object the device encoder shreds (maps as objects)."""
    if v is None:
        return None
    if kind == "metaData":
        return {"id": v["id"], "name": v.get("name"), "description": v.get("description"),
                "format": {"provider": v["format"]["provider"], "options": dict(v["format"].get("options") or {})},
                "schemaString": v["schemaString"], "partitionColumns": v["partitionColumns"],
                "createdTime": v.get("createdTime"), "configuration": dict(v.get("configuration") or {})}
    if kind in ("add", "remove"):
        v = dict(v)
        for m in ("partitionValues", "tags"):
            if isinstance(v.get(m), list):
                v[m] = dict(v[m])
    return v


def _write_gpu(engine, snap, path, now_ms, codec=1):
    """The checkpoint file encoded on the device (dk_ckpt_writer_*): action rows built here go over
    as JSON lines, the old checkpoint's surviving adds never leave the GPU."""
    import ctypes as C
    from ._lib import check, lib
    w = C.c_void_p()
    check(lib().dk_ckpt_writer_open(engine._h, path.encode(), codec, C.byref(w)))
    try:
        def sink(item):
            if item[0] == "rows":
                if item[1]:
                    text = "\n".join(json.dumps({k: _json_value(k, v)}) for k, v in item[1]).encode()
                    check(lib().dk_ckpt_writer_add_json(w, text, len(text)))
            else:
                _, scan, fi, r0, r1 = item
                n = C.c_int64()
                check(lib().dk_ckpt_writer_add_checkpoint_adds(w, scan._rh, fi, r0, r1, C.byref(n)))
        _, n_adds = checkpoint_actions(engine, snap, now_ms, sink=sink)
    except BaseException:
        lib().dk_ckpt_writer_close(w, None, None)
        raise
    nr, size = C.c_int64(), C.c_int64()
    check(lib().dk_ckpt_writer_close(w, C.byref(nr), C.byref(size)))
    return n_adds


def write_checkpoint(engine, table_path, now_ms=None):
    """SnapshotManager.checkpoint at the latest version: <v>.checkpoint.parquet + _last_checkpoint,
    the file encoded on the device (dk_ckpt_writer_*). Returns (version, number of add actions)."""
    from .kernel import Table
    snap = Table.forPath(engine, table_path).getLatestSnapshot(engine)
    v = snap.getVersion()
    validate_write_supported(snap.protocol, snap.metadata, "file:" + os.path.abspath(table_path))
    log = snap.log_segment.log_path
    final = os.path.join(log, "%020d.checkpoint.parquet" % v)
    if os.path.exists(final):
        raise CheckpointAlreadyExistsException("Checkpoint for given version %d already exists in the table" % v)
    tmp = os.path.join(log, ".%020d.checkpoint.parquet.%d.tmp" % (v, os.getpid()))
    try:
        n_adds = _write_gpu(engine, snap, tmp, now_ms)
    except BaseException:
        if os.path.exists(tmp):
            os.remove(tmp)
        raise
    try:
        os.link(tmp, final)                     # atomic, and fails when the checkpoint exists
    except FileExistsError:
        raise CheckpointAlreadyExistsException("Checkpoint for given version %d already exists in the table" % v)
    finally:
        os.remove(tmp)
    lc_tmp = os.path.join(log, "._last_checkpoint.%d.tmp" % os.getpid())
    with open(lc_tmp, "w") as f:
        f.write(json.dumps({"version": v, "size": n_adds}) + "\n")
    os.replace(lc_tmp, os.path.join(log, "_last_checkpoint"))
    return v, n_adds
