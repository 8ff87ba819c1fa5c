"""Oracle (test infrastructure): CreateCheckpointIterator restated on the CPU.

  CreateCheckpointIterator.prepareNext / processRemoves / processAdds / processProtocol /
  processMetadata / processTxn / processDomainMetadata
      kernel/kernel-api/src/main/java/io/delta/kernel/internal/replay/CreateCheckpointIterator.java:
      63-416
  SnapshotImpl.getCreateCheckpointIterator (retention)   internal/SnapshotImpl.java:170-174

Independent of the product: commit lines are read here, keys come from the oracle's own
java.net.URI restatement (ref.json_key) and checkpoint rows from the C decoder. Output: the selected
rows in iterator order as canonical (action, tuple) pairs (see canon()), and the add count.

Parity unpinned: /root/reference holds no checkpoint written by Kernel's CreateCheckpointIterator (no
golden output to compare with), so this restatement is checked on hand-made logs and through round
trips (the written file read back by pyarrow, the table re-read through the new checkpoint), not
against a reference-produced vector.
"""
import json
import os

import numpy as np

from . import ref

_UNITS = {"microsecond": 1e-3, "millisecond": 1, "second": 1000, "minute": 60_000, "hour": 3_600_000,
          "day": 86_400_000, "week": 604_800_000}


def retention_ms(conf):
    text = (conf or {}).get("delta.deletedFileRetentionDuration", "interval 1 week").strip().lower()
    parts = text.split()
    if parts and parts[0] == "interval":
        parts = parts[1:]
    return int(sum(float(parts[i]) * _UNITS[parts[i + 1].rstrip("s")] for i in range(0, len(parts), 2)))


def _t(v):
    return v.decode() if isinstance(v, bytes) else v


def _m(m):
    if m is None:
        return None
    items = m.items() if isinstance(m, dict) else m
    return tuple((_t(k), _t(v)) for k, v in items)


def canon(kind, v):
    """A comparable tuple for one action value (python dicts / lists, as json or pyarrow give them)."""
    if v is None:
        return None
    if kind in ("add", "remove"):
        dv = v.get("deletionVector")
        dvt = None if dv is None else tuple(_t(dv.get(k)) for k in ("storageType", "pathOrInlineDv", "offset",
                                                                    "sizeInBytes", "cardinality"))
        keys = ("path", "size", "modificationTime", "dataChange", "stats", "baseRowId", "defaultRowCommitVersion") \
            if kind == "add" else ("path", "deletionTimestamp", "dataChange", "extendedFileMetadata", "size", "stats",
                                   "baseRowId", "defaultRowCommitVersion")
        return tuple(_t(v.get(k)) for k in keys) + (_m(v.get("partitionValues")), _m(v.get("tags")), dvt)
    if kind == "protocol":
        return (v["minReaderVersion"], v["minWriterVersion"], tuple(v.get("readerFeatures") or ()),
                tuple(v.get("writerFeatures") or ()))
    if kind == "metaData":
        fmt = v.get("format") or {}
        return (v["id"], v.get("name"), v.get("description"), fmt.get("provider"), _m(fmt.get("options") or {}),
                v["schemaString"], tuple(v.get("partitionColumns") or ()), v.get("createdTime"),
                _m(v.get("configuration") or {}))
    if kind == "txn":
        return (v["appId"], v["version"], v.get("lastUpdated"))
    return (v["domain"], v["configuration"], v["removed"])


def checkpoint_actions(table_root, now_ms):
    seg = ref.load_log_segment(table_root)
    prot, meta, _ = ref.load_protocol_metadata(table_root)
    min_ret = now_ms - retention_ms(meta.get("configuration"))
    out, n_adds = [], 0
    tomb, added = set(), set()
    seen = {"protocol": set(), "metaData": set(), "txn": set(), "domainMetadata": set()}

    def first(kind, key):
        if key in seen[kind]:
            return False
        seen[kind].add(key)
        return True

    rep = None
    for f in seg.all_files_reversed():
        if f.kind == "commit":
            with open(f.path, "rb") as fh:
                raw = [json.loads(x) for x in fh.read().decode("utf-8", "replace").splitlines()]
            rows = [r for b in ref.read_json_batches(f.path, 1 << 30, True) for r in b]
            assert len(rows) == len(raw)
            sel = [False] * len(raw)
            for i, row in enumerate(rows):                      # processRemoves
                if row["remove"] is not None:
                    tomb.add(ref.json_key(row["remove"]))
                    sel[i] = int(raw[i]["remove"].get("deletionTimestamp") or 0) > min_ret
            for i, row in enumerate(rows):                      # processAdds
                if row["add"] is not None:
                    k = ref.json_key(row["add"])
                    if k not in added:
                        added.add(k)
                        if k not in tomb:
                            sel[i] = True
            for i, obj in enumerate(raw):
                for kind in ("protocol", "metaData", "txn", "domainMetadata"):
                    if obj.get(kind) is not None:
                        key = 0 if kind in ("protocol", "metaData") else obj[kind].get("appId" if kind == "txn"
                                                                                       else "domain")
                        sel[i] = first(kind, key)
            for i, obj in enumerate(raw):
                if not sel[i]:
                    continue
                kind = next(k for k in ("add", "remove", "protocol", "metaData", "txn", "domainMetadata")
                            if obj.get(k) is not None)
                val = prot if kind == "protocol" else meta if kind == "metaData" else obj[kind]
                out.append((kind, canon(kind, val)))
                n_adds += kind == "add"
            continue
        # checkpoint part: the scan replay's checkpoint selection for adds (same rule), the first
        # protocol / metaData / txn / domainMetadata for the rest
        if rep is None:
            rep = {b.path: b for b in ref.replay(table_root, with_stats=True).checkpoint}
        b = rep[f.path]
        pf = ref.ParquetFile.open(f.path)
        cols = {leaf: pf.read(leaf) for leaf in ("protocol.minReaderVersion", "metaData.id", "txn.appId", "txn.version",
                                                  "txn.lastUpdated", "domainMetadata.domain",
                                                  "domainMetadata.configuration", "domainMetadata.removed")}

        def has(leaf, r):
            c = cols[leaf]
            return c is not None and c.row_def[r] >= 1

        for r in range(pf.num_rows):
            if b.selected[r]:
                a = ref.canon_add_from_cols(b.cols, r)
                v = {"path": a[0], "partitionValues": a[1], "size": a[2], "modificationTime": a[3], "dataChange": a[4],
                     "deletionVector": None if a[5] is None else dict(zip(("storageType", "pathOrInlineDv", "offset",
                                                                            "sizeInBytes", "cardinality"), a[5])),
                     "tags": a[6], "baseRowId": a[7], "defaultRowCommitVersion": a[8], "stats": a[9]}
                out.append(("add", canon("add", v)))
                n_adds += 1
            elif has("protocol.minReaderVersion", r):
                if first("protocol", 0):
                    out.append(("protocol", canon("protocol", prot)))
            elif has("metaData.id", r):
                if first("metaData", 0):
                    out.append(("metaData", canon("metaData", meta)))
            elif has("txn.appId", r):
                app = cols["txn.appId"].string(r).decode()
                if first("txn", app):
                    out.append(("txn", (app, ref._fixed_at(cols["txn.version"], r, np.int64),
                                        ref._fixed_at(cols["txn.lastUpdated"], r, np.int64))))
            elif has("domainMetadata.domain", r):
                dom = cols["domainMetadata.domain"].string(r).decode()
                if first("domainMetadata", dom):
                    rm = cols["domainMetadata.removed"]
                    out.append(("domainMetadata", (dom, _t(ref._str_at(cols["domainMetadata.configuration"], r, 2)),
                                                   None if rm.row_def[r] < rm.max_def else bool(rm.fixed[r]))))
    return out, n_adds


def read_checkpoint(path):
    """A written checkpoint read back with pyarrow: (action, canonical tuple) per row."""
    import pyarrow.parquet as pq
    t = pq.read_table(path)
    out = []
    for row in t.to_pylist():
        kinds = [k for k in ("txn", "add", "remove", "metaData", "protocol", "domainMetadata") if row.get(k) is not None]
        assert len(kinds) == 1, row
        out.append((kinds[0], canon(kinds[0], row[kinds[0]])))
    return out
