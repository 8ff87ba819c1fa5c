"""Partition-pruning planning (host side): the partition part of a scan filter
(PartitionUtils.splitMetadataAndDataPredicates, delta_amd/skipping.split_filters). The predicate is
rewritten over the scan file's partitionValues map and compiled behind the C ABI (dk_part_compile,
delta_amd/programs.py; delta_amd/csrc/dk_expr.cpp), which k_part_eval runs (ScanImpl.applyPartitionPruning,
ScanImpl.java:247-294). This module keeps the partition column table and the checkpoint row-group
predicate (ActionsIterator.java:336-351 -> ParquetFileReader.java:111-132).

The device evaluates partition columns of type string, binary, long, integer, short, byte, date
(java.sql.Date.valueOf, PartitionValueEvaluator.java:72-73), decimal (new BigDecimal(text), :112-113,
compareTo), boolean (Boolean.parseBoolean), float / double (Float.parseFloat / Double.parseDouble,
compared exactly through planned thresholds with Float.compare semantics and ImplicitCastExpression
widening), timestamp / timestamp_ntz (java.sql.Timestamp.valueOf -> InternalUtils.microsSinceEpoch, read
as UTC); =, <, <=, >, >=, IS NOT DISTINCT FROM, IS_NULL, IS_NOT_NULL, NOT, AND, OR, COALESCE,
ALWAYS_TRUE / ALWAYS_FALSE, with no size limit. What the device does not evaluate raises
UnsupportedPartitionFilter (DESIGN.md §4.2 lists it).
"""
from __future__ import annotations

import json

from .expressions import Column, Literal, Predicate


class UnsupportedPartitionFilter(RuntimeError):
    pass


def partition_fields(schema_string: str, partition_columns) -> dict:
    """lower-case partition column name -> (type name, physical name) (ScanImpl.java:86-94)."""
    parts = {p.lower() for p in partition_columns}
    out = {}
    for f in json.loads(schema_string)["fields"]:
        if f["name"].lower() in parts:
            t = f["type"] if isinstance(f["type"], str) else "complex"
            phys = (f.get("metadata") or {}).get("delta.columnMapping.physicalName", f["name"])
            out[f["name"].lower()] = (t, phys)
    return out


# ---- checkpoint row-group pruning (ActionsIterator.java:336-351 -> ParquetFileReader.java:111-132) ----
RF_COL, RF_LIT, RF_NULL, RF_EQ, RF_LT, RF_LE, RF_GT, RF_GE, RF_AND, RF_OR, RF_NOT, RF_ISNULL, RF_ISNOTNULL, \
    RF_UNSUPPORTED = range(14)
RL = {"long": 0, "integer": 1, "short": 2, "byte": 3, "date": 4, "float": 5, "double": 6, "boolean": 7, "string": 8}
_RF_CMP = {"=": RF_EQ, "<": RF_LT, "<=": RF_LE, ">": RF_GT, ">=": RF_GE}


def row_group_filter(pred: Predicate, fields: dict):
    """The partition filter rewritten onto add.partitionValues_parsed.<physical name>
    (PartitionUtils.rewritePartitionPredicateOnCheckpointFileSchema, PartitionUtils.java:275-303) as a
    dk_rg_filter program: (column paths, ops, pool). Conversion to parquet-mr filters and the
    row-group statistics test happen per file in libdkgpu (dk_parquet_prune_row_groups)."""
    import struct
    cols, ops = [], []
    pool = bytearray()

    def col(c: Column):
        name = c.names[0].lower()
        if name not in fields:
            raise ValueError("%s is not present in metadata" % c.names[0])
        path = "add.partitionValues_parsed." + fields[name][1]
        if path not in cols:
            cols.append(path)
        ops.append((RF_COL, cols.index(path), 0))

    def lit(x: Literal):
        if x.value is None:
            ops.append((RF_NULL, 0, 0))
        elif x.type == "string":
            b = x.value.encode("utf-8")
            ops.append((RF_LIT, RL["string"], len(pool) | (len(b) << 32)))
            pool.extend(b)
        elif x.type in ("float", "double"):
            ops.append((RF_LIT, RL[x.type], struct.unpack("<q", struct.pack("<d", float(x.value)))[0]))
        elif x.type == "boolean":
            ops.append((RF_LIT, RL["boolean"], int(bool(x.value))))
        elif x.type in RL:
            ops.append((RF_LIT, RL[x.type], int(x.value)))
        else:
            ops.append((RF_LIT, 9, 0))                     # timestamp / decimal / ...: not convertible

    def expr(e):
        if isinstance(e, Column):
            col(e)
        elif isinstance(e, Literal):
            lit(e)
        else:
            node(e)

    def node(p: Predicate):
        n = p.name.lower()
        c = p.children
        if n in _RF_CMP and len(c) == 2:
            expr(c[0])
            expr(c[1])
            ops.append((_RF_CMP[n], 0, 0))
        elif n in ("and", "or") and len(c) == 2:
            node(c[0])
            node(c[1])
            ops.append((RF_AND if n == "and" else RF_OR, 0, 0))
        elif n == "not" and len(c) == 1:
            node(c[0])
            ops.append((RF_NOT, 0, 0))
        elif n in ("is_null", "is_not_null") and len(c) == 1:
            expr(c[0])
            ops.append((RF_ISNULL if n == "is_null" else RF_ISNOTNULL, 0, 0))
        else:
            for ch in c:                                    # columns must still exist in metadata
                if isinstance(ch, Column):
                    name = ch.names[0].lower()
                    if name not in fields:
                        raise ValueError("%s is not present in metadata" % ch.names[0])
            ops.append((RF_UNSUPPORTED, 0, 0))

    node(pred)
    return cols, ops, bytes(pool)


def pack_row_group_filter(program, struct_type):
    """A dk_rg_filter over arrays this function allocates (kept alive on the returned struct)."""
    import numpy as np
    cols, ops, pool = program
    pool = bytearray(pool)
    off, ln = [], []
    for c in cols:
        b = c.encode("utf-8")
        off.append(len(pool))
        ln.append(len(b))
        pool.extend(b)
    f = struct_type()
    keep = [np.array(off, np.int32), np.array(ln, np.int32), np.array([o for o, _, _ in ops], np.int32),
            np.array([a for _, a, _ in ops], np.int32), np.array([l for _, _, l in ops], np.int64),
            np.frombuffer(bytes(pool) + b"\0", np.uint8).copy()]
    f.n_cols, f.n_ops, f.pool_len = len(cols), len(ops), len(pool)
    f.col_off, f.col_len, f.op, f.arg, f.lit, f.pool = [k.ctypes.data for k in keep]
    f._keep = keep
    return f
