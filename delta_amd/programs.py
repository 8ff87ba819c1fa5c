"""Host side of the predicate compiler behind the C ABI (dk_skip_compile / dk_part_compile,
include/dkgpu.h; delta_amd/csrc/dk_expr.cpp). This module only serializes Kernel expressions to the
ABI's predicate JSON -- the same JSON a Java ExpressionHandler would write with a visitor
 -- and wraps the compiled dk_program handle:

  * data skipping: the DataSkippingPredicate (skipping.construct restates
    DataSkippingUtils.constructDataSkippingFilter, kernel-api/.../internal/skipping/
    DataSkippingUtils.java:156-456) over the pruned stats schema (DataSkippingUtils.pruneStatsSchema,
    ScanImpl.java:309-312), wrapped as ScanImpl wraps it: =(COALESCE(skip, true), ALWAYS_TRUE);
  * partition pruning: the partition predicate rewritten over the scan-file schema
    (PartitionUtils.rewritePartitionPredicateOnScanFileSchema, util/PartitionUtils.java:324-358).
"""
from __future__ import annotations

import ctypes as C
import json
import struct
from decimal import Decimal

from ._lib import DkError, lib
from .expressions import Column, Literal, Predicate

STATUS_UNSUPPORTED_EXPRESSION = 3        # the reference's evaluator throws for this predicate


class Program:
    """A compiled dk_program (owned; freed on close / garbage collection)."""

    def __init__(self, handle):
        self._h = handle
        self._desc = None

    @property
    def handle(self):
        return self._h

    def describe(self) -> dict:
        """dk_program_describe: kind, stack, paths / fields, ops, pool (hex)."""
        if self._desc is None:
            n = lib().dk_program_describe(self._h, None, 0)
            buf = C.create_string_buffer(n + 1)
            lib().dk_program_describe(self._h, buf, n + 1)
            self._desc = json.loads(buf.raw[:n].decode("utf-8"))
        return self._desc

    @property
    def paths(self):
        """Skipping: the stats paths the program reads (tuples of names), in program order."""
        return [tuple(p["path"]) for p in self.describe().get("paths", [])]

    def close(self):
        if self._h:
            lib().dk_program_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _raise(rc, unsupported_cls):
    msg = lib().dk_last_error().decode("utf-8", "replace")
    if rc == STATUS_UNSUPPORTED_EXPRESSION:
        from .skipping import UnsupportedExpression
        raise UnsupportedExpression(msg)
    raise unsupported_cls(msg)


# ---- JSON of Kernel expressions --------------------------------------------------------------------
def literal_json(value, type_name: str) -> dict:
    """{"lit": <value>, "type": <Kernel type>} with exact encodings (floats as IEEE bits)."""
    t = type_name
    if value is None:
        return {"lit": None, "type": t}
    if t == "float":
        return {"lit": "0x%08x" % struct.unpack("<I", struct.pack("<f", float(value)))[0], "type": t}
    if t == "double":
        return {"lit": "0x%016x" % struct.unpack("<Q", struct.pack("<d", float(value)))[0], "type": t}
    if t.startswith("decimal"):
        return {"lit": str(Decimal(value)), "type": t}
    if t == "boolean":
        return {"lit": bool(value), "type": t}
    if t == "string":
        return {"lit": str(value), "type": t}
    if t == "binary":
        return {"lit": bytes(value).hex(), "type": t}
    return {"lit": int(value), "type": t}


def _expr_json(e) -> dict:
    if isinstance(e, Column):
        return {"col": list(e.names)}
    if isinstance(e, Literal):
        return literal_json(e.value, e.type)
    if isinstance(e, Predicate):
        return {"op": e.name, "args": [_expr_json(c) for c in e.children]}
    raise TypeError("not a Kernel expression: %r" % (e,))


def skipping_node_json(node) -> dict:
    """A constructed skipping predicate (skipping.construct's tuples) as Kernel expression JSON:
    stats columns, typed literals, TIMEADD(max, 1 ms) (StatsSchemaHelper.getMaxColumn :140-161)."""
    k = node[0]
    if k in ("AND", "OR"):
        return {"op": k, "args": [skipping_node_json(node[1]), skipping_node_json(node[2])]}
    if k == "stat":
        return {"col": list(node[1])}
    if k == "lit":
        return literal_json(node[1], node[2])
    if k == "timeadd":
        return {"op": "TIMEADD", "args": [skipping_node_json(node[1]), {"lit": 1, "type": "long"}]}
    return {"op": k, "args": [skipping_node_json(node[1]), skipping_node_json(node[2])]}


def pruned_stats_schema(node, leaves) -> dict:
    """StructType JSON of the stats fields the predicate references (DataSkippingUtils.pruneStatsSchema):
    numRecords / nullCount.* are long, minValues / maxValues.* take the column's type."""
    from . import skipping as sk
    root = {}
    for path in sk.referenced_stats(node):
        t = sk.operand_type(("stat", path), leaves)
        d = root
        for comp in path[:-1]:
            d = d.setdefault(comp, {})
        d[path[-1]] = t

    def struct_of(d):
        return {"type": "struct", "fields": [
            {"name": k, "type": struct_of(v) if isinstance(v, dict) else v, "nullable": True, "metadata": {}}
            for k, v in d.items()]}
    return struct_of(root)


def compile_skipping(node, leaves) -> Program:
    """dk_skip_compile of a constructed skipping predicate, as ScanImpl hands it to
    getPredicateEvaluator(prunedStatsSchema, =(COALESCE(skip, true), ALWAYS_TRUE))."""
    from .skipping import UnsupportedSkipping
    pred = {"op": "=", "args": [{"op": "COALESCE", "args": [skipping_node_json(node), {"lit": True, "type": "boolean"}]},
                                {"op": "ALWAYS_TRUE", "args": []}]}
    schema = pruned_stats_schema(node, leaves)
    h = C.c_void_p()
    rc = lib().dk_skip_compile(json.dumps(schema).encode(), json.dumps(pred).encode(), C.byref(h))
    if rc:
        _raise(rc, UnsupportedSkipping)
    return Program(h)


def rewrite_partition_predicate(pred, fields):
    """PartitionUtils.rewritePartitionPredicateOnScanFileSchema (PartitionUtils.java:324-358): a
    partition column becomes element_at(add.partitionValues, <physical name>), inside
    partition_value(.., <type>) unless it is a string; as JSON."""
    def rw(e):
        if isinstance(e, Column):
            name = e.names[0].lower()
            if name not in fields:
                raise ValueError("%s is not present in metadata" % e.names[0])     # PartitionUtils.java:340-343
            t, phys = fields[name]
            ea = {"op": "ELEMENT_AT", "args": [{"col": ["add", "partitionValues"]}, {"lit": phys, "type": "string"}]}
            return ea if t == "string" else {"op": "PARTITION_VALUE", "type": t, "args": [ea]}
        if isinstance(e, Literal):
            return literal_json(e.value, e.type)
        if isinstance(e, Predicate):
            return {"op": e.name, "args": [rw(c) for c in e.children]}
        raise TypeError("not a Kernel expression: %r" % (e,))
    return rw(pred)


def compile_partition(pred, fields) -> Program:
    """dk_part_compile of the rewritten partition predicate (ScanImpl.applyPartitionPruning)."""
    from .partitions import UnsupportedPartitionFilter
    j = rewrite_partition_predicate(pred, fields)
    h = C.c_void_p()
    rc = lib().dk_part_compile(json.dumps(j).encode(), C.byref(h))
    if rc:
        _raise(rc, UnsupportedPartitionFilter)
    return Program(h)


def check_status(rc):
    if rc != 0:
        raise DkError(lib().dk_last_error().decode("utf-8", "replace"))
