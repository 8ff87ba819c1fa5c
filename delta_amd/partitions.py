"""Partition-pruning planning (host side): the partition part of a scan filter
(PartitionUtils.splitMetadataAndDataPredicates, delta_amd/skipping.split_filters) rewritten over the
scan file's partitionValues map (PartitionUtils.rewritePartitionPredicateOnScanFileSchema,
kernel-api/.../internal/util/PartitionUtils.java:324-358: a partition column becomes
element_at(add.partitionValues, <physical name>), deserialized to the column's type unless it is a
string) and compiled to the postfix program k_part_eval runs (ScanImpl.applyPartitionPruning,
ScanImpl.java:247-294).

Supported: partition columns of type string, long, integer, short, byte, date (values through
java.sql.Date.valueOf, PartitionValueEvaluator.java:72-73), decimal (new BigDecimal(text), :112-113,
compared with compareTo); literals of a matching kind (string with string, any integral with
integral, date with date, decimal with decimal, or null); =, <, <=, >, >=, IS NOT DISTINCT
FROM, IS_NULL, IS_NOT_NULL, NOT, AND, OR. Anything else raises UnsupportedPartitionFilter, so an
accepted filter is evaluated exactly as the reference evaluates it.
"""
from __future__ import annotations

import json

from .expressions import Column, Literal, Predicate

PT = {"long": 0, "integer": 1, "short": 2, "byte": 3, "string": 4, "date": 5, "decimal": 6}
INTEGRAL = {"long", "integer", "short", "byte"}
(PO_FIELD, PO_LIT_INT, PO_LIT_STR, PO_LIT_NULL, PO_LT, PO_LE, PO_GT, PO_GE, PO_EQ, PO_NSEQ, PO_ISNULL,
 PO_ISNOTNULL, PO_NOT, PO_AND, PO_OR, PO_LIT_DEC) = range(16)
CMP = {"<": PO_LT, "<=": PO_LE, ">": PO_GT, ">=": PO_GE, "=": PO_EQ, "IS NOT DISTINCT FROM": PO_NSEQ}
MAX_FIELDS, MAX_OPS, MAX_STACK, POOL = 8, 64, 16, 1024


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


def compile_program(pred: Predicate, fields: dict):
    """(field list [(pool offset, length, type code)], ops [(op, arg, lit)], pool bytes)."""
    used, ops = [], []
    pool = bytearray()

    def field(col: Column):
        name = col.names[0].lower()
        if len(col.names) != 1 or name not in fields:
            raise ValueError("%s is not present in metadata" % col.names[0])   # PartitionUtils.java:340-343
        t, phys = fields[name]
        if t.startswith("decimal"):
            t = "decimal"
        if t not in PT:
            raise UnsupportedPartitionFilter("partition pruning on %s column %s is not supported by this engine build"
                                             % (t, col.names[0]))
        if (phys, t) not in used:
            used.append((phys, t))
        return used.index((phys, t)), t

    def operand(node):
        """emit an operand; returns (kind: 'string', 'integral', 'date', 'decimal' or None for a null
        literal, Kernel type name)."""
        if isinstance(node, Column):
            k, t = field(node)
            ops.append((PO_FIELD, k, 0))
            return (t if t in ("string", "date", "decimal") else "integral"), fields[node.names[0].lower()][0]
        if isinstance(node, Literal):
            return operand_lit(node), node.type
        raise UnsupportedPartitionFilter("partition pruning on expression %r is not supported" % (node,))

    def operand_lit(node):
        if isinstance(node, Literal):
            if node.value is None:
                ops.append((PO_LIT_NULL, 0, 0))
                return None
            if node.type == "string":
                b = str(node.value).encode("utf-8")
                ops.append((PO_LIT_STR, len(b), len(pool)))
                pool.extend(b)
                return "string"
            if node.type.startswith("decimal"):                # BigDecimal text, compareTo on the GPU
                from decimal import Decimal
                v = Decimal(node.value)
                if not v.is_finite():
                    raise UnsupportedPartitionFilter("decimal literal %s is not finite" % v)
                b = str(v).encode("ascii")
                ops.append((PO_LIT_DEC, len(b), len(pool)))
                pool.extend(b)
                return "decimal"
            if node.type in INTEGRAL | {"date"} and isinstance(node.value, int) and not isinstance(node.value, bool):
                ops.append((PO_LIT_INT, 0, int(node.value)))   # a date literal is its epoch day
                return "date" if node.type == "date" else "integral"
            raise UnsupportedPartitionFilter("partition pruning with a %s literal is not supported" % node.type)
        raise UnsupportedPartitionFilter("partition pruning on expression %r is not supported" % (node,))

    def pred_(node):
        if not isinstance(node, Predicate):
            raise UnsupportedPartitionFilter("not a predicate: %r" % (node,))
        n = node.name.upper()
        c = node.children
        if n in ("AND", "OR"):
            pred_(c[0])
            pred_(c[1])
            ops.append((PO_AND if n == "AND" else PO_OR, 0, 0))
        elif n == "NOT":
            pred_(c[0])
            ops.append((PO_NOT, 0, 0))
        elif n in ("IS_NULL", "IS_NOT_NULL"):
            operand(c[0])
            ops.append((PO_ISNULL if n == "IS_NULL" else PO_ISNOTNULL, 0, 0))
        elif n in CMP:
            (ka, ta), (kb, tb) = operand(c[0]), operand(c[1])
            # DefaultExpressionEvaluator.transformBinaryComparator (:337-354): differently typed
            # operands need an ImplicitCastExpression up-cast, otherwise the evaluator throws
            from .skipping import UnsupportedExpression, comparable
            if not comparable(ta, tb):
                raise UnsupportedExpression(
                    "Unsupported expression: %s: operands are of different types which are not comparable: "
                    "left type=%s, right type=%s" % (n, ta, tb))
            if ka is not None and kb is not None and ka != kb:
                raise UnsupportedPartitionFilter("comparison of %s with %s is not supported" % (ka, kb))
            ops.append((CMP[n], 0, 0))
        else:
            raise UnsupportedPartitionFilter("partition predicate %s is not supported by this engine build" % n)

    pred_(pred)
    flist = []
    for phys, t in used:
        b = phys.encode("utf-8")
        flist.append((len(pool), len(b), PT[t]))
        pool.extend(b)
    if len(used) > MAX_FIELDS or len(ops) > MAX_OPS or len(pool) > POOL or _depth(ops) > MAX_STACK:
        raise UnsupportedPartitionFilter("partition filter is too large for the device evaluator")
    return flist, ops, bytes(pool)


def _depth(ops):
    d = hi = 0
    for op, _, _ in ops:
        if op in (PO_FIELD, PO_LIT_INT, PO_LIT_STR, PO_LIT_NULL, PO_LIT_DEC):
            d += 1
        elif op not in (PO_ISNULL, PO_ISNOTNULL, PO_NOT):
            d -= 1
        hi = max(hi, d)
    return hi


def pack(program, struct_type):
    """Fill a dk_part_program ctypes struct (include/dkgpu.h)."""
    flist, ops, pool = program
    p = struct_type()
    p.n_fields = len(flist)
    for i, (off, ln, t) in enumerate(flist):
        p.name_off[i], p.name_len[i], p.field_type[i] = off, ln, t
    p.n_ops = len(ops)
    for k, (op, arg, lit) in enumerate(ops):
        p.op[k], p.arg[k], p.lit[k] = op, arg, lit
    p.pool = pool
    return p
