"""Partition-pruning planning (host side): the partition part of a scan filter
(PartitionUtils.splitMetadataAndDataPredicates, delta_amd/skipping.split_filters) rewritten over the
scan file's partitionValues map (PartitionUtils.rewritePartitionPredicateOnScanFileSchema,
kernel-api/.../internal/util/PartitionUtils.java:324-358: a partition column becomes
element_at(add.partitionValues, <physical name>), deserialized to the column's type unless it is a
string) and compiled to the postfix program k_part_eval runs (ScanImpl.applyPartitionPruning,
ScanImpl.java:247-294).

Supported: partition columns of type string, long, integer, short, byte, date (values through
java.sql.Date.valueOf, PartitionValueEvaluator.java:72-73), decimal (new BigDecimal(text), :112-113,
compared with compareTo), boolean (Boolean.parseBoolean), float / double (Float.parseFloat /
Double.parseDouble, compared exactly through delta_amd/binfloat.py thresholds with Float.compare
semantics and ImplicitCastExpression widening of integral operands), timestamp / timestamp_ntz
(java.sql.Timestamp.valueOf -> InternalUtils.microsSinceEpoch, read as UTC); literals of a matching
kind (or null); =, <, <=, >, >=, IS NOT DISTINCT FROM, IS_NULL, IS_NOT_NULL, NOT, AND, OR. A float
comparison needs a column on one side and a literal on the other. Anything else raises
UnsupportedPartitionFilter, so an accepted filter is evaluated exactly as the reference evaluates it.
"""
from __future__ import annotations

import json

from ._lib import put_bytes
from .expressions import Column, Literal, Predicate

PT = {"long": 0, "integer": 1, "short": 2, "byte": 3, "string": 4, "date": 5, "decimal": 6, "boolean": 7,
      "float": 8, "double": 9, "timestamp": 10, "timestamp_ntz": 10}
INTEGRAL = {"long", "integer", "short", "byte"}
FLOATS = ("float", "double")
(PO_FIELD, PO_LIT_INT, PO_LIT_STR, PO_LIT_NULL, PO_LT, PO_LE, PO_GT, PO_GE, PO_EQ, PO_NSEQ, PO_ISNULL,
 PO_ISNOTNULL, PO_NOT, PO_AND, PO_OR, PO_LIT_DEC, PO_FCMP) = range(17)
REVERSE = {"=": "=", "<": ">", "<=": ">=", ">": "<", ">=": "<=", "IS NOT DISTINCT FROM": "IS NOT DISTINCT FROM"}
_KIND = {"string": "string", "date": "date", "decimal": "decimal", "boolean": "boolean", "timestamp": "timestamp",
         "timestamp_ntz": "timestamp", "float": "float", "double": "float"}
CMP = {"<": PO_LT, "<=": PO_LE, ">": PO_GT, ">=": PO_GE, "=": PO_EQ, "IS NOT DISTINCT FROM": PO_NSEQ}
MAX_FIELDS, MAX_OPS, MAX_STACK, POOL = 8, 64, 16, 4096


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
        t = "timestamp" if t == "timestamp_ntz" else t         # one parse for both (Timestamp.valueOf)
        if (phys, t) not in used:
            used.append((phys, t))
        return used.index((phys, t)), t

    def operand(node):
        """emit an operand; returns (kind: 'string', 'integral', 'date', 'decimal' or None for a null
        literal, Kernel type name)."""
        if isinstance(node, Column):
            k, t = field(node)
            ops.append((PO_FIELD, k, 0))
            return _KIND.get(t, "integral"), fields[node.names[0].lower()][0]
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
            if node.type == "boolean":
                ops.append((PO_LIT_INT, 0, int(bool(node.value))))
                return "boolean"
            if node.type in INTEGRAL | {"date", "timestamp", "timestamp_ntz"} and isinstance(node.value, int) \
                    and not isinstance(node.value, bool):
                ops.append((PO_LIT_INT, 0, int(node.value)))   # dates: epoch days, timestamps: micros
                return _KIND.get(node.type, "integral")
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
        elif n in CMP and any(_type(x) in FLOATS for x in c):
            float_cmp(n, c[0], c[1])
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

    def _type(x):
        if isinstance(x, Column) and len(x.names) == 1 and x.names[0].lower() in fields:
            return fields[x.names[0].lower()][0]
        return x.type if isinstance(x, Literal) else None

    def float_cmp(n, left, right):
        """column <op> literal in float / double (either side float-typed): planned exactly by
        binfloat.plan; integral columns widened to float get integer bounds, float columns PO_FCMP."""
        from . import binfloat
        from .skipping import LONG_MAX, LONG_MIN, UnsupportedExpression, _UP_CAST, comparable
        if isinstance(left, Literal) and isinstance(right, Column):
            left, right, n = right, left, REVERSE[n]
        if not (isinstance(left, Column) and isinstance(right, Literal)):
            raise UnsupportedPartitionFilter("float partition comparison needs a column and a literal: %r, %r"
                                             % (left, right))
        ct, lt = _type(left), right.type
        if not comparable(ct, lt):
            raise UnsupportedExpression(
                "Unsupported expression: %s: operands are of different types which are not comparable: "
                "left type=%s, right type=%s" % (n, ct, lt))
        if ct not in FLOATS and ct not in INTEGRAL:
            raise UnsupportedPartitionFilter("comparison of %s with %s is not supported" % (ct, lt))
        if right.value is None:                              # null literal: generic null semantics
            operand(left)
            ops.append((PO_LIT_NULL, 0, 0))
            ops.append((CMP[n], 0, 0))
            return
        cmp_t = ct if ct == lt else (lt if lt in _UP_CAST.get(ct, ()) else ct)
        value_fmt = ct if ct in FLOATS else cmp_t
        op = "=" if n == "IS NOT DISTINCT FROM" else n
        conds, (r_nan, r_pinf, r_ninf) = binfloat.plan(op, right.value, lt, value_fmt, cmp_t)
        terms = 0
        if n == "IS NOT DISTINCT FROM":                      # null-safe: a null column is false
            operand(left)
            ops.append((PO_ISNOTNULL, 0, 0))
            terms += 1
        if ct not in FLOATS:
            b = binfloat.integral_bounds(conds)
            if b is None:
                parts = [(PO_LT, LONG_MIN)]
            else:
                parts = ([(PO_GE, b[0])] if b[0] > LONG_MIN else []) + ([(PO_LE, b[1])] if b[1] < LONG_MAX else [])
                parts = parts or [(PO_GE, LONG_MIN)]
            for cop, v in parts:
                operand(left)
                ops.append((PO_LIT_INT, 0, int(v)))
                ops.append((cop, 0, 0))
                terms += 1
                if terms > 1:
                    ops.append((PO_AND, 0, 0))
            return
        flags = (int(r_nan) << 4) | (int(r_pinf) << 5) | (int(r_ninf) << 6)
        from .skipping import FC_ALL, FC_NONE, _FC_MODE
        for cnd in conds:
            operand(left)
            if cnd in (binfloat.ALL, binfloat.NONE):
                ops.append((PO_FCMP, flags | (FC_ALL if cnd == binfloat.ALL else FC_NONE), (0, 0)))
            else:
                text = binfloat.decimal_text(cnd[1], short=True).encode("ascii")
                ops.append((PO_FCMP, flags | _FC_MODE[cnd[0]], (len(pool), len(text))))
                pool.extend(text)
            terms += 1
            if terms > 1:
                ops.append((PO_AND, 0, 0))

    pred_(pred)
    ops[:] = [(o, a, (l[0] | (l[1] << 32)) if o == PO_FCMP else l) for o, a, l in ops]
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
        elif op not in (PO_ISNULL, PO_ISNOTNULL, PO_NOT, PO_FCMP):
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
    put_bytes(p, "pool", bytes(pool))
    return p


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
    if len(cols) > 8 or len(ops) > 64:
        raise UnsupportedPartitionFilter("partition filter is too large for checkpoint row-group pruning")
    return cols, ops, bytes(pool)


def pack_row_group_filter(program, struct_type):
    cols, ops, pool = program
    f = struct_type()
    pool = bytearray(pool)
    f.n_cols = len(cols)
    for i, c in enumerate(cols):
        b = c.encode("utf-8")
        f.col_off[i], f.col_len[i] = len(pool), len(b)
        pool.extend(b)
    if len(pool) > 2048:
        raise UnsupportedPartitionFilter("partition filter literals exceed 2 KiB for row-group pruning")
    f.n_ops = len(ops)
    for k, (op, arg, lit) in enumerate(ops):
        f.op[k], f.arg[k], f.lit[k] = op, arg, lit
    put_bytes(f, "pool", bytes(pool))
    return f
