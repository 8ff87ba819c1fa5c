"""Data-skipping planning (host side of K11), restating
kernel-api/.../internal/skipping/DataSkippingUtils.java:74-456 and StatsSchemaHelper.java:71-232.
The skipping predicate it constructs is compiled behind the C ABI (delta_amd/programs.py ->
dk_skip_compile) into the postfix program the GPU evaluates per scan-file row over the row's
``add.stats`` JSON or ``add.stats_parsed`` columns (k_stats_eval / k_stats_parsed;
ScanImpl.applyDataSkipping, ScanImpl.java:304-352).

A skipping predicate node is one of
    ("AND", a, b) / ("OR", a, b)
    (cmp, left, right)   cmp in "<", "<=", ">", ">=", "="; operands ("stat", path) or ("lit", int)
where path is a tuple like ("maxValues", "id") or ("numRecords",). IS NOT DISTINCT FROM is rewritten
as in the reference (rewriteEqualNullSafe, :528-534).
"""
from __future__ import annotations

import json

from decimal import Decimal as _Decimal

from .expressions import ALWAYS_TRUE, Column, Literal, Predicate

MIN, MAX, NULL_COUNT, NUM_RECORDS = "minValues", "maxValues", "nullCount", "numRecords"
SKIPPING_ELIGIBLE = {"byte", "short", "integer", "long", "float", "double", "date", "timestamp",
                     "timestamp_ntz", "string"}          # StatsSchemaHelper.java:209-222 (+ decimal)
GPU_TYPES = {"byte", "short", "integer", "long", "date", "string", "timestamp", "decimal", "timestamp_ntz",
             "float", "double"}                          # stats value types k_stats_eval decodes
REVERSE = {"=": "=", "<": ">", "<=": ">=", ">": "<", ">=": "<=",
           "IS NOT DISTINCT FROM": "IS NOT DISTINCT FROM"}   # DataSkippingUtils.java:346-356
NOT_CMP = {"<": ">=", "<=": ">", ">": "<=", ">=": "<"}        # :430-441


class UnsupportedExpression(RuntimeError):
    """The reference's expression handler throws for this predicate (KernelException
    "Unsupported expression"); the scan fails the same way."""


class UnsupportedSkipping(RuntimeError):
    pass


def data_schema_leaves(schema_string: str, partition_columns=()) -> dict:
    """Logical leaf column -> (type name, physical column) over the table's data schema (partition
    columns excluded, Metadata.getDataSchema; StatsSchemaHelper.getLogicalToPhysicalColumnAndDataType
    :297-319; physical names from delta.columnMapping.physicalName, ColumnMapping.getPhysicalName)."""
    schema = json.loads(schema_string)
    parts = {p.lower() for p in partition_columns}
    out = {}

    def walk(fields, prefix, phys):
        for f in fields:
            t = f["type"]
            name = prefix + (f["name"],)
            pname = phys + ((f.get("metadata") or {}).get("delta.columnMapping.physicalName", f["name"]),)
            if not prefix and f["name"].lower() in parts:
                continue
            if isinstance(t, dict) and t.get("type") == "struct":
                walk(t["fields"], name, pname)
            elif isinstance(t, str):
                out[name] = (t, pname)
            else:
                out[name] = (t.get("type", "complex") if isinstance(t, dict) else str(t), pname)
    walk(schema["fields"], (), ())
    return out


def _refs_non_partition(children, parts) -> bool:
    """PartitionUtils.hasNonPartitionColumns (util/PartitionUtils.java:398-415)."""
    for ch in children:
        if isinstance(ch, Column):
            if len(ch.names) != 1 or ch.names[0].lower() not in parts:
                return True
        elif isinstance(ch, Predicate) and _refs_non_partition(ch.children, parts):
            return True
    return False


def _and(a, b):
    """combineWithAndOp (PartitionUtils.java:417-430)."""
    if a.name.upper() == "ALWAYS_FALSE" or b.name.upper() == "ALWAYS_FALSE":
        return Predicate("ALWAYS_FALSE")
    if a.name.upper() == "ALWAYS_TRUE":
        return b
    if b.name.upper() == "ALWAYS_TRUE":
        return a
    return Predicate("AND", a, b)


def split_filters(pred: Predicate, partition_columns=()):
    """(partition predicate, data predicate), each None when ALWAYS_TRUE
    (PartitionUtils.splitMetadataAndDataPredicates :242-263; ScanImpl.removeAlwaysTrue :236-245)."""
    parts = {p.lower() for p in partition_columns}

    def split(p):
        if p.name.upper() == "AND":
            l1, l2 = split(p.children[0])
            r1, r2 = split(p.children[1])
            return _and(l1, r1), _and(l2, r2)
        if _refs_non_partition(p.children, parts):
            return ALWAYS_TRUE, p
        return p, ALWAYS_TRUE
    a, b = split(pred)
    drop = lambda x: None if x.name.upper() == "ALWAYS_TRUE" else x  # noqa: E731
    return drop(a), drop(b)


def _eligible_minmax(leaves, col):
    t = leaves[col.names][0] if col.names in leaves else None
    return t is not None and (t in SKIPPING_ELIGIBLE or t.startswith("decimal"))


def _eligible_literal(lit):                               # isSkippingEligibleLiteral (StatsSchemaHelper :50-52)
    return lit.type in SKIPPING_ELIGIBLE or lit.type.startswith("decimal")


def construct(pred: Predicate, leaves: dict):
    """constructDataSkippingFilter (DataSkippingUtils.java:156-283); None = no skipping filter."""
    n = pred.name.upper()
    c = pred.children
    if n == "AND":                                                              # :178-190
        a, b = construct(c[0], leaves), construct(c[1], leaves)
        if a and b:
            return ("AND", a, b)
        return a or b
    if n == "OR":                                                               # :204-213
        a, b = construct(c[0], leaves), construct(c[1], leaves)
        return ("OR", a, b) if a and b else None
    if n == "IS_NOT_NULL":                                                      # :216-235
        if isinstance(c[0], Column) and c[0].names in leaves:
            return ("<", ("stat", (NULL_COUNT,) + leaves[c[0].names][1]), ("stat", (NUM_RECORDS,)))
        return None
    if n == "IS_NULL":                                                          # :240-252
        if isinstance(c[0], Column) and c[0].names in leaves:
            return (">", ("stat", (NULL_COUNT,) + leaves[c[0].names][1]), ("lit", 0, "long"))
        return None
    if n in ("=", "<", "<=", ">", ">=", "IS NOT DISTINCT FROM"):               # :254-274
        left, right = c
        if isinstance(left, Column) and isinstance(right, Literal):
            if _eligible_minmax(leaves, left) and _eligible_literal(right):
                return _comparator(n, left, right, leaves)
            return None
        if isinstance(right, Column) and isinstance(left, Literal):
            return construct(Predicate(REVERSE[n], right, left), leaves)
        return None
    if n == "NOT":                                                              # :276-278
        return _construct_not(c[0], leaves)
    return None


def _comparator(n, col, lit, leaves):
    """constructComparatorDataSkippingFilters (:286-331)."""
    mn = ("stat", (MIN,) + leaves[col.names][1])
    mx = _max(col, leaves)
    v = ("lit", lit.value, lit.type)
    if n == "=":
        return ("AND", ("<=", mn, v), (">=", mx, v))
    if n == "<":
        return ("<", mn, v)
    if n == "<=":
        return ("<=", mn, v)
    if n == ">":
        return (">", mx, v)
    if n == ">=":
        return (">=", mx, v)
    # IS NOT DISTINCT FROM (rewriteEqualNullSafe :528-534)
    if lit.value is None:
        return construct(Predicate("IS_NULL", col), leaves)
    return construct(Predicate("AND", Predicate("IS_NOT_NULL", col), Predicate("=", col, lit)), leaves)


def _max(col, leaves):
    t, phys = leaves[col.names]
    if t in ("timestamp", "timestamp_ntz"):              # getMaxColumn TIMEADD(+1 ms), StatsSchemaHelper :154-159
        return ("timeadd", ("stat", (MAX,) + phys))
    return ("stat", (MAX,) + phys)


def _construct_not(child: Predicate, leaves):
    """constructNotDataSkippingFilters (:366-487)."""
    n = child.name.upper()
    c = child.children
    if n == "AND":
        return construct(Predicate("OR", Predicate("NOT", c[0]), Predicate("NOT", c[1])), leaves)
    if n == "OR":
        return construct(Predicate("AND", Predicate("NOT", c[0]), Predicate("NOT", c[1])), leaves)
    if n == "IS_NOT_NULL":
        return construct(Predicate("IS_NULL", c[0]), leaves)
    if n == "IS_NULL":
        return construct(Predicate("IS_NOT_NULL", c[0]), leaves)
    if n in ("=", "IS NOT DISTINCT FROM"):
        # constructDataSkippingFiltersForNotEqual (:537-560): a literal on the left swaps sides; the
        # column must be min/max eligible and the literal eligible
        left, right = c
        if isinstance(right, Column) and isinstance(left, Literal):
            return _construct_not(Predicate(child.name, right, left), leaves)
        if not (isinstance(left, Column) and isinstance(right, Literal)
                and _eligible_minmax(leaves, left) and _eligible_literal(right)):
            return None
        if n == "=":                         # NOT(a = x) -> OR(min < x, max > x)
            v = ("lit", right.value, right.type)
            return ("OR", ("<", ("stat", (MIN,) + leaves[left.names][1]), v), (">", _max(left, leaves), v))
        # NOT(a <=> x) -> NOT(rewriteEqualNullSafe(a, x)) (:528-534)
        if right.value is None:
            return construct(Predicate("NOT", Predicate("IS_NULL", left)), leaves)
        return construct(Predicate("NOT", Predicate("AND", Predicate("IS_NOT_NULL", left),
                                                    Predicate("=", left, right))), leaves)
    if n in NOT_CMP:
        return construct(Predicate(NOT_CMP[n], c[0], c[1]), leaves)
    if n == "NOT":
        return construct(c[0], leaves)
    return None


def referenced_stats(node, out=None):
    out = [] if out is None else out
    if node[0] in ("AND", "OR"):
        referenced_stats(node[1], out)
        referenced_stats(node[2], out)
    elif node[0] == "stat":
        if node[1] not in out:
            out.append(node[1])
    elif node[0] == "timeadd":
        referenced_stats(node[1], out)
    elif node[0] != "lit":
        referenced_stats(node[1], out)
        referenced_stats(node[2], out)
    return out


# ---- stats types --------------------------------------------------------------------------------
# (the predicate is compiled behind the C ABI: delta_amd/programs.compile_skipping -> dk_skip_compile)
FLOATS = ("float", "double")
LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1
TYPE_CODE = {"long": 0, "integer": 1, "short": 2, "byte": 3, "date": 4, "string": 5, "timestamp": 6, "decimal": 7,
             "timestamp_ntz": 8, "float": 9, "double": 10}
_CMP = ("<", "<=", ">", ">=", "=")
# opcodes of a compiled skipping program (dk_device.h; dk_program_describe's "ops")
OP_STAT, OP_LIT, OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_AND, OP_OR, OP_LIT_STR, OP_TIMEADD, OP_LIT_DEC, OP_FCMP = range(13)
FC_LT, FC_LE, FC_GT, FC_GE, FC_ALL, FC_NONE = range(6)


def stat_type(path, leaves):
    """Type of a stats field: numRecords / nullCount.* are long (getNullCountSchema :255-273),
    min/max take the column's type."""
    if path[0] in (NUM_RECORDS, NULL_COUNT):
        return "long"
    for t, phys in leaves.values():
        if phys == path[1:]:
            return "decimal" if t.startswith("decimal") else t
    raise KeyError(path)


# ImplicitCastExpression.UP_CASTABLE_TYPE_TABLE (kernel-defaults/.../internal/expressions/
# ImplicitCastExpression.java:30-41, canCastTo :118-125)
_UP_CAST = {"byte": {"short", "integer", "long", "float", "double"}, "short": {"integer", "long", "float", "double"},
            "integer": {"long", "float", "double"}, "long": {"float", "double"}, "float": {"double"}}


def operand_type(n, leaves):
    """Kernel DataType name of a skipping-predicate operand (decimals keep precision and scale)."""
    if n[0] == "stat":
        if n[1][0] in (NUM_RECORDS, NULL_COUNT):
            return "long"
        for t, phys in leaves.values():
            if phys == n[1][1:]:
                return t
        raise KeyError(n[1])
    if n[0] == "lit":
        return n[2]
    if n[0] == "timeadd":
        return operand_type(n[1], leaves)
    return "boolean"


def comparable(lt, rt):
    """ImplicitCastExpression.canCastTo either way, or the same type."""
    return lt == rt or rt in _UP_CAST.get(lt, ()) or lt in _UP_CAST.get(rt, ())


def check_comparable(n, leaves):
    """DefaultExpressionEvaluator.transformBinaryComparator (DefaultExpressionEvaluator.java:337-354):
    operands of different types compare only after an implicit up-cast of one side; any other pair
    makes the evaluator throw (unsupportedExpressionException)."""
    lt, rt = operand_type(n[1], leaves), operand_type(n[2], leaves)
    if comparable(lt, rt):
        return
    raise UnsupportedExpression(
        "Unsupported expression: %s: operands are of different types which are not comparable: "
        "left type=%s, right type=%s" % (n[0], lt, rt))


def check_types(node, leaves):
    """Walk a constructed skipping predicate and apply check_comparable to every comparator."""
    if node is None:
        return
    if node[0] in ("AND", "OR"):
        check_types(node[1], leaves)
        check_types(node[2], leaves)
    elif node[0] in _CMP:
        check_comparable(node, leaves)
