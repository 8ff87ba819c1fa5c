"""CPU ORACLE (test infrastructure only) for checkpoint row-group pruning: the checkpoint predicate
ActionsIterator hands the ParquetHandler for multi-part checkpoint parts and V2 sidecars
(kernel-api/.../internal/replay/ActionsIterator.java:336-351; classic and V2 top-level files get
OR(predicate, sidecar IS NOT NULL), which never converts, :175-226), i.e. the partition filter
rewritten onto add.partitionValues_parsed.<physical name> (PartitionUtils.java:275-303).

  ParquetFilterUtils.toParquetFilter (kernel-defaults/.../internal/parquet/ParquetFilterUtils.java:
      63-440): comparators need a column and a non-null literal; a literal on the left is swapped
      with the operator kept; canUseLiteral decides the literal / column type pairs; AND keeps a
      convertible side, OR needs both, NOT wraps; IS_NULL / IS_NOT_NULL -> eq / notEq(null);
      anything else, or a column the file lacks, converts to nothing.
  parquet-mr 1.12.3 (third-party, not in /root/reference; restated from its published source):
      FilterCompat.get runs LogicalInverseRewriter (NOT pushed into the leaves); StatisticsFilter
      drops a row group when the statistics prove no row matches (eq: value outside [min, max] or
      all nulls; eq(null): no nulls; notEq(null): all nulls; notEq(v): no nulls and min = max = v;
      lt: min >= v; ltEq: min > v; gt: max <= v; gtEq: max < v; AND: either side; OR: both sides);
      float / double statistics with a NaN carry no min / max, and a +0.0 min / -0.0 max widen to
      -0.0 / +0.0. Comparisons: signed integers, Float.compare / Double.compare, unsigned bytes.
The footer statistics come from pyarrow's metadata reader (min / max decoded to Python values).
Nothing here is used by the product path.
"""
from __future__ import annotations

import math

_INTS = ("long", "integer", "short", "byte", "date")


def _can_use_literal(lit_type, value, col):
    """ParquetFilterUtils.canUseLiteral (:92-133) for a pyarrow ColumnSchema."""
    phys = col.physical_type
    lt = col.logical_type.type if col.logical_type is not None else "NONE"
    if phys == "BOOLEAN":
        return lit_type == "boolean"
    if phys == "INT32":
        integer = lit_type in ("byte", "short", "integer", "date") or (
            lit_type == "long" and -(1 << 31) <= value < (1 << 31))
        if not integer:
            return False
        if lt == "NONE" or lt == "DATE":
            return True
        return lt == "INT" and col.logical_type.bit_width <= 32
    if phys == "INT64":
        if lit_type not in _INTS:
            return False
        return lt == "NONE" or (lt == "INT" and col.logical_type.bit_width <= 64)
    if phys == "FLOAT":
        return lit_type == "float"
    if phys == "DOUBLE":
        return lit_type == "double"
    if phys == "BYTE_ARRAY":
        return lit_type == "string" and lt in ("NONE", "STRING")
    return False


def _convert(pred, fields, cols):
    """Optional parquet-mr filter tree: ("eq"|"noteq"|"lt"|"lteq"|"gt"|"gteq", path, value, type)
    or ("and"|"or", a, b) or ("not", a); None = not convertible."""
    kind = type(pred).__name__
    if kind != "Predicate":
        return None
    n = pred.name.lower()
    c = pred.children

    def path_of(col):
        name = col.names[0].lower()
        if name not in fields:
            raise ValueError("%s is not present in metadata" % col.names[0])
        return "add.partitionValues_parsed." + fields[name][1]
    if n in ("=", "<", "<=", ">", ">="):
        a, b = c
        if type(a).__name__ == "Literal" and type(b).__name__ == "Column":
            a, b = b, a                                   # swapped, operator kept (:158-162)
        if type(a).__name__ != "Column" or type(b).__name__ != "Literal":
            return None
        p = path_of(a)
        if p not in cols or b.value is None or not _can_use_literal(b.type, b.value, cols[p]):
            return None
        phys = cols[p].physical_type
        if phys == "BOOLEAN" and n != "=":
            return None
        v = b.value
        if phys == "FLOAT":
            import struct
            v = struct.unpack("<f", struct.pack("<f", float(v)))[0]
        elif phys == "BYTE_ARRAY":
            v = v.encode("utf-8")
        return ({"=": "eq", "<": "lt", "<=": "lteq", ">": "gt", ">=": "gteq"}[n], p, v, phys)
    if n in ("and", "or"):
        la, lb = _convert(c[0], fields, cols), _convert(c[1], fields, cols)
        if la is not None and lb is not None:
            return (n, la, lb)
        return (la if la is not None else lb) if n == "and" else None
    if n == "not":
        x = _convert(c[0], fields, cols)
        return None if x is None else ("not", x)
    if n in ("is_null", "is_not_null"):
        a = c[0]
        if type(a).__name__ != "Column":
            return None
        p = path_of(a)
        if p not in cols:
            return None
        return ("eq" if n == "is_null" else "noteq", p, None, cols[p].physical_type)
    for ch in c:
        if type(ch).__name__ == "Column":
            path_of(ch)
    return None


_INVERT = {"eq": "noteq", "noteq": "eq", "lt": "gteq", "lteq": "gt", "gt": "lteq", "gteq": "lt"}


def _invert(node):
    """LogicalInverter."""
    if node[0] == "and":
        return ("or", _invert(node[1]), _invert(node[2]))
    if node[0] == "or":
        return ("and", _invert(node[1]), _invert(node[2]))
    if node[0] == "not":
        return node[1]
    return (_INVERT[node[0]],) + node[1:]


def _rewrite(node):
    """LogicalInverseRewriter: remove every NOT."""
    if node[0] in ("and", "or"):
        return (node[0], _rewrite(node[1]), _rewrite(node[2]))
    if node[0] == "not":
        return _rewrite(_invert(node[1]))
    return node


def _jcmp(a, b, phys):
    if phys in ("FLOAT", "DOUBLE"):
        an, bn = a != a, b != b
        if an or bn:
            return (an > bn) - (an < bn)
        if a == b == 0:
            sa, sb = math.copysign(1, a), math.copysign(1, b)
            return (sa > sb) - (sa < sb)
    return (a > b) - (a < b)


def _stats(chunk, phys):
    """(has_min_max, min, max, nulls_set, nulls, value_count) as parquet-mr's Statistics reads them."""
    st = chunk.statistics if chunk.is_stats_set else None
    if st is None:
        return False, None, None, False, 0, chunk.num_values
    has = st.has_min_max
    mn, mx = (st.min, st.max) if has else (None, None)
    if has and phys in ("FLOAT", "DOUBLE"):
        if mn != mn or mx != mx:
            has = False
        else:
            if mn == 0:
                mn = -0.0
            if mx == 0:
                mx = 0.0
    if has and phys == "BYTE_ARRAY":
        mn = mn if isinstance(mn, bytes) else str(mn).encode("utf-8")
        mx = mx if isinstance(mx, bytes) else str(mx).encode("utf-8")
    if has and phys == "BOOLEAN":
        mn, mx = bool(mn), bool(mx)
    nulls_set = st.has_null_count
    return has, mn, mx, nulls_set, st.null_count if nulls_set else 0, chunk.num_values


def _can_drop(node, rg, col_index):
    op = node[0]
    if op == "and":
        return _can_drop(node[1], rg, col_index) or _can_drop(node[2], rg, col_index)
    if op == "or":
        return _can_drop(node[1], rg, col_index) and _can_drop(node[2], rg, col_index)
    _, path, v, phys = node
    has, mn, mx, nulls_set, nulls, count = _stats(rg.column(col_index[path]), phys)
    if not has and not nulls_set:
        return False                                      # empty statistics
    all_nulls = nulls_set and nulls == count
    if op == "eq":
        if v is None:
            return nulls_set and nulls == 0
        if all_nulls:
            return True
        return has and (_jcmp(mn, v, phys) > 0 or _jcmp(mx, v, phys) < 0)
    if op == "noteq":
        if v is None:
            return all_nulls
        if nulls_set and nulls > 0:
            return False
        return has and _jcmp(mn, v, phys) == 0 and _jcmp(mx, v, phys) == 0
    if all_nulls:
        return True
    if not has:
        return False
    if op == "lt":
        return _jcmp(mn, v, phys) >= 0
    if op == "lteq":
        return _jcmp(mn, v, phys) > 0
    if op == "gt":
        return _jcmp(mx, v, phys) <= 0
    return _jcmp(mx, v, phys) < 0


def surviving_row_groups(path, pred, fields):
    """keep flag per row group of the Parquet file at `path`."""
    import pyarrow.parquet as pq
    md = pq.ParquetFile(path).metadata
    schema = md.schema
    cols = {schema.column(i).path: schema.column(i) for i in range(md.num_columns)}
    col_index = {schema.column(i).path: i for i in range(md.num_columns)}
    f = _convert(pred, fields, cols)
    if f is None:
        return [True] * md.num_row_groups
    f = _rewrite(f)
    return [not _can_drop(f, md.row_group(g), col_index) for g in range(md.num_row_groups)]
