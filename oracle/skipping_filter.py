"""CPU ORACLE (test infrastructure only): the data-skipping predicate the reference builds from a
scan's data filter, restated on its own so that the product planner (delta_amd/skipping.py) is
checked against it rather than shared with the oracle evaluator (oracle/skipping.py).

  DataSkippingUtils.constructDataSkippingFilter       kernel-api/.../internal/skipping/
                                                      DataSkippingUtils.java:156-283
  constructComparatorDataSkippingFilters              :286-331
  constructBinaryDataSkippingPredicate                :337-344
  REVERSE_COMPARATORS / reverseComparatorFilter       :346-363
  constructNotDataSkippingFilters                     :366-456
  rewriteEqualNullSafe                                :528-534
  constructDataSkippingFiltersForNotEqual             :537-560
  StatsSchemaHelper (eligibility, min / max / nullCount columns, TIMEADD(max, 1 ms) for timestamp
  and timestamp_ntz)                                  kernel-api/.../internal/skipping/
                                                      StatsSchemaHelper.java:50-232, 297-319
  DefaultExpressionEvaluator.transformBinaryComparator (operands of different types compare only
  after an ImplicitCastExpression up-cast)            kernel-defaults/.../internal/expressions/
                                                      DefaultExpressionEvaluator.java:337-354,
                                                      ImplicitCastExpression.java:30-41

Nodes use the evaluator's shape: ("AND"|"OR", a, b); (cmp, left, right) with operands
("stat", path), ("lit", value, type) and ("timeadd", ("stat", path)). None = Optional.empty().
Nothing here is used by the product path.
"""
from __future__ import annotations

import json

NUM_RECORDS, MIN, MAX, NULL_COUNT = "numRecords", "minValues", "maxValues", "nullCount"
_ELIGIBLE_NAMES = ("byte", "short", "integer", "long", "float", "double", "date", "timestamp", "timestamp_ntz",
                   "string")
_REVERSE = {"=": "=", "<": ">", "<=": ">=", ">": "<", ">=": "<=", "IS NOT DISTINCT FROM": "IS NOT DISTINCT FROM"}
_NEGATED = {"<": ">=", "<=": ">", ">": "<=", ">=": "<"}
_UPCAST = {"byte": ("short", "integer", "long", "float", "double"), "short": ("integer", "long", "float", "double"),
           "integer": ("long", "float", "double"), "long": ("float", "double"), "float": ("double",)}


class Incomparable(RuntimeError):
    """DefaultExpressionEvaluator: operands of different types which are not comparable."""


def _type_name(t):
    if isinstance(t, str):
        return t
    return t.get("type", "complex") if isinstance(t, dict) else str(t)


class StatsSchema:
    """StatsSchemaHelper over a table's data schema (partition columns removed,
    Metadata.getDataSchema): every leaf (any non-struct field) maps its logical path to its
    physical path (delta.columnMapping.physicalName) and type."""

    def __init__(self, schema_string, partition_columns=()):
        drop = {c.lower() for c in partition_columns}
        self.cols = {}

        def visit(fields, logical, physical, top):
            for f in fields:
                if top and f["name"].lower() in drop:
                    continue
                meta = f.get("metadata") or {}
                lp = logical + (f["name"],)
                pp = physical + (meta.get("delta.columnMapping.physicalName", f["name"]),)
                t = f["type"]
                if isinstance(t, dict) and t.get("type") == "struct":
                    visit(t["fields"], lp, pp, False)
                else:
                    self.cols[lp] = (pp, _type_name(t))
        visit(json.loads(schema_string)["fields"], (), (), True)

    @staticmethod
    def eligible_type(t):
        return t in _ELIGIBLE_NAMES or t.startswith("decimal")

    def minmax_ok(self, col):
        return col in self.cols and self.eligible_type(self.cols[col][1])

    def nullcount_ok(self, col):
        return col in self.cols

    def min_col(self, col):
        return ("stat", (MIN,) + self.cols[col][0])

    def max_col(self, col):
        phys, t = self.cols[col]
        s = ("stat", (MAX,) + phys)
        return ("timeadd", s) if t in ("timestamp", "timestamp_ntz") else s

    def null_count_col(self, col):
        return ("stat", (NULL_COUNT,) + self.cols[col][0])


def _kind(e):
    """'col' / 'lit' / 'pred' for an expression of delta_amd.expressions (duck-typed)."""
    if hasattr(e, "names"):
        return "col"
    if hasattr(e, "value") and hasattr(e, "type") and not hasattr(e, "children"):
        return "lit"
    return "pred"


def _P(name, *children):
    from delta_amd.expressions import Predicate
    return Predicate(name, *children)


def build(pred, S: StatsSchema):
    """constructDataSkippingFilter."""
    name = pred.name.upper()
    ch = pred.children
    if name == "AND":
        a, b = build(ch[0], S), build(ch[1], S)
        if a is not None and b is not None:
            return ("AND", a, b)
        return a if a is not None else b
    if name == "OR":
        a, b = build(ch[0], S), build(ch[1], S)
        return ("OR", a, b) if a is not None and b is not None else None
    if name == "IS_NOT_NULL":
        c = ch[0]
        if _kind(c) == "col" and S.nullcount_ok(c.names):
            return ("<", S.null_count_col(c.names), ("stat", (NUM_RECORDS,)))
        return None
    if name == "IS_NULL":
        c = ch[0]
        if _kind(c) == "col" and S.nullcount_ok(c.names):
            return (">", S.null_count_col(c.names), ("lit", 0, "long"))
        return None
    if name in _REVERSE:
        left, right = ch
        if _kind(left) == "col" and _kind(right) == "lit":
            if S.minmax_ok(left.names) and S.eligible_type(right.type):
                return _comparator(pred.name.upper(), left, right, S)
            return None
        if _kind(right) == "col" and _kind(left) == "lit":
            return build(_P(_REVERSE[name], right, left), S)
        return None
    if name == "NOT":
        return _build_not(ch[0], S)
    return None


def _comparator(name, col, lit, S):
    """constructComparatorDataSkippingFilters + constructBinaryDataSkippingPredicate."""
    v = ("lit", lit.value, lit.type)
    c = col.names
    if name == "=":
        return ("AND", ("<=", S.min_col(c), v), (">=", S.max_col(c), v))
    if name in ("<", "<="):
        return (name, S.min_col(c), v)
    if name in (">", ">="):
        return (name, S.max_col(c), v)
    return build(_null_safe_eq(col, lit), S)         # IS NOT DISTINCT FROM


def _null_safe_eq(col, lit):
    """rewriteEqualNullSafe."""
    if lit.value is None:
        return _P("IS_NULL", col)
    return _P("AND", _P("IS_NOT_NULL", col), _P("=", col, lit))


def _not_equal(eq, S, then):
    """constructDataSkippingFiltersForNotEqual."""
    left, right = eq.children
    if _kind(right) == "col" and _kind(left) == "lit":
        return build(_P("NOT", _P(eq.name, right, left)), S)
    if _kind(left) == "col" and _kind(right) == "lit":
        if S.minmax_ok(left.names) and S.eligible_type(right.type):
            return then(left, right)
    return None


def _build_not(child, S):
    """constructNotDataSkippingFilters."""
    name = child.name.upper()
    ch = child.children
    if name == "AND":
        return build(_P("OR", _P("NOT", ch[0]), _P("NOT", ch[1])), S)
    if name == "OR":
        return build(_P("AND", _P("NOT", ch[0]), _P("NOT", ch[1])), S)
    if name == "IS_NOT_NULL":
        return build(_P("IS_NULL", ch[0]), S)
    if name == "IS_NULL":
        return build(_P("IS_NOT_NULL", ch[0]), S)
    if name == "=":
        return _not_equal(child, S, lambda c, l: ("OR", ("<", S.min_col(c.names), ("lit", l.value, l.type)),
                                                  (">", S.max_col(c.names), ("lit", l.value, l.type))))
    if name in _NEGATED:
        return build(_P(_NEGATED[name], *ch), S)
    if name == "IS NOT DISTINCT FROM":
        return _not_equal(child, S, lambda c, l: build(_P("NOT", _null_safe_eq(c, l)), S))
    if name == "NOT":
        return build(ch[0], S)
    return None


def _operand_type(e, S):
    if e[0] == "stat":
        p = e[1]
        if p[0] in (NUM_RECORDS, NULL_COUNT):
            return "long"
        for phys, t in S.cols.values():
            if phys == p[1:]:
                return t
        raise KeyError(p)
    if e[0] == "lit":
        return e[2]
    if e[0] == "timeadd":
        return _operand_type(e[1], S)
    return "boolean"


def check(node, S):
    """transformBinaryComparator on every comparator of the built predicate: different types compare
    only when one up-casts to the other."""
    if node is None:
        return
    if node[0] in ("AND", "OR"):
        check(node[1], S)
        check(node[2], S)
        return
    lt, rt = _operand_type(node[1], S), _operand_type(node[2], S)
    if lt == rt or rt in _UPCAST.get(lt, ()) or lt in _UPCAST.get(rt, ()):
        return
    raise Incomparable("Unsupported expression: %s: operands are of different types which are not comparable: "
                       "left type=%s, right type=%s" % (node[0], lt, rt))


def stat_types(node, S, out=None):
    """{stats path: type name} of every stats field the predicate reads (nullCount / numRecords:
    long; min / max: the column's type, decimals as "decimal")."""
    out = {} if out is None else out
    if node[0] in ("AND", "OR"):
        stat_types(node[1], S, out)
        stat_types(node[2], S, out)
    elif node[0] == "timeadd":
        stat_types(node[1], S, out)
    elif node[0] == "stat":
        t = _operand_type(node, S)
        out[node[1]] = "decimal" if t.startswith("decimal") else t
    elif node[0] != "lit":
        stat_types(node[1], S, out)
        stat_types(node[2], S, out)
    return out


def _has_data_columns(children, parts):
    """PartitionUtils.hasNonPartitionColumns (kernel-api/.../internal/util/PartitionUtils.java:398-415)."""
    for c in children:
        k = _kind(c)
        if k == "col":
            if len(c.names) != 1 or c.names[0].lower() not in parts:
                return True
        elif k == "pred" and _has_data_columns(c.children, parts):
            return True
    return False


def split(pred, partition_columns=()):
    """PartitionUtils.splitMetadataAndDataPredicates (:242-263) with combineWithAndOp (:417-430):
    (partition predicate, data predicate), None for ALWAYS_TRUE."""
    parts = {c.lower() for c in partition_columns}

    def conj(a, b):
        if a is None:
            return b
        if b is None:
            return a
        if "ALWAYS_FALSE" in (a.name.upper(), b.name.upper()):
            return _P("ALWAYS_FALSE")
        return _P("AND", a, b)

    def go(p):
        if p.name.upper() == "ALWAYS_TRUE":
            return None, None
        if p.name.upper() == "AND":
            l1, l2 = go(p.children[0])
            r1, r2 = go(p.children[1])
            return conj(l1, r1), conj(l2, r2)
        return (None, p) if _has_data_columns(p.children, parts) else (p, None)
    return go(pred)
