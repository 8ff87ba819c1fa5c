"""CPU ORACLE (test infrastructure only) for partition pruning: ScanImpl.applyPartitionPruning
(kernel-api/.../internal/ScanImpl.java:247-294) restated on the predicate tree itself.

  PartitionUtils.rewritePartitionPredicateOnScanFileSchema (util/PartitionUtils.java:324-358):
      a partition column becomes element_at(add.partitionValues, physical name), deserialized by
      PartitionValueEvaluator (kernel-defaults/.../expressions/PartitionValueEvaluator.java:50-90:
      Long/Integer/Short/Byte.parseX, dates through java.sql.Date.valueOf (:72-73, restated in
      oracle/skipping.py:_date), Boolean.parseBoolean, Float.parseFloat / Double.parseDouble
      (:93-100), timestamps through java.sql.Timestamp.valueOf + InternalUtils.microsSinceEpoch
      (:80-87; InternalUtils.java:95-98) -- a malformed value fails the scan) unless it is a string;
      float comparisons use Float.compare / Double.compare after ImplicitCastExpression widening
  DefaultExpressionEvaluator: comparators are null if a side is null (IS NOT DISTINCT FROM is
      null-safe), AND/OR/NOT are Kleene and are evaluated on every row of the batch; strings compare
      as unsigned UTF-8 bytes, then length (DefaultExpressionUtils.java:39-56)
  DefaultPredicateEvaluator: selection = (selection = true) AND predicate; null drops the row
Nothing here is used by the product path.
"""
from __future__ import annotations

import re

RANGES = {"long": (-(1 << 63), (1 << 63) - 1), "integer": (-(1 << 31), (1 << 31) - 1),
          "short": (-(1 << 15), (1 << 15) - 1), "byte": (-(1 << 7), (1 << 7) - 1)}
_INT = re.compile(rb"^[+-]?[0-9]+$")
_DEC = re.compile(rb"^[+-]?(?:[0-9]+\.?([0-9]*)|\.([0-9]+))(?:[eE]([+-]?[0-9]+))?\Z")


class PartitionValueError(RuntimeError):
    pass


def _b(x):
    return x if isinstance(x, bytes) else str(x).encode("utf-8")


def element_at(pv, key: bytes):
    """pv: None (null map) or list of (key, value) with bytes/str items; first match wins."""
    if pv is None:
        return None
    for k, v in pv:
        if _b(k) == key:
            return None if v is None else _b(v)
    return None


_JFLOAT = re.compile(rb"^([+-]?)(?:(NaN)|(Infinity)|(0[xX][0-9a-fA-F]*\.?[0-9a-fA-F]*[pP][+-]?[0-9]+)|"
                     rb"((?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?))[fFdD]?$")


def _java_trim(b: bytes) -> bytes:
    i, j = 0, len(b)
    while i < j and b[i] <= 0x20:
        i += 1
    while j > i and b[j - 1] <= 0x20:
        j -= 1
    return b[i:j]


def _parse_floating(v: bytes, typ: str):
    """Float.parseFloat / Double.parseDouble (FloatingDecimal.readJavaFormatString): trimmed; sign;
    NaN / Infinity; decimal or hexadecimal digits with an optional f/F/d/D suffix (none after NaN /
    Infinity); correctly rounded, overflow to +-Infinity, the sign kept on zero."""
    import math
    from decimal import Decimal
    from fractions import Fraction
    from oracle.skipping import _to_float32
    t = _java_trim(v)
    m = _JFLOAT.match(t)
    if not m or (m.group(2) or m.group(3)) and t[-1:] in b"fFdD" and not t.endswith((b"NaN", b"Infinity")):
        raise PartitionValueError("For input string: %r" % v)
    neg = m.group(1) == b"-"
    if m.group(2):
        return math.nan
    if m.group(3):
        return -math.inf if neg else math.inf
    if m.group(4):
        hx = m.group(4).decode().lower()
        mant, ex = hx[2:].split("p")
        ip, _, fp = mant.partition(".")
        x = Fraction(int((ip + fp) or "0", 16), 16 ** len(fp)) * Fraction(2) ** int(ex)
    else:
        x = Fraction(Decimal(m.group(5).decode()))
    if typ == "float":
        r = _to_float32(x) if x else 0.0
    else:
        try:
            r = x.numerator / x.denominator if x else 0.0
        except OverflowError:
            r = math.inf
    return -r if neg else r


def _timestamp_valueof(v: bytes) -> int:
    """java.sql.Timestamp.valueOf(s) then InternalUtils.microsSinceEpoch (InternalUtils.java:95-98):
    "yyyy-[m]m-[d]d hh:mm:ss[.f{1,9}]" split on the first space / dashes / colons / period, each
    field Integer.parseInt, month 1..12 and day 1..31, then the lenient calendar rolls the fields
    over; the local date-time is read back in the same zone, so the fields count as UTC here.
    Years before 1583 (Julian calendar) are refused, as for dates."""
    import datetime as _dt
    bad = PartitionValueError("Timestamp format must be yyyy-mm-dd hh:mm:ss[.fffffffff]: %r" % v)
    s = _java_trim(v).decode("utf-8", "replace")

    def pint(x):
        if not re.fullmatch(r"[+-]?[0-9]+", x):
            raise bad
        i = int(x)
        if not -(1 << 31) <= i < (1 << 31):
            raise bad
        return i
    sp = s.find(" ")
    if sp <= 0:
        raise bad
    date_s, time_s = s[:sp], s[sp + 1:]
    d1 = date_s.find("-")
    d2 = date_s.find("-", d1 + 1)
    if not (d1 > 0 and d2 > 0 and d2 < len(date_s) - 1):
        raise bad
    yyyy, mm, dd = date_s[:d1], date_s[d1 + 1:d2], date_s[d2 + 1:]
    if not (len(yyyy) == 4 and 1 <= len(mm) <= 2 and 1 <= len(dd) <= 2):
        raise bad
    y, mo, d = pint(yyyy), pint(mm), pint(dd)
    if not (1 <= mo <= 12 and 1 <= d <= 31) or y < 1583:
        raise bad
    c1 = time_s.find(":")
    c2 = time_s.find(":", c1 + 1)
    per = time_s.find(".", c2 + 1)
    if not (c1 > 0 and c2 > 0 and c2 < len(time_s) - 1):
        raise bad
    h, mi = pint(time_s[:c1]), pint(time_s[c1 + 1:c2])
    nanos = 0
    if 0 < per < len(time_s) - 1:
        sec = pint(time_s[c2 + 1:per])
        frac = time_s[per + 1:]
        if len(frac) > 9 or not frac[0].isdigit():
            raise bad
        nanos = pint(frac) * 10 ** (9 - len(frac))
    elif per > 0:
        raise bad
    else:
        sec = pint(time_s[c2 + 1:])
    days = (_dt.date(y, mo, 1) - _dt.date(1970, 1, 1)).days + d - 1
    total = (days * 86400 + h * 3600 + mi * 60 + sec) * 1_000_000_000 + nanos
    return total // 1000 if total >= 0 else -((-total) // 1000)


def deserialize(v, typ):
    if v is None or typ == "string":
        return v
    if typ == "boolean":                               # Boolean.parseBoolean: never fails
        return v.lower() == b"true"
    if typ in ("float", "double"):
        return _parse_floating(v, typ)
    if typ in ("timestamp", "timestamp_ntz"):
        return _timestamp_valueof(v)
    if typ.startswith("decimal"):                      # new BigDecimal(text): PartitionValueEvaluator :112-113
        from decimal import Decimal
        m = _DEC.match(v)
        if not m:
            raise PartitionValueError("Character array is missing \"exponent\" mark 'e' or 'E': %r" % v)
        frac = len(m.group(1) or m.group(2) or b"")
        if not -(1 << 31) <= frac - int(m.group(3) or 0) < (1 << 31):
            raise PartitionValueError("Scale out of range: %r" % v)
        return Decimal(v.decode("ascii"))
    if typ == "date":                                  # PartitionValueEvaluator.java:72-73
        from oracle.skipping import StatsDecodeError, _date
        try:
            return _date(v.decode("utf-8", "replace"))
        except StatsDecodeError as e:
            raise PartitionValueError(str(e)) from e
    if not _INT.match(v):
        raise PartitionValueError("For input string: %r" % v)
    x = int(v)
    lo, hi = RANGES[typ]
    if not lo <= x <= hi:
        raise PartitionValueError("Value out of range: %r" % v)
    return x


def evaluate(node, pv, fields):
    """True / False / None. `node` is a delta_amd.expressions node; fields: lower name -> (type, phys)."""
    kind = type(node).__name__
    if kind == "Column":
        t, phys = fields[node.names[0].lower()]
        return deserialize(element_at(pv, phys.encode("utf-8")), t)
    if kind == "Literal":
        return None if node.value is None else (_b(node.value) if node.type == "string" else node.value)
    n = node.name.upper()
    c = node.children
    if n in ("ALWAYS_TRUE", "ALWAYS_FALSE"):                  # ExpressionVisitor.java:91-94
        return n == "ALWAYS_TRUE"
    if n == "COALESCE":                                        # DefaultExpressionEvaluator.java:577-590
        vals = [evaluate(x, pv, fields) for x in c]            # (every argument evaluated)
        return next((v for v in vals if v is not None), None)
    if n == "STARTS_WITH":                                     # StartsWithExpressionEvaluator.java:62-92
        a, b = evaluate(c[0], pv, fields), evaluate(c[1], pv, fields)
        return None if a is None or b is None else a.decode("utf-8").startswith(b.decode("utf-8"))
    if n == "LIKE":                                            # LikeExpressionEvaluator.java:82-186
        a, b = evaluate(c[0], pv, fields), evaluate(c[1], pv, fields)
        esc = evaluate(c[2], pv, fields).decode("utf-8") if len(c) == 3 else "\\"
        if a is None or b is None:
            return None
        return re.fullmatch(_like_regex(b.decode("utf-8"), esc), a.decode("utf-8"), re.DOTALL) is not None
    if n == "SUBSTRING":                                       # SubstringEvaluator.java:92-156
        a = evaluate(c[0], pv, fields)
        if a is None:
            return None
        s = a.decode("utf-8")
        pos = c[1].value
        length = c[2].value if len(c) == 3 else None
        L = len(s)
        if pos > L or (length is not None and length < 1):
            return b""
        start = L + pos if pos < 0 else max(pos - 1, 0)
        si = max(start, 0)
        if length is None:
            return s[si:].encode("utf-8")
        e = start + length
        e = (e + 2 ** 31) % 2 ** 32 - 2 ** 31                 # Java int arithmetic
        ei = min(L, max(e, 0))
        if ei < si:
            raise PartitionValueError("begin %d, end %d" % (si, ei))   # String.substring throws
        return s[si:ei].encode("utf-8")
    if n == "TIMEADD":                                         # DefaultExpressionEvaluator.java:593-626
        a, b = evaluate(c[0], pv, fields), evaluate(c[1], pv, fields)
        if a is None or b is None:
            return None
        v = (a + ((b * 1000 + 2 ** 63) % 2 ** 64 - 2 ** 63)) % 2 ** 64          # Java long arithmetic
        return v - 2 ** 64 if v >= 2 ** 63 else v
    if n in ("AND", "OR"):
        a, b = evaluate(c[0], pv, fields), evaluate(c[1], pv, fields)
        if n == "AND":
            return False if (a is False or b is False) else (True if (a is True and b is True) else None)
        return True if (a is True or b is True) else (False if (a is False and b is False) else None)
    if n == "NOT":
        a = evaluate(c[0], pv, fields)
        return None if a is None else (not a)
    if n in ("IS_NULL", "IS_NOT_NULL"):
        a = evaluate(c[0], pv, fields)
        return (a is None) if n == "IS_NULL" else (a is not None)
    a, b = evaluate(c[0], pv, fields), evaluate(c[1], pv, fields)
    ta, tb = _type(c[0], fields), _type(c[1], fields)
    if ta in ("float", "double") or tb in ("float", "double"):
        from oracle.skipping import _float_compare
        cmp = (lambda x, y: _float_compare(x, ta, y, tb))
    else:
        cmp = (lambda x, y: (x > y) - (x < y))
    if n == "IS NOT DISTINCT FROM":
        if a is None or b is None:
            return a is None and b is None
        return cmp(a, b) == 0
    if a is None or b is None:
        return None
    r = cmp(a, b)
    return {"<": r < 0, "<=": r <= 0, ">": r > 0, ">=": r >= 0, "=": r == 0}[n]


def _like_regex(pattern, esc):
    """LikeExpressionEvaluator.escapeLikeRegex (:155-186) as a Python regex."""
    out, i = [], 0
    while i < len(pattern):
        ch = pattern[i]
        if ch == esc:
            if i == len(pattern) - 1 or pattern[i + 1] not in ("_", "%", esc):
                raise PartitionValueError("LIKE expression has invalid escape sequence: %r" % pattern)
            out.append(re.escape(pattern[i + 1]))
            i += 2
            continue
        out.append("." if ch == "_" else ".*" if ch == "%" else re.escape(ch))
        i += 1
    return "".join(out)


def _type(node, fields):
    kind = type(node).__name__
    if kind == "Predicate" and node.name.upper() == "SUBSTRING":
        return "string"
    if kind == "Predicate" and node.name.upper() == "TIMEADD":
        return _type(node.children[0], fields)
    if kind == "Column":
        return fields[node.names[0].lower()][0]
    if kind == "Literal":
        return node.type
    return "boolean"


def json_map(add: dict):
    pv = add.get("partitionValues")
    return None if pv is None else list(pv.items()) if isinstance(pv, dict) else pv
