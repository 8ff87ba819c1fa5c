"""CPU ORACLE (test infrastructure only) for K11 data skipping: a restatement of what the reference
does with a data-skipping predicate once the scan files are reconciled.

  ScanImpl.applyDataSkipping            kernel-api/.../internal/ScanImpl.java:304-352
      filter = COALESCE(skippingPredicate, true); rows selected = existing selection AND filter
  DataSkippingUtils.parseJsonStats      kernel-api/.../internal/skipping/DataSkippingUtils.java:41-52
      only selected rows with non-null stats are parsed (DefaultJsonHandler.parseJson :60-76)
  DefaultJsonHandler.parseJson(String)  kernel-defaults/.../engine/DefaultJsonHandler.java:193-200
      Jackson readTree with USE_BIG_DECIMAL_FOR_FLOATS (:48); trailing content ignored; the root
      must be an object
  DefaultJsonRow.decodeElement          kernel-defaults/.../internal/data/DefaultJsonRow.java:136-270
      long/integer: an integral token in range; short/byte: any number whose exact value is an
      integer in range (canConvertToExactIntegral); date: a string through java.sql.Date.valueOf
      (:249-252); string: a JSON string, compared as unsigned UTF-8 bytes then length
      (DefaultExpressionUtils.java:49-54); float/double: the exact number rounded to the format
      (an infinite result is an error) or one of the NaN / Infinity strings (:182-238), compared
      with Float.compare / Double.compare (DefaultExpressionUtils.java:146-153) after
      ImplicitCastExpression widening; struct: an object; JSON null = null
  DefaultExpressionEvaluator            kernel-defaults/.../internal/expressions/
      comparators are null when either side is null; AND/OR are Kleene (visitAnd/visitOr)

The predicate tree is the planner's (delta_amd/skipping.py, itself restating DataSkippingUtils
.constructDataSkippingFilter); `types` maps each referenced stats path to its Kernel type name.
Nothing here is used by the product path.
"""
from __future__ import annotations

import datetime as _dt
import json
import math
import re
from decimal import Decimal
from fractions import Fraction

import numpy as np

RANGES = {"long": (-(1 << 63), (1 << 63) - 1), "integer": (-(1 << 31), (1 << 31) - 1),
          "short": (-(1 << 15), (1 << 15) - 1), "byte": (-(1 << 7), (1 << 7) - 1)}


class StatsDecodeError(RuntimeError):
    pass


def _reject_constant(tok):
    raise StatsDecodeError("non-standard JSON token %s" % tok)


_DECODER = json.JSONDecoder(parse_float=Decimal, parse_constant=_reject_constant)


def parse_root(s: str):
    i = 0
    while i < len(s) and s[i] in " \t\r\n":
        i += 1
    try:
        obj, _ = _DECODER.raw_decode(s, i)          # trailing content is ignored, as readTree does
    except json.JSONDecodeError as e:
        raise StatsDecodeError("Could not parse JSON: %s" % s) from e
    if not isinstance(obj, dict):
        raise StatsDecodeError("stats root is not an object: %s" % s)
    return obj


def _date_field(t):
    if len(t) >= 2 and t[0] == "+":                   # Integer.parseInt accepts a leading '+'
        t = t[1:]
    if not t or any(c not in "0123456789" for c in t):
        raise StatsDecodeError("Couldn't decode %r, expected a date" % t)
    return int(t)


def _date(text):
    """InternalUtils.daysSinceEpoch(java.sql.Date.valueOf(text)): DefaultJsonRow.java:249-252,
    InternalUtils.java:85-89. valueOf: a 4-char year, 1-2 char month and day, month 1..12, day
    1..31; the lenient calendar carries a day past the month end into the next month. Years before
    1583 (Julian part of the hybrid calendar) and non-ASCII digits are refused by this build."""
    n = len(text)
    d1 = text.find("-")
    d2 = text.find("-", d1 + 1)
    if not (d1 > 0 and d2 > 0 and d2 < n - 1 and d1 == 4 and 1 < d2 - d1 <= 3 and 1 < n - d2 <= 3):
        raise StatsDecodeError("Couldn't decode %r, expected a date" % text)
    y, m, d = _date_field(text[:4]), _date_field(text[d1 + 1:d2]), _date_field(text[d2 + 1:])
    if not (1 <= m <= 12 and 1 <= d <= 31) or y < 1583:
        raise StatsDecodeError("Couldn't decode %r, expected a date" % text)
    return (_dt.date(y, m, 1) - _dt.date(1970, 1, 1)).days + d - 1


_TS = re.compile(r"(\d{4})-(\d{2})-(\d{2})[Tt](\d{2}):(\d{2})(?::(\d{2})(?:\.(\d{1,9}))?)?"
                 r"(?:([Zz])|([+-])(\d{2}):(\d{2})(?::(\d{2}))?)")


def _timestamp(text):
    """MICROS.between(EPOCH, OffsetDateTime.parse(text).toInstant()): DefaultJsonRow.java:254-258.
    ISO_OFFSET_DATE_TIME with the strict resolver; years outside 1678..2261 (where Instant.until's
    nanosecond difference would overflow), signed years and '.' without digits are refused here."""
    m = _TS.fullmatch(text) if text.isascii() else None
    if not m:
        raise StatsDecodeError("Couldn't decode %r, expected a timestamp" % text)
    y, mo, d, h, mi = (int(m.group(i)) for i in range(1, 6))
    sec = int(m.group(6) or 0)
    nanos = int((m.group(7) or "").ljust(9, "0") or 0)
    try:
        day = _dt.date(y, mo, d)
    except ValueError:
        raise StatsDecodeError("Couldn't decode %r, expected a timestamp" % text) from None
    if not 1678 <= y <= 2261 or h > 23 or mi > 59 or sec > 59:
        raise StatsDecodeError("Couldn't decode %r, expected a timestamp" % text)
    off = 0
    if m.group(9):
        oh, om, os_ = int(m.group(10)), int(m.group(11)), int(m.group(12) or 0)
        off = oh * 3600 + om * 60 + os_
        if oh > 18 or om > 59 or os_ > 59 or off > 18 * 3600:
            raise StatsDecodeError("Couldn't decode %r, expected a timestamp" % text)
        off = -off if m.group(9) == "-" else off
    secs = (day - _dt.date(1970, 1, 1)).days * 86400 + h * 3600 + mi * 60 + sec - off
    total = secs * 1_000_000_000 + nanos
    return total // 1000 if total >= 0 else -((-total) // 1000)     # Java division: toward zero


_TS_NTZ = re.compile(r"(\d{4})-(\d{2})-(\d{2})T(\d{2}):(\d{2}):(\d{2})(?:\.(\d{0,6}))?")


def _timestamp_ntz(text):
    """DefaultKernelUtils.parseTimestampNTZ (DefaultKernelUtils.java:34-40,91-95): pattern
    yyyy-MM-dd'T'HH:mm:ss + optional 1-6 digit fraction, SMART resolver (a day past the month end is
    clamped to its last day), read as UTC. Same year window and refusals as _timestamp."""
    m = _TS_NTZ.fullmatch(text) if text.isascii() else None
    if not m:
        raise StatsDecodeError("Couldn't decode %r, expected a timestamp_ntz" % text)
    y, mo, d, h, mi, sec = (int(m.group(i)) for i in range(1, 7))
    # appendFraction(MICRO_OF_SECOND, 0, 6, true): minimum width 0, so "." alone is a zero fraction
    micros = int((m.group(7) or "").ljust(6, "0") or 0)
    # java.time.format.Parsed.resolveTime, SMART: 24:00:00(.0) is the end of the day = next midnight
    end_of_day = h == 24 and mi == 0 and sec == 0 and micros == 0
    if not (1678 <= y <= 2261 and 1 <= mo <= 12 and 1 <= d <= 31 and (h <= 23 or end_of_day) and mi <= 59
            and sec <= 59):
        raise StatsDecodeError("Couldn't decode %r, expected a timestamp_ntz" % text)
    import calendar
    d = min(d, calendar.monthrange(y, mo)[1])
    secs = (_dt.date(y, mo, d) - _dt.date(1970, 1, 1)).days * 86400 + h * 3600 + mi * 60 + sec
    return secs * 1_000_000 + micros


_F32_MAX = float.fromhex("0x1.fffffep127")


def _nearest_even(x: Fraction, lo: float, hi: float, lo_even: bool) -> float:
    """Whichever of lo < hi (adjacent binary values around x) is nearer to x; ties to the even one."""
    dl, dh = x - Fraction(lo), Fraction(hi) - x
    return lo if dl < dh or (dl == dh and lo_even) else hi


def _to_float32(x: Fraction):
    """Correctly rounded binary32 value of an exact x (as a Python float), +-inf on overflow.
    The double nearest x is found first (correctly rounded by Python), then the two binary32
    neighbours around x are compared exactly, so double rounding cannot creep in."""
    if x == 0:
        return 0.0
    a = abs(x)
    d = float(a) if a < Fraction(2) ** 1030 else math.inf
    f = float(np.float32(d)) if d <= _F32_MAX else math.inf
    # neighbours of x in binary32 (inf stands for the first value past the largest)
    if f != math.inf and Fraction(f) > a:
        hi, lo = f, float(np.nextafter(np.float32(f), np.float32(0)))
    elif f != math.inf:
        lo = f
        hi = float(np.nextafter(np.float32(f), np.float32(np.inf))) if f < _F32_MAX else 2.0 ** 128
    else:
        lo, hi = _F32_MAX, 2.0 ** 128
    if Fraction(lo) == a:
        r = lo
    else:
        lo_even = lo == 0 or (int(np.float32(lo).view(np.uint32)) & 1) == 0
        r = _nearest_even(a, lo, hi, lo_even)
    r = math.inf if r >= 2.0 ** 128 else r
    return r if x > 0 else -r


_SPECIAL = {"NaN": math.nan, "+INF": math.inf, "+Infinity": math.inf, "Infinity": math.inf,
            "-INF": -math.inf, "-Infinity": -math.inf}


def _floating(v, typ):
    """DefaultJsonRow.java:182-238: a number is rounded from its exact value (DecimalNode
    floatValue / doubleValue; IntNode / LongNode / BigIntegerNode widen), an infinite result is a
    decode error; the strings NaN / +INF / +Infinity / Infinity / -INF / -Infinity are accepted.
    Zero is +0.0 whatever its sign (BigDecimal has no negative zero)."""
    if isinstance(v, str):
        if v in _SPECIAL:
            return _SPECIAL[v]
        raise StatsDecodeError("Couldn't decode %r, expected a %s" % (v, typ))
    if isinstance(v, bool) or not isinstance(v, (int, Decimal)):
        raise StatsDecodeError("Couldn't decode %r, expected a %s" % (v, typ))
    x = Fraction(v)
    if x == 0:
        return 0.0
    r = _to_float32(x) if typ == "float" else float(Decimal(v))
    if math.isinf(r):
        raise StatsDecodeError("Couldn't decode %r, expected a %s" % (v, typ))
    return r


def _leaf(v, typ):
    if v is None:
        return None
    if typ in ("float", "double"):
        return _floating(v, typ)
    if typ == "decimal":                               # DefaultJsonRow: isNumber -> decimalValue()
        if isinstance(v, bool) or not isinstance(v, (int, Decimal)):
            raise StatsDecodeError("Couldn't decode %r, expected a decimal" % (v,))
        return Decimal(v)
    if typ == "timestamp_ntz":
        if not isinstance(v, str):
            raise StatsDecodeError("Couldn't decode %r, expected a timestamp_ntz" % (v,))
        return _timestamp_ntz(v)
    if typ == "timestamp":
        if not isinstance(v, str):
            raise StatsDecodeError("Couldn't decode %r, expected a timestamp" % (v,))
        return _timestamp(v)
    if typ == "string":                                # DefaultJsonRow.java:170-173 (isTextual),
        if not isinstance(v, str):                     # compared as String.getBytes(UTF_8): a lone
            raise StatsDecodeError("Couldn't decode %r, expected a string" % (v,))   # surrogate is '?'
        return v.encode("utf-8", "replace")
    if typ == "date":
        if not isinstance(v, str):
            raise StatsDecodeError("Couldn't decode %r, expected a date" % (v,))
        return _date(v)
    lo, hi = RANGES[typ]
    if isinstance(v, bool) or not isinstance(v, (int, Decimal)):
        raise StatsDecodeError("Couldn't decode %r, expected a %s" % (v, typ))
    if isinstance(v, Decimal):
        if typ in ("long", "integer") or v != v.to_integral_value():
            raise StatsDecodeError("Couldn't decode %r, expected a %s" % (v, typ))
        v = int(v)
    if not lo <= v <= hi:
        raise StatsDecodeError("Couldn't decode %r, expected a %s" % (v, typ))
    return v


def decode_stats(s: str, types: dict) -> dict:
    """path tuple -> python int or None, for every referenced path."""
    root = parse_root(s)
    out = {}
    for path, typ in types.items():
        node = root
        for comp in path[:-1]:
            node = node.get(comp)
            if node is None:
                break
            if not isinstance(node, dict):
                raise StatsDecodeError("Couldn't decode %r, expected a object" % (node,))
        out[path] = None if node is None else _leaf(node.get(path[-1]), typ)
    return out


_WIDEN = {"byte": 0, "short": 1, "integer": 2, "long": 3, "float": 4, "double": 5}


def _java_compare(a, b) -> int:
    """Float.compare / Double.compare: -0.0 < 0.0, NaN above everything and equal to itself."""
    an, bn = a != a, b != b
    if an or bn:
        return (an > bn) - (an < bn)
    if a == b == 0:
        sa, sb = math.copysign(1.0, a), math.copysign(1.0, b)
        return (sa > sb) - (sa < sb)
    return (a > b) - (a < b)


def _cast(v, frm, to):
    """ImplicitCastExpression (ImplicitCastExpression.java:30-41, 118-125): integral -> float /
    double rounds to nearest even, float -> double is exact."""
    if frm == to or frm in ("float", "double"):
        return float(v)
    return _to_float32(Fraction(v)) if to == "float" else float(v)


def _float_compare(a, ta, b, tb):
    """The comparator over two operands of which one is float / double typed."""
    w = ta if _WIDEN.get(ta, -1) >= _WIDEN.get(tb, -1) else tb
    return _java_compare(_cast(a, ta, w), _cast(b, tb, w))


def _type_of(node, types):
    if node[0] == "stat":
        return types.get(node[1]) if types else None
    if node[0] == "lit":
        return node[2] if len(node) > 2 else None
    if node[0] == "timeadd":
        return _type_of(node[1], types)
    return "boolean"


def evaluate(node, vals, types=None):
    """True / False / None (null) for a planner node over decoded stats."""
    k = node[0]
    if k == "stat":
        return vals[node[1]]
    if k == "timeadd":                                 # DefaultExpressionEvaluator.visitTimeAdd
        a = evaluate(node[1], vals)
        return None if a is None else a + 1000
    if k == "lit":
        return node[1].encode("utf-8", "replace") if isinstance(node[1], str) else node[1]
    if k == "AND":
        a, b = evaluate(node[1], vals, types), evaluate(node[2], vals, types)
        if a is False or b is False:
            return False
        return True if (a is True and b is True) else None
    if k == "OR":
        a, b = evaluate(node[1], vals, types), evaluate(node[2], vals, types)
        if a is True or b is True:
            return True
        return False if (a is False and b is False) else None
    a, b = evaluate(node[1], vals, types), evaluate(node[2], vals, types)
    if a is None or b is None:
        return None
    ta, tb = _type_of(node[1], types), _type_of(node[2], types)
    if ta in ("float", "double") or tb in ("float", "double"):
        c = _float_compare(a, ta, b, tb)
        return {"<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0, "=": c == 0}[k]
    return {"<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b, "=": a == b}[k]


def keep(stats: str | None, node, types) -> bool:
    """COALESCE(skippingPredicate, true) for one selected row (null stats -> kept)."""
    if stats is None:
        return True
    return evaluate(node, decode_stats(stats, types), types) is not False


# ---- the C fast path (oracle/dk_skip.c) for predicates over integral stats only ----------------
_INTEGRAL = {"long": 0, "integer": 1, "short": 2, "byte": 3}
_CMP_OPS = {"<": 3, "<=": 4, ">": 5, ">=": 6, "=": 7}


def compile_integral(node, types):
    """(paths blob, number of paths, int64 program) for dk_skip.c when every referenced stat is
    long / integer / short / byte and every literal an integer in the long range; else None (the
    caller evaluates every row with `keep`)."""
    import struct
    if not types or len(types) > 16 or any(t not in _INTEGRAL for t in types.values()):
        return None
    order = list(types)
    ops = []

    def emit(n):
        k = n[0]
        if k == "stat":
            ops.append((1, order.index(n[1])))
        elif k == "lit":
            v = n[1]
            if isinstance(v, bool) or not isinstance(v, int) or not -(1 << 63) <= v < (1 << 63):
                raise ValueError
            ops.append((2, v))
        elif k in ("AND", "OR"):
            emit(n[1]); emit(n[2]); ops.append((8 if k == "AND" else 9, 0))
        elif k in _CMP_OPS:
            emit(n[1]); emit(n[2]); ops.append((_CMP_OPS[k], 0))
        else:
            raise ValueError
    try:
        emit(node)
    except (ValueError, IndexError):
        return None
    if len(ops) > 60:
        return None
    blob = bytearray()
    for p in order:
        if len(p) > 8:
            return None
        blob += bytes([_INTEGRAL[types[p]], len(p)])
        for comp in p:
            b = comp.encode("utf-8")
            blob += struct.pack("<H", len(b)) + b
    return bytes(blob), len(order), np.array([x for op in ops for x in op], dtype=np.int64)


def apply_to_column(col, sel, node, types, max_def=2):
    """Data skipping over one decoded add.stats column: sel (uint8, one per row) is cleared where
    COALESCE(predicate, true) is FALSE. Integral predicates go through dk_skip.c (rows it is unsure
    about, and every row of other predicates, through `keep`); other selected rows through `keep`."""
    import ctypes as C
    rows = np.nonzero(sel)[0]
    if col is None or not len(rows):
        return sel
    prog = compile_integral(node, types)
    if prog is not None:
        from .ref import lib
        blob, n_paths, ops = prog
        defer = np.zeros(len(sel), dtype=np.uint8)
        chars = col.chars if col.chars is not None and len(col.chars) else np.zeros(1, np.uint8)
        P = C.c_void_p
        nd = lib().dkr_skip_eval(P(chars.ctypes.data), P(col.offs.ctypes.data), P(col.row_def.ctypes.data),
                                 max_def, P(sel.ctypes.data), P(defer.ctypes.data), len(sel), blob, len(blob),
                                 n_paths, P(ops.ctypes.data), len(ops) // 2)
        if nd < 0:
            raise RuntimeError("dkr_skip_eval: malformed program")
        rows = np.nonzero(defer)[0]
    for i in rows:
        i = int(i)
        st = None if col.row_def[i] < max_def else col.string(i).decode("utf-8", "replace")
        if not keep(st, node, types):
            sel[i] = 0
    return sel
