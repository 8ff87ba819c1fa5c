"""Exact float / double comparison planning for the device evaluators.

The reference compares a float or double stats value (or partition value) with a literal after
rounding the exact decimal it was written as to the binary format (Jackson DecimalNode.floatValue /
doubleValue with USE_BIG_DECIMAL_FOR_FLOATS, DefaultJsonHandler.java:48, DefaultJsonRow.java:182-238;
Float.parseFloat / Double.parseDouble, PartitionValueEvaluator.java:93-100), then Float.compare /
Double.compare (DefaultExpressionUtils.java:146-153): -0.0 < 0.0 and NaN above everything, equal to
itself. Integral operands compared with a float literal are widened by ImplicitCastExpression
(int/long -> float/double, round to nearest even).

Rounding is monotone, so for a fixed literal the set of exact values x whose rounded value satisfies
`round(x) <op> literal` is an interval of the reals, bounded by the edge of a rounding cell (a
midpoint between two neighbouring binary values, i.e. a dyadic rational with a finite decimal
expansion). The planner turns each comparison into "x < B", "x <= B", "x > B", "x >= B", always or
never, plus the constant results for the NaN / +Infinity / -Infinity stats values; the GPU then
compares the value's decimal digits with B exactly (no binary conversion on the device).
"""
from __future__ import annotations

import math
import struct
from fractions import Fraction

# (precision bits, smallest ulp exponent, largest unbiased exponent)
FORMATS = {"float": (24, -149, 127), "double": (53, -1074, 1023)}
NAN, PINF, NINF = "nan", "+inf", "-inf"
ALL, NONE = "all", "none"


def _fmt(name):
    p, emin_ulp, emax = FORMATS[name]
    return p, emin_ulp, emax


def max_finite(name) -> Fraction:
    p, _, emax = _fmt(name)
    return Fraction((1 << p) - 1) * Fraction(2) ** (emax - p + 1)


def overflow_threshold(name) -> Fraction:
    """Smallest |x| that rounds to infinity (the tie above the largest value goes to the even
    neighbour, infinity)."""
    p, _, emax = _fmt(name)
    return Fraction(2) ** (emax + 1) - Fraction(2) ** (emax - p)


def _ulp_exp(a: Fraction, name) -> int:
    """Exponent of the ulp of the format's binade holding a > 0."""
    p, emin_ulp, _ = _fmt(name)
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    return max(e - (p - 1), emin_ulp)


def _index_floor(a: Fraction, name) -> int:
    """IEEE bit pattern (as an integer) of the largest non-negative finite value <= a (a >= 0)."""
    p, emin_ulp, emax = _fmt(name)
    if a <= 0:
        return 0
    if a >= max_finite(name):
        return index_of(max_finite(name), name)
    ue = _ulp_exp(a, name)
    m = math.floor(a / Fraction(2) ** ue)
    if m >= 1 << p:                      # rounding of ue at a binade edge
        ue += 1
        m = math.floor(a / Fraction(2) ** ue)
    return index_of(Fraction(m) * Fraction(2) ** ue, name)


def index_of(v: Fraction, name) -> int:
    """Bit pattern of a non-negative finite value of the format."""
    p, emin_ulp, _ = _fmt(name)
    if v == 0:
        return 0
    ue = _ulp_exp(v, name)
    m = v / Fraction(2) ** ue
    assert m.denominator == 1, "not a value of the format"
    m = m.numerator
    if ue == emin_ulp and m < 1 << (p - 1):
        return m                                          # subnormal
    biased = ue - emin_ulp + 1
    return (biased << (p - 1)) | (m - (1 << (p - 1)))


def value_of(bits: int, name) -> Fraction:
    p, emin_ulp, _ = _fmt(name)
    biased, frac = bits >> (p - 1), bits & ((1 << (p - 1)) - 1)
    if biased == 0:
        return Fraction(frac) * Fraction(2) ** emin_ulp
    return Fraction((1 << (p - 1)) | frac) * Fraction(2) ** (emin_ulp + biased - 1)


def _max_index(name):
    return index_of(max_finite(name), name)


# ranks: a total order over the format with -inf < ... < -0 < +0 < ... < +inf (NaN kept apart):
# rank r >= 0 is the bit pattern of +value, rank -1 - bits is -value
def _rank_value(r, name):
    mx = _max_index(name)
    if r > mx:
        return PINF
    if r < -mx - 1:
        return NINF
    if r >= 0:
        return (value_of(r, name), False)
    return (-value_of(-r - 1, name), True)


def cell(r, name):
    """Rounding cell of rank r: (lo, lo_included, hi, hi_included); None ends are unbounded."""
    mx = _max_index(name)
    T = overflow_threshold(name)
    if r == mx + 1:
        return (T, True, None, False)
    if r == -mx - 2:
        return (None, False, -T, True)
    v = _rank_value(r, name)
    x, negz = v
    if x == 0:
        h = value_of(1, name) / 2                          # half the smallest subnormal; ties -> 0
        return (Fraction(0), True, h, True) if not negz else (-h, True, Fraction(0), False)
    mag = abs(x)
    i = index_of(mag, name)
    even = (i & 1) == 0
    lo = (value_of(i - 1, name) + mag) / 2
    hi = (mag + value_of(i + 1, name)) / 2 if i < mx else T
    hi_inc = even and i < mx
    if x > 0:
        return (lo, even, hi, hi_inc)
    return (-hi, hi_inc, -lo, even)


def round_exact(x: Fraction, name):
    """Round-to-nearest-even of an exact value: (Fraction, negative_zero) | PINF | NINF."""
    if x == 0:
        return (Fraction(0), False)
    a = abs(x)
    if a >= overflow_threshold(name):
        return PINF if x > 0 else NINF
    ue = _ulp_exp(a, name)
    q = a / Fraction(2) ** ue
    m = math.floor(q)
    rem = q - m
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and m & 1):
        m += 1
    v = Fraction(m) * Fraction(2) ** ue
    return (v, False) if x > 0 else (-v, v == 0)


def literal_value(value, lit_type, target):
    """A literal of `lit_type` as a `target` format value: NAN | PINF | NINF | (Fraction, negz)."""
    if lit_type in ("float", "double"):
        f = float(value)
        if f != f:
            return NAN
        if f in (math.inf, -math.inf):
            return PINF if f > 0 else NINF
        if lit_type == "float":
            f = struct.unpack("<f", struct.pack("<f", f))[0]      # ofFloat keeps a float
        if target == "float" and lit_type == "double":
            raise ValueError("double literal narrowed to float")
        return (Fraction(f), math.copysign(1.0, f) < 0 and f == 0)
    return round_exact(Fraction(int(value)), target)     # int/long widened to float/double


def java_compare(a, b) -> int:
    """Float.compare / Double.compare over NAN | PINF | NINF | (Fraction, negz)."""
    def key(v):
        if v == NAN:
            return (3, 0)
        if v == PINF:
            return (2, 0)
        if v == NINF:
            return (0, 0)
        x, negz = v
        return (1, x, 0 if negz else 1)
    ka, kb = key(a), key(b)
    return (ka > kb) - (ka < kb)


_TEST = {"<": lambda c: c < 0, "<=": lambda c: c <= 0, ">": lambda c: c > 0, ">=": lambda c: c >= 0,
         "=": lambda c: c == 0}


def plan(op: str, lit, lit_type: str, value_fmt: str, cmp_fmt: str):
    """Comparison `round_{value_fmt}(x) <op> literal` compared in cmp_fmt (value_fmt is cmp_fmt or
    float widened to double). Returns (conditions, (nan_result, pinf_result, ninf_result)):
    conditions is a list of ("<"|"<="|">"|">=", Fraction) whose AND holds exactly for the exact
    values x (finite or overflowing) that satisfy it, or [ALL] / [NONE]; the results are those of
    the NaN / +Infinity / -Infinity values."""
    (a, b), specials = rank_run(op, lit, lit_type, value_fmt, cmp_fmt)
    mx = _max_index(value_fmt)
    lo_r, hi_r = -mx - 2, mx + 1
    if a > b:
        return [NONE], specials
    conds = []
    if a > lo_r:
        lo, lo_inc, _, _ = cell(a, value_fmt)
        conds.append((">=" if lo_inc else ">", lo))
    if b < hi_r:
        _, _, hi, hi_inc = cell(b, value_fmt)
        conds.append(("<=" if hi_inc else "<", hi))
    return (conds or [ALL]), specials


def rank(bits: int, name) -> int:
    """Rank of a non-NaN value of the format from its IEEE bits: the bit pattern for +0.0 and up
    (+Infinity is max_index + 1), -1 - |bits| below (-0.0 is -1, -Infinity -max_index - 2) -- the
    Float.compare / Double.compare order."""
    p = FORMATS[name][0]
    sign_bit = 1 << (31 if p == 24 else 63)
    mag = bits & (sign_bit - 1)
    return -mag - 1 if bits & sign_bit else mag


def rank_run(op: str, lit, lit_type: str, value_fmt: str, cmp_fmt: str):
    """The values of value_fmt (as ranks, see rank) whose comparison `value <op> literal` in
    cmp_fmt holds: one contiguous run ((a, b); a > b when empty), plus the NaN / +Infinity /
    -Infinity results."""
    V = literal_value(lit, lit_type, cmp_fmt)
    test = _TEST[op]
    specials = tuple(test(java_compare(s, V)) for s in (NAN, PINF, NINF))
    mx = _max_index(value_fmt)
    lo_r, hi_r = -mx - 2, mx + 1                  # ranks of -Infinity and +Infinity
    # f = the largest rank whose value is <= the literal (total order); exact: equal to it
    if V == NAN:
        f, exact = hi_r + 1, False                # NaN sits above every rank
    elif V == PINF:
        f, exact = hi_r, True
    elif V == NINF:
        f, exact = lo_r, True
    else:
        x, negz = V
        if x == 0:
            f, exact = (-1 if negz else 0), True
        elif x > 0:
            if x > max_finite(value_fmt):
                f, exact = mx, False
            else:
                f = _index_floor(x, value_fmt)
                exact = value_of(f, value_fmt) == x
        else:
            if -x > max_finite(value_fmt):
                f, exact = lo_r, False
            else:
                g = _index_floor(-x, value_fmt)
                exact = value_of(g, value_fmt) == -x
                f = -g - 1 if exact else -g - 2       # the next value below a negative literal
    # the ranks satisfying the comparison form one contiguous run [a, b]
    if op == "<":
        ok = (lo_r, f - 1 if exact else f)
    elif op == "<=":
        ok = (lo_r, f)
    elif op == ">":
        ok = (f + 1, hi_r)
    elif op == ">=":
        ok = (f if exact else f + 1, hi_r)
    else:
        ok = (f, f) if exact else (1, 0)
    ok = (max(ok[0], lo_r), min(ok[1], hi_r))
    if ok[0] > ok[1]:
        ok = (1, 0)
    return ok, specials


def decimal_text(q: Fraction, short=False) -> str:
    """Exact decimal text of a dyadic rational; short: scientific notation when that is shorter
    (thresholds near the subnormal range have hundreds of leading zeros)."""
    n, d = q.numerator, q.denominator
    k = d.bit_length() - 1
    assert d == 1 << k, "not dyadic"
    digits = abs(n) * 5 ** k
    s = str(digits)
    sign = "-" if n < 0 else ""
    plain = s
    if k:
        plain = s.rjust(k + 1, "0")
        plain = plain[:-k] + "." + plain[-k:]
        plain = plain.rstrip("0").rstrip(".")
    if not short or n == 0:
        return sign + plain
    sig = s.rstrip("0")
    exp = len(s) - 1 - k                                 # value = digits * 10^-k
    sci = sig[0] + ("." + sig[1:] if len(sig) > 1 else "") + "E" + str(exp)
    return sign + (sci if len(sci) < len(plain) else plain)


def integral_bounds(conds, lo=-(1 << 63), hi=(1 << 63) - 1):
    """The same conditions over integer x in [lo, hi]: (min, max) inclusive, or None when empty."""
    a, b = lo, hi
    for c in conds:
        if c == ALL:
            continue
        if c == NONE:
            return None
        op, B = c
        if op == "<":
            b = min(b, math.ceil(B) - 1)
        elif op == "<=":
            b = min(b, math.floor(B))
        elif op == ">":
            a = max(a, math.floor(B) + 1)
        else:
            a = max(a, math.ceil(B))
    return (a, b) if a <= b else None
