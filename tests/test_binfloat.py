"""delta_amd/binfloat.py (the planner's exact float / double comparison thresholds) against the
oracle's independent rounding and Float.compare / Double.compare (oracle/skipping.py): for random
literals and exact values around every planned threshold, `x satisfies the planned bounds` must equal
`Float.compare(round(x), literal) <op> 0`."""
import math
import random
import struct
from fractions import Fraction

import pytest

from delta_amd import binfloat as bf


def _holds(conds, x):
    for c in conds:
        if c == bf.ALL:
            continue
        if c == bf.NONE:
            return False
        op, b = c
        if not {"<": x < b, "<=": x <= b, ">": x > b, ">=": x >= b}[op]:
            return False
    return True


def _oracle_round(x, fmt):
    from oracle import skipping as osk
    if x == 0:
        return 0.0
    if fmt == "float":
        return osk._to_float32(x)
    try:
        return x.numerator / x.denominator            # int / int: correctly rounded
    except OverflowError:
        return math.inf if x > 0 else -math.inf


def _literals(rng):
    out = [0.0, -0.0, 1.5, -1.5, 0.1, 1e-45, -1e-45, 3.4028234663852886e38, math.inf, -math.inf, math.nan,
           16777216.0, 16777217.0, 5e-324, 1.7976931348623157e308]
    out += [struct.unpack("<f", struct.pack("<I", rng.getrandbits(32)))[0] for _ in range(25)]
    out += [struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0] for _ in range(10)]
    return out


@pytest.mark.parametrize("lit_t,value_fmt,cmp_fmt", [("float", "float", "float"), ("double", "float", "double"),
                                                     ("float", "double", "double"), ("double", "double", "double"),
                                                     ("long", "float", "float"), ("long", "double", "double")])
def test_plan_matches_oracle(lit_t, value_fmt, cmp_fmt):
    from oracle import skipping as osk
    rng = random.Random(hash((lit_t, value_fmt, cmp_fmt)) & 0xffff)
    for lit in _literals(rng):
        if lit_t == "long":
            if lit != lit or math.isinf(lit) or abs(lit) >= 2 ** 63:
                continue
            lit = int(lit)
        if lit_t == "float" and not math.isinf(lit) and lit == lit and abs(lit) > 3.4028234663852886e38:
            continue
        lv = osk._cast(lit, lit_t, cmp_fmt) if lit_t == "long" else \
            (struct.unpack("<f", struct.pack("<f", lit))[0] if lit_t == "float" else lit)
        for op in ("<", "<=", ">", ">=", "="):
            conds, specials = bf.plan(op, lit, lit_t, value_fmt, cmp_fmt)
            test = {"<": lambda c: c < 0, "<=": lambda c: c <= 0, ">": lambda c: c > 0, ">=": lambda c: c >= 0,
                    "=": lambda c: c == 0}[op]
            for sv, got in zip((math.nan, math.inf, -math.inf), specials):
                assert got == test(osk._java_compare(sv, lv))
            xs = [Fraction(0), Fraction(-1, 10 ** 60), Fraction(1, 10 ** 60)]
            for c in conds:
                if isinstance(c, tuple):
                    e = Fraction(1, 2 ** 1100)
                    xs += [c[1], c[1] + e, c[1] - e]
            if lv == lv and not math.isinf(lv):
                xs += [Fraction(lv), Fraction(lv) + Fraction(1, 2 ** 1100), Fraction(lv) - Fraction(1, 2 ** 1100)]
            xs += [Fraction(rng.uniform(-4, 4)).limit_denominator(999) * Fraction(10) ** rng.randint(-60, 60)
                   for _ in range(10)]
            for x in xs:
                r = _oracle_round(x, value_fmt)
                want = test(osk._java_compare(r, lv))
                assert _holds(conds, x) == want, (op, lit, x, conds)


def test_decimal_text_is_exact():
    for q in (Fraction(3, 2), Fraction(-1, 2 ** 60), Fraction(2 ** 70 + 1, 1), bf.overflow_threshold("float")):
        assert Fraction(bf.decimal_text(q)) == q
    assert bf.decimal_text(bf.overflow_threshold("float")) == "340282356779733661637539395458142568448"
