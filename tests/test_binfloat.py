"""delta_amd/binfloat.py (the planner's exact float / double comparison thresholds) against the
oracle's independent rounding and Float.compare / Double.compare (oracle/skipping.py): for random
literals and exact values around every planned threshold, `x satisfies the planned bounds` must equal
`Float.compare(round(x), literal) <op> 0`."""
import math
import random
import struct
from fractions import Fraction

import pytest

from tests import binfloat_ref as bf


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


_UP = {"byte": {"short", "integer", "long", "float", "double"}, "short": {"integer", "long", "float", "double"},
       "integer": {"long", "float", "double"}, "long": {"float", "double"}, "float": {"double"}}


def _expected_ops(op, st, lt, v):
    """The float comparison as the reference planner (tests/binfloat_ref.py) plans it: FCMP entries
    (mode | flags, threshold text, rank run) for a float / double stat, integer bounds otherwise."""
    from delta_amd import skipping as sk
    cmp_t = st if st == lt else (lt if lt in _UP.get(st, ()) else st)
    value_fmt = st if st in ("float", "double") else cmp_t
    conds, (r_nan, r_pinf, r_ninf) = bf.plan(op, v, lt, value_fmt, cmp_t)
    ranks = bf.rank_run(op, v, lt, value_fmt, cmp_t)[0]
    if st not in ("float", "double"):
        b = bf.integral_bounds(conds)
        if b is None:
            return [("int", sk.OP_LT, -(1 << 63))]
        parts = ([("int", sk.OP_GE, b[0])] if b[0] > -(1 << 63) else []) + \
            ([("int", sk.OP_LE, b[1])] if b[1] < (1 << 63) - 1 else [])
        return parts or [("int", sk.OP_GE, -(1 << 63))]
    flags = (int(r_nan) << 4) | (int(r_pinf) << 5) | (int(r_ninf) << 6)
    modes = {"<": sk.FC_LT, "<=": sk.FC_LE, ">": sk.FC_GT, ">=": sk.FC_GE}
    out = []
    for c in conds:
        if c in (bf.ALL, bf.NONE):
            out.append(("fcmp", flags | (sk.FC_ALL if c == bf.ALL else sk.FC_NONE), b"", tuple(ranks)))
        else:
            out.append(("fcmp", flags | modes[c[0]], bf.decimal_text(c[1], short=True).encode(), tuple(ranks)))
    return out


def test_cpp_planner_matches_reference_planner():
    """The float / double planning behind the C ABI (dk_expr.cpp: exact dyadic arithmetic) emits the
    same thresholds, rank runs and integer bounds as the reference planner tests/binfloat_ref.py
    (itself checked against the oracle's rounding above), over random and edge literals, all operators
    and every stat / literal type pair the reference compares."""
    from delta_amd import skipping as sk
    from tests.test_skipping import _compiled
    rnd = random.Random(11)
    specials = [0.0, -0.0, 1.5, -1.5, 0.1, 1e-45, 1.4e-45, 5e-324, 2.2250738585072014e-308, 3.4028234663852886e38,
                1.7976931348623157e308, 16777217.0, 9007199254740993.0, float("inf"), float("-inf"), float("nan"),
                1e30, -1e-30, 2.0 ** 63, -(2.0 ** 63), 2.0 ** 64]
    pairs = [("float", "float"), ("double", "double"), ("float", "double"), ("long", "float"), ("long", "double"),
             ("integer", "float"), ("short", "double"), ("byte", "float"), ("float", "long"), ("double", "integer")]
    n = 0
    for st, lt in pairs:
        leaves = {("c",): (st, ("c",))}
        for _ in range(60):
            if lt in ("float", "double"):
                v = rnd.choice(specials) if rnd.random() < 0.5 else rnd.uniform(-1e6, 1e6) * 10.0 ** rnd.randint(-40, 40)
                if lt == "float":
                    v = struct.unpack("<f", struct.pack("<f", v if abs(v) < 3.5e38 or v != v or math.isinf(v) else 1e38))[0]
            else:
                v = rnd.choice([0, 1, -1, 16777217, 2 ** 53 + 1, 2 ** 63 - 1, -(2 ** 63), rnd.randint(-2 ** 62, 2 ** 62)])
                if lt == "integer":
                    v = max(-(2 ** 31), min(2 ** 31 - 1, v))
            for op in ("<", "<=", ">", ">=", "="):
                node = (op, ("stat", ("minValues", "c")), ("lit", v, lt))
                _, _, ops = _compiled(node, leaves)
                want = _expected_ops(op, st, lt, v)
                if st in ("float", "double"):
                    got = [("fcmp", o[1], o[3], o[4]) for o in ops if o[0] == sk.OP_FCMP]
                else:
                    lits = [o for o in ops if o[0] == sk.OP_LIT]
                    cmps = [o for o in ops if o[0] in (sk.OP_LT, sk.OP_LE, sk.OP_GE, sk.OP_GT)]
                    got = [("int", c[0], l[2]) for l, c in zip(lits, cmps)]
                assert got == want, (st, lt, v, op, got, want)
                n += 1
    assert n == len(pairs) * 60 * 5
