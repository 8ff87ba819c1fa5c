"""Partition predicates with scalar expressions over partition values, all evaluated on the device
(k_part_eval) as DefaultExpressionEvaluator evaluates them:

* LIKE with a per-row pattern (LikeExpressionEvaluator.java:85-186: the pattern is any string
  expression, the escape a literal; an invalid escape in a row's pattern fails the scan);
* TIMEADD(timestamp, long millis) (DefaultExpressionEvaluator.java:260-288, 593-626: null if either is
  null, ts + millis * 1000 in Java long arithmetic), compared, null-tested, nested;
* arbitrarily deep alternating AND / NOT chains (the compiler emits the deeper operand of AND / OR
  first, so the device stack never overflows).
The CPU tests hold the compiler (dk_part_compile) to status 0 and a bounded stack; the GPU tests hold
the scan files and counters to the oracle (oracle/partitions.py)."""
import json
import os

import pytest

from delta_amd import partitions as pp
from delta_amd import programs
from delta_amd.expressions import Column, Literal, Predicate
from tests.test_partitions import _gpu_files, oracle_files


def col(n):
    return Column(n)


def cmp(op, a, b):
    return Predicate(op, a, b)


FIELDS_SCHEMA = [("ts", "timestamp"), ("ms", "long"), ("s", "string"), ("pat", "string"), ("k", "integer")]


def _write_table(root, rows):
    log = os.path.join(root, "_delta_log")
    os.makedirs(log)
    schema = {"type": "struct", "fields": [{"name": n, "type": t, "nullable": True, "metadata": {}} for n, t in FIELDS_SCHEMA]
              + [{"name": "id", "type": "long", "nullable": True, "metadata": {}}]}
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        f.write(json.dumps({"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}) + "\n")
        f.write(json.dumps({"metaData": {"id": "t", "format": {"provider": "parquet", "options": {}},
                                         "schemaString": json.dumps(schema),
                                         "partitionColumns": [n for n, _ in FIELDS_SCHEMA],
                                         "configuration": {}, "createdTime": 0}}) + "\n")
        for i, pv in enumerate(rows):
            f.write(json.dumps({"add": {"path": "p%d.parquet" % i, "partitionValues": pv, "size": 1,
                                        "modificationTime": 0, "dataChange": True}}) + "\n")


ROWS = [
    {"ts": "2021-09-08 11:11:11", "ms": "1000", "s": "abc", "pat": "a%", "k": "1"},
    {"ts": "2021-09-08 11:11:11", "ms": "-1000", "s": "abc", "pat": "_b_", "k": "2"},
    {"ts": "2021-09-08 11:11:12", "ms": None, "s": "a_c", "pat": "a!_c", "k": "3"},
    {"ts": None, "ms": "5", "s": "xyz", "pat": "%", "k": "4"},
    {"ts": "1970-01-01 00:00:00", "ms": "0", "s": None, "pat": "%", "k": "5"},
    {"ts": "2021-09-08 11:11:10", "ms": "2000", "s": "héllo", "pat": "h_llo", "k": "6"},
    {"ts": "2021-09-08 11:11:11", "ms": "9223372036854775", "s": "100%", "pat": "100!%", "k": "7"},
    {"ts": "2021-09-08 11:11:11", "ms": "1", "s": "", "pat": None, "k": "8"},
    {"ts": "2021-09-08 11:11:11", "ms": "1", "s": "a\\b", "pat": "a\\\\b", "k": "9"},
    {"ts": "2021-09-08 11:11:11", "ms": "1", "s": "abc", "pat": "%c", "k": "10"},
]
T0 = 1631099471000000                        # 2021-09-08 11:11:11 UTC in micros


def predicates():
    ta = Predicate("TIMEADD", col("ts"), col("ms"))
    out = [
        cmp(">", ta, Literal.ofTimestamp(T0)),
        cmp("=", ta, Literal.ofTimestamp(T0 + 1_000_000)),
        cmp("<=", Predicate("TIMEADD", col("ts"), Literal.ofLong(-500)), Literal.ofTimestamp(T0)),
        Predicate("IS_NULL", ta),
        cmp("<", ta, Predicate("TIMEADD", col("ts"), Literal.ofLong(1))),          # wraps for row 7
        cmp("=", Predicate("TIMEADD", ta, Literal.ofLong(1000)), Literal.ofTimestamp(T0 + 2_000_000)),
        Predicate("LIKE", col("s"), col("pat")),
        Predicate("LIKE", col("s"), col("pat"), Literal.ofString("!")),
        Predicate("NOT", Predicate("LIKE", col("s"), col("pat"), Literal.ofString("!"))),
        Predicate("LIKE", col("s"), Predicate("SUBSTRING", col("pat"), Literal.ofInt(1), Literal.ofInt(1))),
        Predicate("AND", Predicate("LIKE", col("s"), col("pat"), Literal.ofString("!")),
                  cmp(">", ta, Literal.ofTimestamp(0))),
    ]
    return out


def deep_chain(depth):
    """AND(NOT(k = i), NOT(AND(NOT(k = i+1), NOT(...)))): nesting `depth` deep on the right."""
    node = cmp(">", col("k"), Literal.ofInt(depth % 10))
    for i in reversed(range(depth)):
        node = Predicate("AND", Predicate("NOT", cmp("=", col("k"), Literal.ofInt(i % 10))), Predicate("NOT", node))
    return node


def _fields():
    schema = {"type": "struct", "fields": [{"name": n, "type": t, "nullable": True, "metadata": {}} for n, t in FIELDS_SCHEMA]}
    return pp.partition_fields(json.dumps(schema), [n for n, _ in FIELDS_SCHEMA])


@pytest.mark.parametrize("i", range(11))
def test_compile_scalar_partition_expressions(i):
    p = programs.compile_partition(predicates()[i], _fields())
    d = p.describe()
    assert d["stack"] <= 32
    p.close()


@pytest.mark.parametrize("depth", [40, 200])
def test_compile_deep_not_chain(depth):
    """An AND / NOT chain far deeper than the 32-slot device stack compiles (deeper operand first)."""
    p = programs.compile_partition(deep_chain(depth), _fields())
    assert p.describe()["stack"] <= 3
    p.close()


def test_oracle_scalar_expressions(tmp_path):
    root = str(tmp_path / "t")
    _write_table(root, ROWS)
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in predicates()]
    # by hand: row 0 is T0 + 1 s; row 1 T0 - 1 s; row 5 T0 + 1 s; row 6 adds 9223372036854775 ms
    # (x1000 wraps negative); rows 7-9 T0 + 1 ms
    assert got[0] == [0, 5, 7, 8, 9] and got[1] == [0, 5]
    assert got[3] == [2, 3]                                   # a null ts or ms: null
    assert got[6] == [0, 1, 3, 5, 8, 9]                       # "a_c" vs "a!_c" no; '\\\\' escapes '\\'
    assert got[7] == [0, 1, 2, 3, 5, 6, 9]                    # with '!' as the escape


@pytest.mark.gpu
def test_gpu_scalar_partition_expressions(tmp_path):
    from delta_amd import kernel as K
    root = str(tmp_path / "t")
    _write_table(root, ROWS)
    eng = K.GpuEngine()
    for p in predicates() + [deep_chain(40), deep_chain(200)]:
        assert _gpu_files(root, p, eng) == oracle_files(root, p), p
    eng.close()


@pytest.mark.gpu
def test_gpu_like_pattern_invalid_escape_fails(tmp_path):
    """A row whose pattern ends in the escape fails the scan (the reference's escapeLikeRegex throws);
    a null input or pattern never reaches it."""
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    from oracle import partitions as opp
    root = str(tmp_path / "t")
    _write_table(root, ROWS[:2] + [{"ts": None, "ms": None, "s": "x", "pat": "ab!", "k": "1"}])
    p = Predicate("LIKE", col("s"), col("pat"), Literal.ofString("!"))
    with pytest.raises(opp.PartitionValueError):
        oracle_files(root, p)
    eng = K.GpuEngine()
    with pytest.raises(DkError, match="partition"):
        _gpu_files(root, p, eng)
    ok = str(tmp_path / "ok")
    _write_table(ok, ROWS[:2] + [{"ts": None, "ms": None, "s": None, "pat": "ab!", "k": "1"}])
    assert _gpu_files(ok, p, eng) == oracle_files(ok, p)
    eng.close()


# ------------------------------------------------------------ float / double between two columns
# ComparatorEvaluator over two float-typed partition values (no literal side, so no threshold can be
# planned on the host): k_part_eval_wide rounds each value's digits to its own type exactly
# (Float.parseFloat / Double.parseDouble), widens (ImplicitCastExpression: integral -> float rounds
# directly, float -> double is exact) and compares with Float.compare / Double.compare.
FP_SCHEMA = [("f", "float"), ("g", "float"), ("d", "double"), ("e", "double"), ("l", "long"), ("i", "integer")]
HALF_F = "1.000000059604644775390625"                  # 1 + 2^-24: halfway between two floats
FP_ROWS = [
    {"f": "1.5", "g": "1.5", "d": "1.5", "e": "1.5", "l": "1", "i": "1"},
    {"f": "0.1", "g": "0.1f", "d": "0.1", "e": "0.1d", "l": "0", "i": "0"},           # (double)0.1f > 0.1
    {"f": HALF_F, "g": "1.0", "d": HALF_F, "e": "1.0000000596046448", "l": "1", "i": "1"},  # ties to even
    {"f": HALF_F + "000001", "g": "1.0000001", "d": "1", "e": "1", "l": "1", "i": "1"},
    {"f": "16777217", "g": "16777216", "d": "16777217", "e": "9007199254740993", "l": "16777217", "i": "16777217"},
    {"f": "9007199254740993", "g": "9.007199254740992E15", "d": "9007199254740993", "e": "9007199254740992",
     "l": "9007199254740993", "i": "-5"},
    {"f": "3.4028235e38", "g": "3.4028236e38", "d": "3.4028235677973366e38", "e": "1e400", "l": "-1", "i": "7"},
    {"f": "1e-45", "g": "7e-46", "d": "1.401298464324817e-45", "e": "2.4703282292062328e-324", "l": "0", "i": "0"},
    {"f": "-0.0", "g": "0", "d": "-0", "e": "1e-400", "l": "0", "i": "0"},
    {"f": "-1e-400", "g": "-0f", "d": "-1e-400", "e": "-0.0", "l": "0", "i": "0"},
    {"f": "NaN", "g": "NaN", "d": "Infinity", "e": "-Infinity", "l": "9223372036854775807", "i": "-2147483648"},
    {"f": None, "g": "2", "d": None, "e": "2.5", "l": None, "i": "3"},
    {"f": " 2.5e0 ", "g": "25E-1", "d": "0.25e1", "e": "2.50000000000000000000000000000000000001", "l": "2", "i": "3"},
    {"f": "1" + "0" * 40 + ".5e-40", "g": "10.00000000000000000000000000000000005", "d": "0." + "0" * 300 + "1e301",
     "e": "0." + "3" * 900, "l": "10", "i": "10"},
    {"f": "4.9e-324", "g": "1.17549435E-38", "d": "2.2250738585072011e-308", "e": "2.2250738585072012e-308",
     "l": "-9223372036854775808", "i": "0"},
]


def _write_fp_table(root, rows):
    log = os.path.join(root, "_delta_log")
    os.makedirs(log)
    schema = {"type": "struct", "fields": [{"name": n, "type": t, "nullable": True, "metadata": {}} for n, t in FP_SCHEMA]
              + [{"name": "id", "type": "long", "nullable": True, "metadata": {}}]}
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        f.write(json.dumps({"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}) + "\n")
        f.write(json.dumps({"metaData": {"id": "t", "format": {"provider": "parquet", "options": {}},
                                         "schemaString": json.dumps(schema),
                                         "partitionColumns": [n for n, _ in FP_SCHEMA],
                                         "configuration": {}, "createdTime": 0}}) + "\n")
        for i, pv in enumerate(rows):
            f.write(json.dumps({"add": {"path": "p%d.parquet" % i, "partitionValues": pv, "size": 1,
                                        "modificationTime": 0, "dataChange": True}}) + "\n")


def fp_predicates():
    out = []
    for a, b in [("f", "g"), ("f", "d"), ("d", "e"), ("g", "e"), ("l", "f"), ("l", "d"), ("i", "f"), ("d", "i"),
                 ("e", "f")]:
        for op in ["<", "<=", "=", ">", ">=", "IS NOT DISTINCT FROM"]:
            out.append(cmp(op, col(a), col(b)))
    out.append(Predicate("NOT", cmp("<", col("f"), col("d"))))
    out.append(Predicate("OR", cmp("=", col("f"), col("g")), cmp(">", col("l"), Literal.ofLong(5))))
    out.append(Predicate("AND", cmp("<=", col("e"), col("d")), cmp("=", col("f"), Literal.ofFloat(1.5))))
    return out


def test_compile_float_column_comparison():
    schema = {"type": "struct", "fields": [{"name": n, "type": t, "nullable": True, "metadata": {}} for n, t in FP_SCHEMA]}
    fields = pp.partition_fields(json.dumps(schema), [n for n, _ in FP_SCHEMA])
    for p in fp_predicates():
        prog = programs.compile_partition(p, fields)
        ops = [o[0] for o in prog.describe()["ops"]]
        assert 23 in ops, p                                        # PO_FCMP2
        prog.close()
    d = programs.compile_partition(cmp("<", col("l"), col("f")), fields).describe()
    # l (integral, form 0) below f (float, form 1), compared as float: PO_LT | 0 << 8 | 0 << 12 | 1 << 16
    assert d["ops"][-1][:2] == [23, 4 | (1 << 16)]


def test_oracle_float_column_comparison(tmp_path):
    root = str(tmp_path / "t")
    _write_fp_table(root, FP_ROWS)
    def ids(p):
        return sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0])
    assert 1 in ids(cmp(">", col("f"), col("d")))          # (double)0.1f = 0.100000001490116...
    assert 2 in ids(cmp("=", col("f"), col("g")))          # 1 + 2^-24 ties to 1.0f
    assert 3 in ids(cmp(">", col("f"), col("g"))) or 3 in ids(cmp("=", col("f"), col("g")))
    assert 4 in ids(cmp("=", col("l"), col("f")))          # (float)16777217L == 16777216f == parse("16777217")
    assert 8 in ids(cmp("<", col("f"), col("g")))          # -0.0f < 0.0f
    assert 10 in ids(cmp("=", col("f"), col("g")))         # NaN == NaN under Float.compare


@pytest.mark.gpu
def test_gpu_float_column_comparison(tmp_path):
    from delta_amd import kernel as K
    root = str(tmp_path / "t")
    _write_fp_table(root, FP_ROWS)
    eng = K.GpuEngine()
    for p in fp_predicates():
        assert _gpu_files(root, p, eng) == oracle_files(root, p), p
    eng.close()


def _halfway_rows(n, seed):
    """Rows whose f / d values sit exactly on, just above or just below the midpoint between two
    adjacent floats / doubles (written out in full: up to ~770 significant digits for doubles near
    the subnormal range), and whose g / e values are the lower neighbour's shortest repr."""
    import random
    import struct
    from fractions import Fraction
    import numpy as np
    rnd = random.Random(seed)

    def full(q):                              # exact decimal text of a dyadic rational
        num, den = q.numerator, q.denominator
        k = den.bit_length() - 1
        digits = str(num * 5 ** k)
        if k == 0:
            return digits
        digits = digits.rjust(k + 1, "0")
        return digits[:-k] + "." + digits[-k:]

    def variant(mid):
        t = full(mid)
        v = rnd.randrange(3)
        if v == 1:
            return t + ("1" if "." in t else ".1")
        if v == 2 and t.endswith("5"):
            return t[:-1] + "4999"
        return t

    rows = []
    for _ in range(n):
        e32 = rnd.choice([rnd.randrange(0, 255), 0, 1, 254])
        b32 = (e32 << 23) | rnd.getrandbits(23)
        lo32 = struct.unpack("<f", struct.pack("<I", b32))[0]
        hi32 = struct.unpack("<f", struct.pack("<I", b32 + 1))[0] if b32 + 1 < 0x7f800000 else None
        e64 = rnd.choice([rnd.randrange(0, 2047), 0, 1, 2046, rnd.randrange(1000, 1100)])
        b64 = (e64 << 52) | rnd.getrandbits(52)
        lo64 = struct.unpack("<d", struct.pack("<Q", b64))[0]
        hi64 = struct.unpack("<d", struct.pack("<Q", b64 + 1))[0] if b64 + 1 < 0x7ff0000000000000 else None
        f = variant((Fraction(lo32) + Fraction(hi32)) / 2) if hi32 is not None else repr(lo32)
        d = variant((Fraction(lo64) + Fraction(hi64)) / 2) if hi64 is not None else repr(lo64)
        rows.append({"f": f, "g": str(np.float32(lo32)),
                     "d": d, "e": repr(lo64), "l": str(rnd.getrandbits(63)), "i": str(rnd.getrandbits(24))})
    return rows


@pytest.mark.gpu
def test_gpu_float_halfway_rounding(tmp_path):
    """Round-to-nearest-even on exact and near-halfway decimal inputs, against the oracle's exact
    rational rounding (Fraction -> binary32 / binary64)."""
    from delta_amd import kernel as K
    root = str(tmp_path / "t")
    _write_fp_table(root, _halfway_rows(600, 7))
    eng = K.GpuEngine()
    preds = [cmp("=", col("f"), col("g")), cmp(">", col("f"), col("g")), cmp("=", col("d"), col("e")),
             cmp(">", col("d"), col("e")), cmp("<", col("f"), col("d")), cmp("=", col("l"), col("d")),
             cmp("<", col("i"), col("f"))]
    for p in preds:
        got, want = _gpu_files(root, p, eng), oracle_files(root, p)
        assert got == want, p
    eng.close()


def test_halfway_rows_oracle_split(tmp_path):
    """The generated rows hit both sides: some round down onto the lower neighbour, some up."""
    root = str(tmp_path / "t")
    _write_fp_table(root, _halfway_rows(200, 7))
    eq = len(oracle_files(root, cmp("=", col("d"), col("e")))[0])
    gt = len(oracle_files(root, cmp(">", col("d"), col("e")))[0])
    assert 20 < eq < 180 and 20 < gt < 180 and eq + gt == 200
