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
