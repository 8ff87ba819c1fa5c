"""K11 data skipping (delta_amd/skipping.py planner, k_stats_eval on the GPU, oracle/skipping.py).

Pinned to the reference's own expectations on its golden tables (KDT = kernel-defaults/src/test/scala/
io/delta/kernel/defaults):
  ScanSuite.scala:1150-1196  basic data skipping for all types (+ column mapping name/id, checkpoint):
                             hits / misses for int, long, byte, short, float, double, date, string
                             and decimal
  ScanSuite.scala:1198-1212  implicit casting (short column vs float literal, float column vs short)
  ScanSuite.scala:846-887    float / double columns with float literals (Spark-style stats)
  ScanSuite.scala:1233-1239  filter on a non-existent column -> no skipping
  ScanSuite.scala:1243-1253  AND of two data columns -> 1 file
  ScanSuite.scala:1255-1267  stats collected changing across versions -> 1 / 2 / 1 files
  ScanSuite.scala:1508-1545  referenced stats columns per predicate
GPU tests compare the product's ordered scan files and counters with the oracle on the same tables,
on synthetic tables with stats (commit tail + checkpoint), and on hand-written stats JSON edge cases.
"""
import json
import os

import pytest

from delta_amd import skipping as sk
from delta_amd import synth
from delta_amd.expressions import ALWAYS_TRUE, And, Column, Literal, Or, Predicate
from tests.golden_util import TABLES

ALL_TYPES = ["data-skipping-basic-stats-all-types", "data-skipping-basic-stats-all-types-columnmapping-name",
             "data-skipping-basic-stats-all-types-columnmapping-id",
             "data-skipping-basic-stats-all-types-checkpoint"]
INTEGRAL = {"as_int": Literal.ofInt, "as_long": Literal.ofLong, "as_byte": Literal.ofByte,
            "as_short": Literal.ofShort}


def col(n):
    return Column(n)


def cmp(op, c, v):
    return Predicate(op, c, v)


def _days(text):
    import datetime
    return (datetime.date.fromisoformat(text) - datetime.date(1970, 1, 1)).days


# ScanSuite.scala:1158-1160: as_date value 2000-01-01, smaller 1999-01-01, bigger 2000-01-02
DATES = tuple(Literal.ofDate(_days(t)) for t in ("2000-01-01", "1999-01-01", "2000-01-02"))


def all_types_hits_misses():
    """ScanSuite.scala:1150-1183: value in table 0, smaller -1, bigger 1 (dates: DATES)."""
    hits, misses = [], []
    cases = [(name, lit(0), lit(-1), lit(1)) for name, lit in INTEGRAL.items()] + [("as_date",) + DATES]
    cases.append(("as_string", Literal.ofString("0"), Literal.ofString("!"), Literal.ofString("1")))   # :1157
    cases.append(("as_big_decimal",) + tuple(Literal.ofDecimal(v, 1, 0) for v in (0, -1, 1)))        # :1162-1164
    cases.append(("as_float",) + tuple(Literal.ofFloat(v) for v in (0, -1, 1)))                      # :1155
    cases.append(("as_double",) + tuple(Literal.ofDouble(v) for v in (0, -1, 1)))                    # :1156
    for name, value, small, big in cases:
        c = col(name)
        misses += [cmp("=", c, small), cmp(">", c, value), cmp(">=", c, big), cmp("<", c, value),
                   cmp("<=", c, small)]
        hits += [cmp("=", c, value), cmp(">", c, small), cmp(">=", c, value), cmp("<", c, big),
                 cmp("<=", c, value)]
    return hits, misses


def table_metadata(root):
    """(schemaString, partitionColumns) of the latest metaData in the table's commits (or its
    checkpoint when the commits carry none)."""
    log = os.path.join(root, "_delta_log")
    md = None
    for f in sorted(os.listdir(log)):
        if f.endswith(".json"):
            with open(os.path.join(log, f)) as fh:
                for line in fh:
                    o = json.loads(line)
                    if o.get("metaData"):
                        md = o["metaData"]
    if md is None:
        import pyarrow.parquet as pq
        for f in sorted(os.listdir(log)):
            if ".checkpoint" in f and f.endswith(".parquet"):
                t = pq.read_table(os.path.join(log, f), columns=["metaData"]).column(0).to_pylist()
                md = next((x for x in t if x), md)
    return md["schemaString"], md.get("partitionColumns") or []


def oracle_skipping(root, predicate):
    """The oracle's own skipping predicate (oracle/skipping_filter.py restates
    constructDataSkippingFilter; the product planner is not used) and its stats types."""
    from oracle import skipping_filter as osf
    schema, parts = table_metadata(root)
    pf, data = osf.split(predicate, parts)
    assert pf is None
    if data is None:
        return None
    S = osf.StatsSchema(schema, parts)
    node = osf.build(data, S)
    if node is None:
        return None
    osf.check(node, S)
    return node, osf.stat_types(node, S)


def oracle_files(root, predicate, bs=1024):
    from oracle import ref
    r = ref.replay(root, json_batch_size=bs, with_stats=True, skipping=oracle_skipping(root, predicate))
    return r.scan_files(), r.counters.as_tuple()


# ---------------------------------------------------------------- planner (host logic, CPU)
def test_split_filters():
    p = And(cmp(">", col("part"), Literal.ofInt(0)), cmp(">", col("id"), Literal.ofInt(0)))
    a, b = sk.split_filters(p, ["PART"])
    assert a == cmp(">", col("part"), Literal.ofInt(0)) and b == cmp(">", col("id"), Literal.ofInt(0))
    a, b = sk.split_filters(Or(cmp(">", col("part"), Literal.ofInt(0)), cmp(">", col("id"), Literal.ofInt(0))),
                            ["part"])
    assert a is None and b.name == "OR"
    assert sk.split_filters(ALWAYS_TRUE, []) == (None, None)
    # literal-only predicates have no non-partition column: they go to the partition side
    assert sk.split_filters(cmp("=", Literal.ofInt(1), Literal.ofInt(1)), [])[1] is None


def test_referenced_stats_match_reference():
    # ScanSuite.scala:1527-1538
    schema, parts = table_metadata(os.path.join(TABLES, "data-skipping-basic-stats-all-types"))
    leaves = sk.data_schema_leaves(schema, parts)
    z = Literal.ofInt(0)
    cases = [(cmp("=", col("as_int"), z), {("minValues", "as_int"), ("maxValues", "as_int")}),
             (cmp("<", col("as_int"), z), {("minValues", "as_int")}),
             (cmp(">", col("as_int"), z), {("maxValues", "as_int")}),
             (cmp(">=", col("as_int"), z), {("maxValues", "as_int")}),
             (cmp("<=", col("as_int"), z), {("minValues", "as_int")}),
             (And(cmp("<", col("as_int"), z), cmp(">", col("as_long"), z)),
              {("minValues", "as_int"), ("maxValues", "as_long")})]
    for p, want in cases:
        assert set(sk.referenced_stats(sk.construct(p, leaves))) == want


def test_construct_rules():
    leaves = {("a",): ("long", ("a",)), ("b",): ("integer", ("col-b",)), ("m",): ("map", ("m",))}
    v = Literal.ofLong(5)
    # literal on the left is reversed; OR needs both sides; AND keeps one side
    assert sk.construct(cmp("<", v, col("a")), leaves) == (">", ("stat", ("maxValues", "a")), ("lit", 5, "long"))
    assert sk.construct(Or(cmp("<", col("a"), v), cmp("<", col("m"), v)), leaves) is None
    assert sk.construct(And(cmp("<", col("a"), v), cmp("<", col("m"), v)), leaves) == \
        ("<", ("stat", ("minValues", "a")), ("lit", 5, "long"))
    # physical names; IS_NULL / IS_NOT_NULL use nullCount and numRecords
    assert sk.construct(Predicate("IS_NOT_NULL", col("b")), leaves) == \
        ("<", ("stat", ("nullCount", "col-b")), ("stat", ("numRecords",)))
    assert sk.construct(Predicate("NOT", Predicate("IS_NOT_NULL", col("b"))), leaves) == \
        (">", ("stat", ("nullCount", "col-b")), ("lit", 0, "long"))
    # NOT(a = 5) -> min < 5 OR max > 5; NOT(a < 5) -> max >= 5
    assert sk.construct(Predicate("NOT", cmp("=", col("a"), v)), leaves) == \
        ("OR", ("<", ("stat", ("minValues", "a")), ("lit", 5, "long")), (">", ("stat", ("maxValues", "a")), ("lit", 5, "long")))
    assert sk.construct(Predicate("NOT", cmp("<", col("a"), v)), leaves) == \
        (">=", ("stat", ("maxValues", "a")), ("lit", 5, "long"))
    # IS NOT DISTINCT FROM null -> IS_NULL
    assert sk.construct(cmp("IS NOT DISTINCT FROM", col("a"), Literal.ofNull("long")), leaves) == \
        (">", ("stat", ("nullCount", "a")), ("lit", 0, "long"))
    # non-existent column: no skipping (ScanSuite.scala:1233-1239)
    assert sk.construct(cmp("=", col("foo"), Literal.ofInt(1)), leaves) is None


@pytest.mark.parametrize("coltype,lit,ok", [
    ("integer", Literal.ofLong(5), True),            # int -> long up-cast
    ("long", Literal.ofInt(5), True),
    ("byte", Literal.ofShort(5), True),
    ("long", Literal.ofLong(5), True),
    ("date", Literal.ofDate(5), True),
    ("timestamp_ntz", Literal.ofTimestamp(5), False),
    ("timestamp", Literal.ofTimestampNtz(5), False),
    ("date", Literal.ofTimestamp(5), False),
    ("date", Literal.ofLong(5), False),
    ("timestamp_ntz", Literal.ofLong(5), False),
    ("decimal(10,2)", Literal.ofDecimal("1.5", 10, 2), True),
    ("decimal(10,2)", Literal.ofDecimal("1.5", 5, 1), False),    # DecimalType.equals: precision + scale
    ("string", Literal.ofInt(5), False),
])
def test_comparator_types(coltype, lit, ok):
    """DefaultExpressionEvaluator.transformBinaryComparator (:337-354): only ImplicitCastExpression
    .canCastTo up-casts make differently typed operands comparable; other pairs throw."""
    leaves = {("a",): (coltype, ("a",))}
    node = sk.construct(cmp(">", col("a"), lit), leaves)
    if ok:
        sk.check_types(node, leaves)
    else:
        with pytest.raises(sk.UnsupportedExpression, match="operands are of different types"):
            sk.check_types(node, leaves)


def _compiled(node, leaves):
    """dk_skip_compile of a constructed predicate (delta_amd/programs.py) as (paths, type codes, ops)
    with each op's literal bytes decoded from the program's pool: (op, arg, lit, bytes | None, ranks | None)."""
    import struct
    from delta_amd import programs
    d = programs.compile_skipping(node, leaves).describe()
    pool = bytes.fromhex(d["pool"])
    ops = []
    for op, arg, lit in d["ops"]:
        if op in (sk.OP_LIT_STR, sk.OP_LIT_DEC):
            ops.append((op, arg, lit, pool[lit:lit + arg], None))
        elif op == sk.OP_FCMP:
            off, ln = lit & 0xffffffff, lit >> 32
            ops.append((op, arg, lit, pool[off:off + ln], struct.unpack("<qq", pool[off + ln:off + ln + 16])))
        else:
            ops.append((op, arg, lit, None, None))
    return [tuple(p["path"]) for p in d["paths"]], [p["type"] for p in d["paths"]], ops


def test_compile_refuses_unsupported():
    """The compiler behind the C ABI (dk_skip_compile) applies transformBinaryComparator's type check
    itself (status 3 -> UnsupportedExpression), and compiles an equality to min <= v AND max >= v."""
    leaves = {("f",): ("float", ("f",)), ("s",): ("string", ("s",)), ("a",): ("long", ("a",))}
    for p in (cmp("=", col("s"), Literal.ofInt(1)), cmp("=", col("a"), Literal.ofString("1"))):
        node = sk.construct(p, leaves)
        assert node is not None
        with pytest.raises(sk.UnsupportedExpression, match="operands are of different types"):
            _compiled(node, leaves)
    node = sk.construct(cmp("=", col("a"), Literal.ofLong(3)), leaves)
    paths, types, ops = _compiled(node, leaves)
    assert paths == [("minValues", "a"), ("maxValues", "a")] and types == [0, 0]
    assert [o[0] for o in ops] == [sk.OP_STAT, sk.OP_LIT, sk.OP_LE, sk.OP_STAT, sk.OP_LIT, sk.OP_GE, sk.OP_AND]


def test_compile_float_comparisons():
    """Float / double comparisons compile to exact thresholds: a float stat gets OP_FCMP against the
    rounding-cell edge, an integral stat widened to float integer bounds."""
    leaves = {("f",): ("float", ("f",)), ("a",): ("long", ("a",)), ("d",): ("double", ("d",))}
    paths, types, ops = _compiled(sk.construct(cmp("<", col("f"), Literal.ofFloat(1.5)), leaves), leaves)
    assert types == [9] and [o[0] for o in ops] == [sk.OP_STAT, sk.OP_FCMP]
    # round_float(x) < 1.5f  <=>  x < 1.5 - 2^-24 (the tie goes to the even neighbour 1.5)
    assert ops[1][1] & 15 == sk.FC_LT and ops[1][3] == b"1.499999940395355224609375"
    assert ops[1][1] >> 4 == 0b100                       # NaN: false, +Inf: false, -Inf: true
    # long column = float literal 2^24 + 1 (stored as 16777216f): min <= V holds for the longs that
    # round to at most 16777216f (x <= 16777217, the tie rounds to even), max >= V for x >= 16777216
    _, _, ops = _compiled(sk.construct(cmp("=", col("a"), Literal.ofFloat(16777217)), leaves), leaves)
    assert [(o[0], o[2]) for o in ops if o[0] in (sk.OP_LIT, sk.OP_LE, sk.OP_GE)] == \
        [(sk.OP_LIT, 16777217), (sk.OP_LE, 0), (sk.OP_LIT, 16777216), (sk.OP_GE, 0)]
    # double column vs NaN literal: < holds for every non-NaN value
    _, _, ops = _compiled(sk.construct(cmp("<", col("d"), Literal.ofDouble(float("nan"))), leaves), leaves)
    assert ops[1][0] == sk.OP_FCMP and ops[1][1] & 15 == sk.FC_ALL and ops[1][1] >> 4 == 0b110


def test_oracle_date_decoding_rules():
    """java.sql.Date.valueOf + daysSinceEpoch (DefaultJsonRow.java:249-252): 1-2 char month/day, a
    '+' sign on a field, lenient day carry; bad shapes and pre-1583 years raise."""
    from oracle import skipping as osk
    t = {("minValues", "d"): "date"}
    for text, want in (("2000-01-01", "2000-01-01"), ("2000-1-2", "2000-01-02"), ("2021-02-30", "2021-03-02"),
                       ("2020-02-30", "2020-03-01"), ("2000-+1-+9", "2000-01-09"), ("1970-01-01", "1970-01-01"),
                       ("1583-01-01", "1583-01-01"), ("9999-12-31", "9999-12-31")):
        got = osk.decode_stats('{"minValues":{"d":"%s"}}' % text, t)[("minValues", "d")]
        assert got == _days(want), text
    for bad in ("2000-13-01", "2000-00-10", "2000-01-32", "2000-01-0", "200-01-01", "2000-001-01",
                "2000/01/01", "2000-01-", "-999-01-01", "1582-12-31", "+999-01-01", "2000-01-+",
                "2000-01-01T00", ""):
        with pytest.raises(osk.StatsDecodeError):
            osk.decode_stats('{"minValues":{"d":"%s"}}' % bad, t)
    for bad in ('{"minValues":{"d":10957}}', '{"minValues":{"d":true}}'):
        with pytest.raises(osk.StatsDecodeError):
            osk.decode_stats(bad, t)


def test_program_paths():
    """A nested column-mapped stats path keeps its physical components (the add.stats_parsed leaf)."""
    leaves = {("s", "x"): ("short", ("col-s", "col-x"))}
    paths, types, _ = _compiled(sk.construct(cmp(">", Column("s", "x"), Literal.ofShort(3)), leaves), leaves)
    assert paths == [("maxValues", "col-s", "col-x")] and types == [2]


# ---------------------------------------------------------------- oracle (pinned to the reference)
def test_oracle_stats_decoding_rules():
    from oracle import skipping as osk
    t = {("minValues", "x"): "short", ("maxValues", "y"): "long", ("numRecords",): "long"}
    d = osk.decode_stats('{"numRecords":7,"minValues":{"x":5.0E0},"maxValues":{"y":-3}} trailing', t)
    assert d == {("minValues", "x"): 5, ("maxValues", "y"): -3, ("numRecords",): 7}
    assert osk.decode_stats('{"minValues":null,"numRecords":1,"numRecords":2}', t) == \
        {("minValues", "x"): None, ("maxValues", "y"): None, ("numRecords",): 2}
    for bad in ('{"maxValues":{"y":1.0}}', '{"minValues":{"x":5.5}}', '{"minValues":{"x":40000}}',
                '{"minValues":3}', '{"numRecords":"1"}', '[]', '', '{"numRecords":true}',
                '{"maxValues":{"y":9223372036854775808}}', '{"numRecords":01}'):
        with pytest.raises(osk.StatsDecodeError):
            osk.decode_stats(bad, t)


@pytest.mark.parametrize("name", ALL_TYPES)
def test_oracle_all_types_hits_and_misses(name):
    root = os.path.join(TABLES, name)
    hits, misses = all_types_hits_misses()
    for p in hits:
        assert oracle_files(root, p, bs=2)[0], ("expected hit", name, p)
    for p in misses:
        assert not oracle_files(root, p, bs=2)[0], ("expected miss", name, p)


def test_oracle_non_existent_column_and_counts():
    root = os.path.join(TABLES, "data-skipping-basic-stats-all-types")
    assert oracle_files(root, cmp("=", col("foo"), Literal.ofInt(1)))[0]
    root = os.path.join(TABLES, "data-skipping-partition-and-data-column")
    p = And(cmp(">", col("part"), Literal.ofInt(0)), cmp(">", col("id"), Literal.ofInt(0)))
    assert len(oracle_files(root, p)[0]) == 1
    root = os.path.join(TABLES, "data-skipping-change-stats-collected-across-versions")
    for p, n in ((cmp("=", col("col1"), Literal.ofInt(1)), 1), (cmp("=", col("col2"), Literal.ofInt(1)), 2),
                 (And(cmp("=", col("col1"), Literal.ofInt(1)), cmp("=", col("col2"), Literal.ofInt(1))), 1)):
        assert len(oracle_files(root, p)[0]) == n, p


def test_oracle_skipping_leaves_counters_unchanged(tmp_path):
    from oracle import ref
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=3_000, n_parts=2, n_commits=4, dv_frac=0.1,
                                                     ckpt_removes=20, with_stats=True))
    full = ref.replay(str(tmp_path), with_stats=True)
    files, counters = oracle_files(str(tmp_path), cmp(">", col("id"), Literal.ofLong(30_000_000)))
    assert counters == full.counters.as_tuple()
    assert 0 < len(files) < len(full.scan_files())


# ---------------------------------------------------------------- GPU parity
def _gpu_files(root, predicate, eng):
    from delta_amd import kernel as K
    from oracle import ref
    snap = K.Table.forPath(eng, root).getLatestSnapshot(eng)
    scan = snap.getScanBuilder().withFilter(predicate).build()
    try:
        rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in scan.getScanFiles(eng)
                for i in b.selected_rows()]
        return rows, scan.metrics.as_tuple()
    finally:
        scan.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ALL_TYPES)
def test_gpu_all_types_hits_and_misses(name):
    from delta_amd import kernel as K
    root = os.path.join(TABLES, name)
    eng = K.GpuEngine(json_batch_size=2)
    hits, misses = all_types_hits_misses()
    for p in hits + misses:
        g = _gpu_files(root, p, eng)
        o = oracle_files(root, p, bs=2)
        assert g == o, (name, p)
        assert bool(g[0]) == (p in hits), (name, p)
    eng.close()


@pytest.mark.gpu
def test_gpu_golden_counts():
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    root = os.path.join(TABLES, "data-skipping-partition-and-data-column")
    p = And(cmp(">", col("part"), Literal.ofInt(0)), cmp(">", col("id"), Literal.ofInt(0)))
    assert len(_gpu_files(root, p, eng)[0]) == 1
    root = os.path.join(TABLES, "data-skipping-change-stats-collected-across-versions")
    for p, n in ((cmp("=", col("col1"), Literal.ofInt(1)), 1), (cmp("=", col("col2"), Literal.ofInt(1)), 2),
                 (And(cmp("=", col("col1"), Literal.ofInt(1)), cmp("=", col("col2"), Literal.ofInt(1))), 1)):
        g = _gpu_files(root, p, eng)
        assert len(g[0]) == n and g == oracle_files(root, p), p
    eng.close()


SYNTH_PREDICATES = [
    cmp(">", col("id"), Literal.ofLong(30_000_000)),
    cmp("<=", col("id"), Literal.ofInt(20_000_000)),
    cmp("=", col("id"), Literal.ofLong(25_000_123)),
    And(cmp(">=", col("id"), Literal.ofLong(15_000_000)), cmp("<", col("id"), Literal.ofLong(35_000_000))),
    Or(cmp("<", col("id"), Literal.ofLong(12_000_000)), cmp(">", col("id"), Literal.ofLong(48_000_000))),
    Predicate("NOT", cmp("<", col("id"), Literal.ofLong(40_000_000))),
    Predicate("IS_NOT_NULL", col("id")),
    Predicate("IS_NULL", col("id")),
    cmp("IS NOT DISTINCT FROM", col("id"), Literal.ofLong(33_333_333)),
]


@pytest.mark.gpu
def test_gpu_synthetic_parity(tmp_path):
    from delta_amd import kernel as K
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=40_000, n_parts=3, n_commits=6, dv_frac=0.2,
                                                     ckpt_removes=200, with_stats=True))
    eng = K.GpuEngine()
    for p in SYNTH_PREDICATES:
        g = _gpu_files(str(tmp_path), p, eng)
        o = oracle_files(str(tmp_path), p)
        assert g[1] == o[1], p
        assert len(g[0]) == len(o[0]) and g[0] == o[0], p
    eng.close()


def _write_edge_table(root, stats_list, columns=(("x", "short"), ("id", "long"))):
    """A commit-only table whose adds carry the given raw stats strings (None = no stats)."""
    log = os.path.join(root, "_delta_log")
    os.makedirs(log)
    schema = {"type": "struct", "fields": [{"name": n, "type": t, "nullable": True, "metadata": {}}
                                           for n, t in columns]}
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        f.write(json.dumps({"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}) + "\n")
        f.write(json.dumps({"metaData": {"id": "t", "format": {"provider": "parquet", "options": {}},
                                         "schemaString": json.dumps(schema), "partitionColumns": [],
                                         "configuration": {}, "createdTime": 0}}) + "\n")
        for i, st in enumerate(stats_list):
            a = {"path": "f%d.parquet" % i, "partitionValues": {}, "size": 1, "modificationTime": 0,
                 "dataChange": True}
            if st is not None:
                a["stats"] = st
            f.write(json.dumps({"add": a}) + "\n")


EDGE_STATS = [
    '{"numRecords":3,"minValues":{"x":2,"id":10},"maxValues":{"x":9,"id":20},"nullCount":{"x":0,"id":0}}',
    '{"numRecords":3,"minValues":{"x":2.0,"id":10},"maxValues":{"x":9E0,"id":20}}',
    '{"numRecords":3,"minValues":{"x":-0.0e3,"id":-5},"maxValues":{"x":1.50e1,"id":5}}',
    '{"numRecords":3,"minValues":{"x":7},"maxValues":{"x":8}} {"ignored": 1}',
    '{"numRecords":3,"minValues":{"x":1,"x":7},"maxValues":{"x":3,"x":8}}',
    '{"numRecords":3,"minValues":null,"maxValues":{"x":null}}',
    '{"numRecords":3,"min\\u0056alues":{"x":100},"maxValues":{"\\u0078":200}}',
    '{"numRecords":3,"minValues":{"x":4,"other":[1,{"a":"}"}]},"maxValues":{"x":6,"s":"\\"x\\""}}',
    '{ "numRecords" : 3 , "minValues" : { "x" : 4 } , "maxValues" : { "x" : 4 } }',
    '{"numRecords":3,"nullCount":{"x":3,"id":1},"minValues":{"x":4,"id":0},"maxValues":{"x":4,"id":0}}',
    None,
    '{}',
]
EDGE_PREDICATES = [cmp("=", col("x"), Literal.ofShort(4)), cmp(">", col("x"), Literal.ofShort(8)),
                   cmp("<", col("x"), Literal.ofInt(2)), Predicate("IS_NULL", col("x")),
                   Predicate("IS_NOT_NULL", col("id")), cmp("=", col("id"), Literal.ofLong(15)),
                   Or(cmp("=", col("x"), Literal.ofShort(7)), cmp("=", col("id"), Literal.ofLong(0)))]


@pytest.mark.gpu
def test_gpu_stats_json_edge_cases(tmp_path):
    from delta_amd import kernel as K
    root = str(tmp_path / "t")
    _write_edge_table(root, EDGE_STATS)
    eng = K.GpuEngine()
    for p in EDGE_PREDICATES:
        g = _gpu_files(root, p, eng)
        o = oracle_files(root, p)
        assert g == o, p
    eng.close()


def test_oracle_edge_cases_expected():
    """The oracle's answers on the edge-case table, written out by hand from the decoding rules."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        root = os.path.join(d, "t")
        _write_edge_table(root, EDGE_STATS)
        got = {i: sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0])
               for i, p in enumerate(EDGE_PREDICATES)}
    every = list(range(len(EDGE_STATS)))
    assert got[0] == [0, 1, 2, 5, 7, 8, 9, 10, 11]      # min.x <= 4 AND max.x >= 4 (row 4: last key wins)
    assert got[1] == [0, 1, 2, 5, 6, 10, 11]            # max.x > 8 (row 6: escaped key names)
    assert got[2] == [2, 5, 10, 11]                     # min.x < 2 (row 2: -0.0e3 is 0)
    assert got[3] == every[1:]                          # nullCount.x > 0: only row 0 is provably false
    assert got[4] == every                              # nullCount.id < numRecords
    assert got[5] == [i for i in every if i not in (2, 9)]
    assert got[6] == every                              # F OR null = null -> kept


BAD_STATS = ['{"numRecords":3,"minValues":{"x":4.5}}', '{"numRecords":3,"minValues":{"x":40000}}',
             '{"numRecords":3,"minValues":{"id":1.0}}', '{"numRecords":3,"minValues":3}',
             '{"numRecords":3,"minValues":{"x":"4"}}', '[1]', '{"numRecords":3,"minValues":{"x":4}',
             '{"numRecords":3,"minValues":{"x":04}}']
BAD_PREDICATE = And(cmp("<=", col("x"), Literal.ofShort(100)), cmp("<=", col("id"), Literal.ofLong(100)))


def test_oracle_bad_stats_raise(tmp_path):
    from oracle import skipping as osk
    for i, bad in enumerate(BAD_STATS):
        root = str(tmp_path / str(i))
        _write_edge_table(root, [EDGE_STATS[0], bad])
        with pytest.raises(osk.StatsDecodeError):
            oracle_files(root, BAD_PREDICATE)


@pytest.mark.gpu
def test_gpu_stats_decode_errors_raise(tmp_path):
    """A stats string the reference cannot decode fails the scan on the GPU too."""
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    eng = K.GpuEngine()
    for i, bad in enumerate(BAD_STATS):
        root = str(tmp_path / str(i))
        _write_edge_table(root, [EDGE_STATS[0], bad])
        with pytest.raises(DkError, match="data skipping"):
            _gpu_files(root, BAD_PREDICATE, eng)
    eng.close()


DATE_COLUMNS = (("d", "date"), ("id", "long"))
DATE_EDGE_STATS = [
    '{"numRecords":2,"minValues":{"d":"2000-01-01","id":1},"maxValues":{"d":"2000-1-5","id":2}}',
    '{"numRecords":2,"minValues":{"d":"2021-02-30"},"maxValues":{"d":"2021-3-+9"}}',
    '{"numRecords":2,"minValues":{"d":null},"maxValues":{"d":"1999-12-31"},"nullCount":{"d":1}}',
    '{"numRecords":2,"minValues":{"d":"2000-01-01","d":"2010-06-15"},"maxValues":{"d":"2020-01-01"}}',
    '{"numRecords":2,"minValues":{"d":"1583-01-01"},"maxValues":{"d":"9999-12-31"},"nullCount":{"d":0}}',
    None,
]
DATE_PREDICATES = [cmp("=", col("d"), Literal.ofDate(_days("2000-01-03"))),
                   cmp(">", col("d"), Literal.ofDate(_days("2021-03-01"))),
                   cmp("<", col("d"), Literal.ofDate(_days("2000-01-01"))),
                   And(cmp(">=", col("d"), Literal.ofDate(_days("2010-06-15"))),
                       cmp("<=", col("d"), Literal.ofDate(_days("2021-03-02")))),
                   Predicate("IS_NULL", col("d")),
                   Or(cmp("=", col("d"), Literal.ofDate(_days("1583-01-01"))), cmp("=", col("id"), Literal.ofLong(7)))]
DATE_BAD_STATS = ['{"numRecords":2,"minValues":{"d":10957}}', '{"numRecords":2,"minValues":{"d":"1500-01-01"}}',
                  '{"numRecords":2,"minValues":{"d":"2000-13-01"}}', '{"numRecords":2,"minValues":{"d":"2000-01"}}',
                  '{"numRecords":2,"minValues":{"d":{"a":1}}}', '{"numRecords":2,"minValues":{"d":"2000-01-1x"}}']
DATE_BAD_PREDICATE = cmp("<=", col("d"), Literal.ofDate(_days("2030-01-01")))


def test_oracle_date_edge_cases_expected(tmp_path):
    root = str(tmp_path / "t")
    _write_edge_table(root, DATE_EDGE_STATS, DATE_COLUMNS)
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in DATE_PREDICATES]
    assert got[0] == [0, 4, 5]                          # 2000-01-01 <= d <= 2000-01-05
    assert got[1] == [1, 4, 5]                          # max > 2021-03-01 (row 1: 2021-3-+9)
    assert got[2] == [2, 4, 5]                          # min < 2000-01-01 (row 2: null min -> kept)
    assert got[3] == [1, 3, 4, 5]                       # row 1 min is 2021-03-02 (lenient carry)
    assert got[4] == [0, 1, 2, 3, 5]                    # nullCount.d > 0 provably false only on row 4
    assert got[5] == [1, 2, 3, 4, 5]                    # row 0: both sides provably false
    for i, bad in enumerate(DATE_BAD_STATS):
        r = str(tmp_path / ("b%d" % i))
        _write_edge_table(r, [DATE_EDGE_STATS[0], bad], DATE_COLUMNS)
        from oracle import skipping as osk
        with pytest.raises(osk.StatsDecodeError):
            oracle_files(r, DATE_BAD_PREDICATE)


@pytest.mark.gpu
def test_gpu_date_stats_parity(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    root = str(tmp_path / "t")
    _write_edge_table(root, DATE_EDGE_STATS, DATE_COLUMNS)
    eng = K.GpuEngine()
    for p in DATE_PREDICATES:
        assert _gpu_files(root, p, eng) == oracle_files(root, p), p
    for i, bad in enumerate(DATE_BAD_STATS):
        r = str(tmp_path / ("b%d" % i))
        _write_edge_table(r, [DATE_EDGE_STATS[0], bad], DATE_COLUMNS)
        with pytest.raises(DkError, match="data skipping"):
            _gpu_files(r, DATE_BAD_PREDICATE, eng)
    eng.close()


STRING_COLUMNS = (("s", "string"), ("id", "long"))
STRING_EDGE_STATS = [
    '{"numRecords":2,"minValues":{"s":"apple"},"maxValues":{"s":"banana"}}',
    '{"numRecords":2,"minValues":{"s":"b"},"maxValues":{"s":"ba"}}',
    '{"numRecords":2,"minValues":{"s":"\\u00e9t\\u00e9"},"maxValues":{"s":"\u00fcber"}}',
    '{"numRecords":2,"minValues":{"s":"\\ud83d\\ude00"},"maxValues":{"s":"\\ud83d\\ude00z"}}',
    '{"numRecords":2,"minValues":{"s":"\\ud800x"},"maxValues":{"s":"?y"}}',
    '{"numRecords":2,"minValues":{"s":"a\\"b\\\\c\\n"},"maxValues":{"s":"a\\/z\\t"}}',
    '{"numRecords":2,"minValues":{"s":""},"maxValues":{"s":null},"nullCount":{"s":1}}',
    '{"numRecords":2,"minValues":{"s":"zz","s":"c"},"maxValues":{"s":"cz"}}',
    None,
]
STRING_PREDICATES = [cmp("=", col("s"), Literal.ofString("b")),
                     cmp(">", col("s"), Literal.ofString("\u00e9")),
                     cmp("<", col("s"), Literal.ofString("a/")),
                     cmp("=", col("s"), Literal.ofString("\U0001F600")),
                     cmp(">=", col("s"), Literal.ofString("?x")),
                     cmp("=", col("s"), Literal.ofString('a"b\\c\n')),
                     Or(cmp("<", col("s"), Literal.ofString("")), cmp("=", col("s"), Literal.ofString("ca"))),
                     Predicate("NOT", cmp("<=", col("s"), Literal.ofString("banana")))]
STRING_BAD_STATS = ['{"numRecords":2,"minValues":{"s":1}}', '{"numRecords":2,"minValues":{"s":true}}',
                    '{"numRecords":2,"minValues":{"s":{"x":"a"}}}', '{"numRecords":2,"minValues":{"s":["a"]}}']


def test_oracle_string_edge_cases_expected(tmp_path):
    root = str(tmp_path / "t")
    _write_edge_table(root, STRING_EDGE_STATS, STRING_COLUMNS)
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in STRING_PREDICATES]
    assert got[0] == [0, 1, 6, 8]                      # min <= "b" <= max; row 6: null max -> kept
    assert got[1] == [2, 3, 6, 8]                      # max > "é" (UTF-8 bytes: é = c3 a9 < ü, emoji)
    assert got[2] == [4, 5, 6, 8]                      # min < "a/" ("?" < "a", '"' < "/" < "p")
    assert got[3] == [3, 6, 8]                         # escaped surrogate pair == the code point
    assert got[4] == [0, 1, 2, 3, 4, 5, 6, 7, 8]       # lone surrogate -> "?x" (max "?y" >= "?x")
    assert got[5] == [5, 6, 8]                         # escapes decoded: a"b\\c<LF> <= lit <= a/z<TAB>
    assert got[6] == [6, 7, 8]                         # "" < "" false (null OR); row 7: last key wins
    assert got[7] == [2, 3, 6, 7, 8]                   # NOT (max <= "banana") -> max > "banana"
    from oracle import skipping as osk
    for i, bad in enumerate(STRING_BAD_STATS):
        r = str(tmp_path / ("b%d" % i))
        _write_edge_table(r, [STRING_EDGE_STATS[0], bad], STRING_COLUMNS)
        with pytest.raises(osk.StatsDecodeError):
            oracle_files(r, STRING_PREDICATES[0])


@pytest.mark.gpu
def test_gpu_string_stats_parity(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    root = str(tmp_path / "t")
    _write_edge_table(root, STRING_EDGE_STATS, STRING_COLUMNS)
    eng = K.GpuEngine()
    for p in STRING_PREDICATES:
        assert _gpu_files(root, p, eng) == oracle_files(root, p), p
    for i, bad in enumerate(STRING_BAD_STATS):
        r = str(tmp_path / ("b%d" % i))
        _write_edge_table(r, [STRING_EDGE_STATS[0], bad], STRING_COLUMNS)
        with pytest.raises(DkError, match="data skipping"):
            _gpu_files(r, STRING_PREDICATES[0], eng)
    eng.close()


# ScanSuite.scala:808-842 (TIMESTAMP): Spark writes ms-truncated stats in yyyy-MM-dd'T'HH:mm:ss.SSSXXX;
# the max is widened by TIMEADD(+1 ms) before comparing.
def _micros(text):
    import datetime
    t = datetime.datetime.fromisoformat(text.replace("Z", "+00:00"))
    d = t - datetime.datetime(1970, 1, 1, tzinfo=datetime.timezone.utc)
    return (d.days * 86400 + d.seconds) * 1_000_000 + d.microseconds


def _ts(op, c, text):
    return cmp(op, c, Literal.ofTimestamp(_micros(text)))


TS_COLUMNS = (("ts", "timestamp"), ("nested", {"type": "struct", "fields": [
    {"name": "ts", "type": "timestamp", "nullable": True, "metadata": {}}]}))
TS_SPARK_STATS = ('{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02:03.456Z","nested":{"ts":"2019-09-09T01:02:03.456Z"}},'
                  '"maxValues":{"ts":"2019-09-09T01:02:03.456Z","nested":{"ts":"2019-09-09T01:02:03.456Z"}},'
                  '"nullCount":{"ts":0,"nested":{"ts":0}}}')
NTS = Column("nested", "ts")
TS_HITS = [_ts("=", col("ts"), "2019-09-09T01:02:03.456789Z"), _ts(">=", col("ts"), "2019-09-09T01:02:03.456789Z"),
           _ts("<=", col("ts"), "2019-09-09T01:02:03.456789Z"), _ts(">=", NTS, "2019-09-09T01:02:03.456789Z"),
           _ts("<=", NTS, "2019-09-09T01:02:03.456789Z")]
TS_MISSES = [_ts("=", col("ts"), "2019-09-09T01:02:03.457001Z"), _ts(">=", col("ts"), "2019-09-09T01:02:03.457001Z"),
             _ts("<=", col("ts"), "2019-09-09T01:02:03.455999Z"), _ts(">=", NTS, "2019-09-09T01:02:03.457001Z"),
             _ts("<=", NTS, "2019-09-09T01:02:03.455999Z")]
TS_EDGE_STATS = [
    '{"numRecords":1,"minValues":{"ts":"2019-09-09t01:02:03+05:30"},"maxValues":{"ts":"2019-09-08T20:32:03.000001z"}}',
    '{"numRecords":1,"minValues":{"ts":"1969-12-31T23:59:59.9999995Z"},"maxValues":{"ts":"1970-01-01T00:00-00:00"}}',
    '{"numRecords":1,"minValues":{"ts":"2000-02-29T23:59:59.123456789-18:00"},"maxValues":{"ts":"2000-03-01T17:59:59.123456789Z"}}',
    '{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02:03.456Z","ts":"2020-01-01T00:00:00Z"},"maxValues":{"ts":null}}',
    None,
]
TS_EDGE_PREDICATES = [_ts("=", col("ts"), "2019-09-08T20:32:03Z"), _ts("<", col("ts"), "1970-01-01T00:00:00Z"),
                      _ts(">", col("ts"), "2000-03-01T17:59:59.124Z"), _ts(">=", col("ts"), "2020-01-01T00:00:00Z"),
                      _ts("=", col("ts"), "1970-01-01T00:00:00.001Z")]
TS_BAD_STATS = ['{"numRecords":1,"minValues":{"ts":"2019-02-29T00:00:00Z"}}', '{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02:03"}}',
                '{"numRecords":1,"minValues":{"ts":"2019-09-09 01:02:03Z"}}', '{"numRecords":1,"minValues":{"ts":"2019-09-09T24:00:00Z"}}',
                '{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02:03+19:00"}}', '{"numRecords":1,"minValues":{"ts":12}}',
                '{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02:03.1234567891Z"}}', '{"numRecords":1,"minValues":{"ts":"1500-01-01T00:00:00Z"}}']


def test_oracle_timestamp_reference_hits_and_misses(tmp_path):
    root = str(tmp_path / "t")
    _write_edge_table(root, [TS_SPARK_STATS], TS_COLUMNS)
    for p in TS_HITS:
        assert oracle_files(root, p)[0], p
    for p in TS_MISSES:
        assert not oracle_files(root, p)[0], p
    r = str(tmp_path / "e")
    _write_edge_table(r, TS_EDGE_STATS, TS_COLUMNS)
    got = [sorted(int(x[0].decode()[1:-8]) for x in oracle_files(r, p)[0]) for p in TS_EDGE_PREDICATES]
    assert got[0] == [0, 4]                         # row 0: +05:30 is 20:32:03Z (row 3: min 2020 wins)
    assert got[1] == [4]                            # row 1 min: -500 ns truncates toward zero to 0
    assert got[2] == [0, 2, 3, 4]                   # row 2 max .123456 + 1 ms = .124456 > .124
    assert got[3] == [3, 4]                         # row 3: last min key wins (2020), null max -> kept
    assert got[4] == [1, 4]                         # row 1: max 0 + 1 ms = 1 ms
    from oracle import skipping as osk
    for i, bad in enumerate(TS_BAD_STATS):
        b = str(tmp_path / ("b%d" % i))
        _write_edge_table(b, [TS_SPARK_STATS, bad], TS_COLUMNS)
        with pytest.raises(osk.StatsDecodeError):
            oracle_files(b, TS_HITS[0])


@pytest.mark.gpu
def test_gpu_timestamp_stats_parity(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    root = str(tmp_path / "t")
    _write_edge_table(root, [TS_SPARK_STATS], TS_COLUMNS)
    eng = K.GpuEngine()
    for p in TS_HITS + TS_MISSES:
        g = _gpu_files(root, p, eng)
        assert g == oracle_files(root, p) and bool(g[0]) == (p in TS_HITS), p
    r = str(tmp_path / "e")
    _write_edge_table(r, TS_EDGE_STATS, TS_COLUMNS)
    for p in TS_EDGE_PREDICATES:
        assert _gpu_files(r, p, eng) == oracle_files(r, p), p
    for i, bad in enumerate(TS_BAD_STATS):
        b = str(tmp_path / ("b%d" % i))
        _write_edge_table(b, [TS_SPARK_STATS, bad], TS_COLUMNS)
        with pytest.raises(DkError, match="data skipping"):
            _gpu_files(b, TS_HITS[0], eng)
    eng.close()


DEC_COLUMNS = (("x", "decimal(38,4)"), ("id", "long"))
DEC_EDGE_STATS = [
    '{"numRecords":2,"minValues":{"x":1.50},"maxValues":{"x":2}}',
    '{"numRecords":2,"minValues":{"x":-1E+2},"maxValues":{"x":-0.0001}}',
    '{"numRecords":2,"minValues":{"x":123456789012345678901234567890.12},"maxValues":{"x":1.2345678901234567890123456789012E+31}}',
    '{"numRecords":2,"minValues":{"x":0},"maxValues":{"x":0.00e5},"nullCount":{"x":0}}',
    '{"numRecords":2,"minValues":{"x":null},"maxValues":{"x":1.5}}',
    None,
]
# literals of the column's own type (decimal(38,4)): differently typed decimals are not comparable
# (DecimalType.equals, DefaultExpressionEvaluator.transformBinaryComparator); the values keep their
# own digits and scale, which compareTo ignores
DEC_PREDICATES = [cmp("=", col("x"), Literal.ofDecimal("1.5", 38, 4)),
                  cmp("<", col("x"), Literal.ofDecimal("0", 38, 4)),
                  cmp(">", col("x"), Literal.ofDecimal("1.2345678901234567890123456789011E+31", 38, 4)),
                  cmp("=", col("x"), Literal.ofDecimal("0.000", 38, 4)),
                  cmp(">=", col("x"), Literal.ofDecimal("1.5001", 38, 4))]
DEC_BAD_STATS = ['{"numRecords":2,"minValues":{"x":"1.5"}}', '{"numRecords":2,"minValues":{"x":true}}',
                 '{"numRecords":2,"minValues":{"x":{"a":1}}}']


def test_oracle_decimal_stats_expected(tmp_path):
    root = str(tmp_path / "t")
    _write_edge_table(root, DEC_EDGE_STATS, DEC_COLUMNS)
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in DEC_PREDICATES]
    assert got == [[0, 4, 5], [1, 4, 5], [2, 5], [3, 4, 5], [0, 2, 5]]   # row 4: null min -> kept
    from oracle import skipping as osk
    for i, bad in enumerate(DEC_BAD_STATS):
        r = str(tmp_path / ("b%d" % i))
        _write_edge_table(r, [DEC_EDGE_STATS[0], bad], DEC_COLUMNS)
        with pytest.raises(osk.StatsDecodeError):
            oracle_files(r, DEC_PREDICATES[0])


@pytest.mark.gpu
def test_gpu_decimal_stats_parity(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    root = str(tmp_path / "t")
    _write_edge_table(root, DEC_EDGE_STATS, DEC_COLUMNS)
    eng = K.GpuEngine()
    for p in DEC_PREDICATES:
        assert _gpu_files(root, p, eng) == oracle_files(root, p), p
    for i, bad in enumerate(DEC_BAD_STATS):
        r = str(tmp_path / ("b%d" % i))
        _write_edge_table(r, [DEC_EDGE_STATS[0], bad], DEC_COLUMNS)
        with pytest.raises(DkError, match="data skipping"):
            _gpu_files(r, DEC_PREDICATES[0], eng)
    eng.close()


# ScanSuite.scala:808-842 (TIMESTAMP_NTZ): stats written without an offset; max widened by +1 ms
NTZ_COLUMNS = (("ts", "timestamp_ntz"), ("nested", {"type": "struct", "fields": [
    {"name": "ts", "type": "timestamp_ntz", "nullable": True, "metadata": {}}]}))
NTZ_SPARK_STATS = TS_SPARK_STATS.replace(".456Z", ".456")


def _ntz(op, c, text):
    return cmp(op, c, Literal.ofTimestampNtz(_micros(text)))


NTZ_HITS = [_ntz(p.name, p.children[0], t) for p, t in zip(TS_HITS, ["2019-09-09T01:02:03.456789Z"] * 5)]
NTZ_MISSES = [_ntz(p.name, p.children[0], t) for p, t in zip(TS_MISSES, ["2019-09-09T01:02:03.457001Z"] * 2 +
                                                            ["2019-09-09T01:02:03.455999Z"] +
                                                            ["2019-09-09T01:02:03.457001Z", "2019-09-09T01:02:03.455999Z"])]
NTZ_EDGE_STATS = ['{"numRecords":1,"minValues":{"ts":"2019-02-30T00:00:00"},"maxValues":{"ts":"2019-02-28T00:00:00.5"}}',
                  '{"numRecords":1,"minValues":{"ts":"2020-02-31T23:59:59.999999"},"maxValues":{"ts":"2020-03-01T00:00:00"}}',
                  # SMART end of day: 24:00:00 is next midnight; a bare '.' is a zero fraction
                  '{"numRecords":1,"minValues":{"ts":"2019-02-28T24:00:00"},"maxValues":{"ts":"2019-03-01T00:00:00."}}',
                  None]
NTZ_EDGE_PREDICATES = [_ntz("=", col("ts"), "2019-02-28T00:00:00.200000Z"), _ntz("<", col("ts"), "2020-02-29T23:59:59.999999Z"),
                       _ntz(">", col("ts"), "2020-03-01T00:00:00.000500Z"), _ntz("=", col("ts"), "2019-03-01T00:00:00Z")]
NTZ_BAD_STATS = ['{"numRecords":1,"minValues":{"ts":"2019-09-09t01:02:03"}}', '{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02"}}',
                 '{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02:03Z"}}', '{"numRecords":1,"minValues":{"ts":"2019-09-09T01:02:03.1234567"}}',
                 '{"numRecords":1,"minValues":{"ts":"2019-09-32T01:02:03"}}',
                 '{"numRecords":1,"minValues":{"ts":"2019-09-09T24:00:01"}}', '{"numRecords":1,"minValues":{"ts":"2019-09-09T24:00:00.1"}}']


def test_oracle_timestamp_ntz(tmp_path):
    root = str(tmp_path / "t")
    _write_edge_table(root, [NTZ_SPARK_STATS], NTZ_COLUMNS)
    for p in NTZ_HITS:
        assert oracle_files(root, p)[0], p
    for p in NTZ_MISSES:
        assert not oracle_files(root, p)[0], p
    r = str(tmp_path / "e")
    _write_edge_table(r, NTZ_EDGE_STATS, NTZ_COLUMNS)
    got = [sorted(int(x[0].decode()[1:-8]) for x in oracle_files(r, p)[0]) for p in NTZ_EDGE_PREDICATES]
    # Feb 30 -> Feb 28 and Feb 31 -> Feb 29 (SMART clamp); row 2's 24:00:00 is Mar 1 00:00
    assert got == [[0, 3], [0, 2, 3], [1, 3], [2, 3]]
    from oracle import skipping as osk
    for i, bad in enumerate(NTZ_BAD_STATS):
        b = str(tmp_path / ("b%d" % i))
        _write_edge_table(b, [NTZ_SPARK_STATS, bad], NTZ_COLUMNS)
        with pytest.raises(osk.StatsDecodeError):
            oracle_files(b, NTZ_HITS[0])


@pytest.mark.gpu
def test_gpu_timestamp_ntz_parity(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    root = str(tmp_path / "t")
    _write_edge_table(root, [NTZ_SPARK_STATS], NTZ_COLUMNS)
    eng = K.GpuEngine()
    for p in NTZ_HITS + NTZ_MISSES:
        g = _gpu_files(root, p, eng)
        assert g == oracle_files(root, p) and bool(g[0]) == (p in NTZ_HITS), p
    r = str(tmp_path / "e")
    _write_edge_table(r, NTZ_EDGE_STATS, NTZ_COLUMNS)
    for p in NTZ_EDGE_PREDICATES:
        assert _gpu_files(r, p, eng) == oracle_files(r, p), p
    for i, bad in enumerate(NTZ_BAD_STATS):
        b = str(tmp_path / ("b%d" % i))
        _write_edge_table(b, [NTZ_SPARK_STATS, bad], NTZ_COLUMNS)
        with pytest.raises(DkError, match="data skipping"):
            _gpu_files(b, NTZ_HITS[0], eng)
    eng.close()


# ---------------------------------------------------------------- float / double
def test_oracle_implicit_casting(tmp_path):
    """ScanSuite.scala:1198-1212 on the golden table (short column vs float literal and back)."""
    root = os.path.join(TABLES, "data-skipping-basic-stats-all-types")
    for p in (cmp("=", col("as_short"), Literal.ofFloat(0)), cmp("=", col("as_float"), Literal.ofShort(0))):
        assert oracle_files(root, p)[0], p
    for p in (cmp("=", col("as_short"), Literal.ofFloat(1)), cmp("=", col("as_float"), Literal.ofShort(1))):
        assert not oracle_files(root, p)[0], p


SPARK_FP_COLUMNS = (("c1", "long"), ("c3", "float"), ("c4", "double"))
SPARK_FP_STATS = ['{"numRecords":2,"minValues":{"c1":1,"c3":1.0,"c4":1.0},"maxValues":{"c1":2,"c3":2.0,"c4":2.0},'
                  '"nullCount":{"c1":0,"c3":0,"c4":0}}']
SPARK_FP_HITS = [cmp("<", col("c3"), Literal.ofFloat(1.5)), cmp(">", col("c4"), Literal.ofFloat(1.0))]
SPARK_FP_MISSES = [cmp("<", col("c3"), Literal.ofFloat(0.5)), cmp(">", col("c4"), Literal.ofFloat(5.0))]

FP_COLUMNS = (("f", "float"), ("d", "double"), ("i", "long"))
FP_EDGE_STATS = [
    '{"numRecords":1,"minValues":{"f":0.1,"d":0.1,"i":16777217},"maxValues":{"f":0.1,"d":0.1,"i":16777217}}',
    '{"numRecords":1,"minValues":{"f":"NaN","d":"-Infinity","i":-1},"maxValues":{"f":"NaN","d":"+INF","i":1}}',
    '{"numRecords":1,"minValues":{"f":-0.0,"d":-1E-400,"i":0},"maxValues":{"f":1E-50,"d":-0,"i":0}}',
    '{"numRecords":1,"minValues":{"f":16777217,"d":9007199254740993,"i":9007199254740993},'
    '"maxValues":{"f":16777217.000000001,"d":9007199254740993.5,"i":9007199254740993}}',
    '{"numRecords":1,"minValues":{"f":"\\u004eaN","d":"Infinity"},"maxValues":{"f":"-INF","d":"NaN"}}',
    '{"numRecords":1,"minValues":{"f":3.4028235677973366E38,"d":1.7976931348623157E308},'
    '"maxValues":{"f":-3.4028235677973366E38,"d":4.9E-324}}',
    '{"numRecords":1,"minValues":{"f":1.4999999403953552,"d":1.5},"maxValues":{"f":1.49999994039535522,"d":2}}',
    None,
]
FP_EDGE_PREDICATES = [
    cmp("=", col("f"), Literal.ofFloat(0.1)),                      # 0.1 rounds to 0.1f
    cmp("=", col("d"), Literal.ofDouble(0.1)),
    cmp("=", col("f"), Literal.ofDouble(0.1)),                      # float(0.1) widened != 0.1d
    cmp("<", col("f"), Literal.ofFloat(float("nan"))),              # everything but NaN is < NaN
    cmp("=", col("f"), Literal.ofFloat(float("nan"))),
    cmp(">", col("d"), Literal.ofDouble(float("inf"))),             # only NaN is > +Inf
    cmp("<", col("d"), Literal.ofDouble(float("-inf"))),
    cmp("<", col("f"), Literal.ofFloat(0.0)),                       # -0.0 < 0.0 (Float.compare)
    cmp(">=", col("f"), Literal.ofFloat(-0.0)),
    cmp("=", col("d"), Literal.ofDouble(-0.0)),                     # -1E-400 rounds to -0.0
    cmp("=", col("f"), Literal.ofFloat(16777216)),                  # 16777217 rounds (tie) to 2^24
    cmp(">", col("f"), Literal.ofFloat(16777216)),                  # 16777217.000000001 -> 16777218
    cmp("=", col("d"), Literal.ofDouble(9007199254740992)),
    cmp("=", col("i"), Literal.ofFloat(16777216)),                  # long widened to float
    cmp(">", col("i"), Literal.ofDouble(9007199254740992)),         # long widened to double: tie -> even
    cmp("<", col("f"), Literal.ofFloat(1.5)),                       # 1.4999999403953552 is the tie
    cmp(">=", col("d"), Literal.ofDouble(1.7976931348623157e308)),
    cmp(">", col("d"), Literal.ofDouble(0.0)),                      # 4.9E-324: the smallest subnormal
    Or(cmp("<", col("f"), Literal.ofFloat(-3e38)), cmp(">", col("f"), Literal.ofFloat(3e38))),
    Predicate("NOT", cmp("=", col("d"), Literal.ofDouble(1.5))),
]
FP_BAD_STATS = ['{"numRecords":1,"minValues":{"f":3.4028235677973367E38}}',     # rounds to +Infinity
                '{"numRecords":1,"minValues":{"d":1E309}}', '{"numRecords":1,"minValues":{"f":"nan"}}',
                '{"numRecords":1,"minValues":{"d":"1.5"}}', '{"numRecords":1,"minValues":{"f":true}}',
                '{"numRecords":1,"minValues":{"d":{"a":1}}}', '{"numRecords":1,"minValues":{"f":"-Inf"}}']
FP_BAD_PREDICATE = And(cmp("<=", col("f"), Literal.ofFloat(100)), cmp("<=", col("d"), Literal.ofDouble(100)))


def test_oracle_float_stats_expected(tmp_path):
    root = str(tmp_path / "s")
    _write_edge_table(root, SPARK_FP_STATS, SPARK_FP_COLUMNS)
    for p in SPARK_FP_HITS:
        assert oracle_files(root, p)[0], p
    for p in SPARK_FP_MISSES:
        assert not oracle_files(root, p)[0], p
    r = str(tmp_path / "t")
    _write_edge_table(r, FP_EDGE_STATS, FP_COLUMNS)
    got = [sorted(int(x[0].decode()[1:-8]) for x in oracle_files(r, p)[0]) for p in FP_EDGE_PREDICATES]
    # worked by hand from the decoding rules: row 2's "-0.0" is +0.0 (BigDecimal) while -1E-400 rounds
    # to -0.0; row 3's 16777217 ties to 2^24 and 9007199254740993 to 2^53; row 6's float minimum sits
    # just below the 1.5f tie; row 5's float extremes stay finite; NaN compares above +Infinity
    want = [[0, 7], [0, 1, 7], [7], [0, 2, 3, 5, 6, 7], [1, 7], [4, 7], [7], [7], [0, 1, 2, 3, 6, 7],
            [1, 2, 7], [3, 7], [1, 3, 7], [1, 3, 7], [0, 4, 5, 6, 7], [4, 5, 6, 7], [0, 2, 6, 7], [1, 4, 7],
            [0, 1, 3, 4, 5, 6, 7], [1, 7], [0, 1, 2, 3, 4, 6, 7]]
    assert got == want
    from oracle import skipping as osk
    for i, bad in enumerate(FP_BAD_STATS):
        b = str(tmp_path / ("b%d" % i))
        _write_edge_table(b, [FP_EDGE_STATS[0], bad], FP_COLUMNS)
        with pytest.raises(osk.StatsDecodeError):
            oracle_files(b, FP_BAD_PREDICATE)


@pytest.mark.gpu
def test_gpu_float_stats_parity(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    eng = K.GpuEngine()
    for name in ALL_TYPES[:1]:
        root = os.path.join(TABLES, name)
        for p in (cmp("=", col("as_short"), Literal.ofFloat(0)), cmp("=", col("as_float"), Literal.ofShort(0)),
                  cmp("=", col("as_short"), Literal.ofFloat(1)), cmp("=", col("as_float"), Literal.ofShort(1))):
            assert _gpu_files(root, p, eng) == oracle_files(root, p), p
    s = str(tmp_path / "s")
    _write_edge_table(s, SPARK_FP_STATS, SPARK_FP_COLUMNS)
    for p in SPARK_FP_HITS + SPARK_FP_MISSES:
        g = _gpu_files(s, p, eng)
        assert g == oracle_files(s, p) and bool(g[0]) == (p in SPARK_FP_HITS), p
    r = str(tmp_path / "t")
    _write_edge_table(r, FP_EDGE_STATS, FP_COLUMNS)
    for p in FP_EDGE_PREDICATES:
        assert _gpu_files(r, p, eng) == oracle_files(r, p), p
    for i, bad in enumerate(FP_BAD_STATS):
        b = str(tmp_path / ("b%d" % i))
        _write_edge_table(b, [FP_EDGE_STATS[0], bad], FP_COLUMNS)
        with pytest.raises(DkError, match="data skipping"):
            _gpu_files(b, FP_BAD_PREDICATE, eng)
    eng.close()


# ---------------------------------------------------------------- stats_parsed fast path
def _gpu_files_parsed(root, predicate, eng):
    """_gpu_files plus the number of checkpoint files whose skipping read add.stats_parsed."""
    from delta_amd import kernel as K
    from delta_amd._lib import lib
    from oracle import ref
    snap = K.Table.forPath(eng, root).getLatestSnapshot(eng)
    scan = snap.getScanBuilder().withFilter(predicate).build()
    try:
        rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in scan.getScanFiles(eng)
                for i in b.selected_rows()]
        return rows, scan.metrics.as_tuple(), lib().dk_replay_stats_parsed_files(scan._rh)
    finally:
        scan.close()


@pytest.mark.gpu
def test_gpu_stats_parsed_equals_json(tmp_path):
    """Checkpoint files with add.stats_parsed (Spark's from_json(stats)): skipping over the typed
    columns must select exactly what the JSON path (the oracle, DataSkippingUtils over add.stats)
    selects; string predicates fall back to the JSON stats."""
    from delta_amd import kernel as K
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=40_000, n_parts=3, n_commits=6, dv_frac=0.2,
                                                     ckpt_removes=200, with_stats=True, with_stats_parsed=True,
                                                     pv_keys=2))
    eng = K.GpuEngine()
    for p in SYNTH_PREDICATES:
        g = _gpu_files_parsed(str(tmp_path), p, eng)
        o = oracle_files(str(tmp_path), p)
        assert g[1] == o[1], p
        assert g[0] == o[0], p
        assert g[2] == 3, p                       # every checkpoint part used stats_parsed
    # a string stat reads the typed BYTE_ARRAY leaf too
    p = cmp(">", col("name"), Literal.ofString("n25"))
    g = _gpu_files_parsed(str(tmp_path), p, eng)
    assert g[2] == 3 and g[0] == oracle_files(str(tmp_path), p)[0]
    eng.close()


def typed_predicates(mins, ts_unit):
    """Predicates over every column of synth.TYPED_STATS_COLUMNS; '=' literals taken from the table."""
    def pick(c, k):
        vs = [v for v in mins[c] if v == v]
        return vs[k % len(vs)]
    us = (lambda v: v * 1000) if ts_unit == "ms" else (lambda v: v)
    nan, inf = float("nan"), float("inf")
    return [
        cmp("=", col("l"), Literal.ofLong(pick("l", 3))), cmp(">", col("l"), Literal.ofLong(0)),
        cmp("<=", col("i"), Literal.ofInt(pick("i", 5))), cmp(">", col("i"), Literal.ofLong(1 << 40)),
        cmp("=", col("d"), Literal.ofDate(pick("d", 2))), cmp(">", col("d"), Literal.ofDate(10000)),
        cmp("=", col("ts"), Literal.ofTimestamp(us(pick("ts", 4)))),
        cmp("<", col("ts"), Literal.ofTimestamp(us(pick("ts", 9)))),
        cmp(">=", col("tz"), Literal.ofTimestampNtz(us(pick("tz", 1)))),
        cmp(">=", col("s"), Literal.ofString("b")), cmp("=", col("s"), Literal.ofString(pick("s", 4))),
        cmp("<", col("s"), Literal.ofString("\u4e2d")), cmp(">", col("s"), Literal.ofString("z\U0001f600")),
        cmp("=", col("dc"), Literal.ofDecimal(str(pick("dc", 1)), 12, 2)),
        cmp(">", col("dc"), Literal.ofDecimal("0.00", 12, 2)),
        cmp("<", col("dd"), Literal.ofDecimal("-0.5", 6, 1)),
        cmp("<", col("f"), Literal.ofFloat(0.0)), cmp(">=", col("f"), Literal.ofFloat(-0.0)),
        cmp("=", col("f"), Literal.ofFloat(pick("f", 3))), cmp("<", col("f"), Literal.ofFloat(nan)),
        cmp(">", col("f"), Literal.ofDouble(10.5)), cmp("=", col("f"), Literal.ofFloat(inf)),
        cmp("=", col("g"), Literal.ofDouble(pick("g", 2))), cmp(">", col("g"), Literal.ofDouble(inf)),
        cmp("<=", col("g"), Literal.ofDouble(-0.0)), cmp(">", col("g"), Literal.ofFloat(-3.25)),
        Predicate("IS_NULL", col("s")), Predicate("IS_NOT_NULL", col("g")),
        And(cmp(">", col("l"), Literal.ofLong(0)), cmp("<", col("f"), Literal.ofFloat(100.0))),
        Or(cmp("=", col("d"), Literal.ofDate(pick("d", 7))), cmp(">", col("dc"), Literal.ofDecimal("5.00", 12, 2))),
        And(cmp(">=", col("s"), Literal.ofString("x")), cmp("<", col("ts"), Literal.ofTimestamp(0))),
    ]


@pytest.mark.gpu
@pytest.mark.parametrize("ts_unit", ["us", "ms", "int96"])
def test_gpu_typed_stats_parsed_equals_json(tmp_path, ts_unit):
    """Typed add.stats_parsed for every stats type (synth.write_typed_stats_table): timestamps as
    INT64 micros / millis or INT96, strings, INT32 / INT64 decimals, floats and doubles with NaN,
    +-Infinity and -0.0 (evaluated from the row's JSON: Kernel reads "-0.0" as +0.0), rows with only
    one of add.stats / stats_parsed. Every predicate selects what the oracle (add.stats only)
    selects, and the checkpoint's skipping ran over stats_parsed."""
    from delta_amd import kernel as K
    root = str(tmp_path / "t")
    mins = synth.write_typed_stats_table(root, n=3000, seed=11, ts_unit=ts_unit)
    eng = K.GpuEngine()
    try:
        for p in typed_predicates(mins, ts_unit):
            g = _gpu_files_parsed(root, p, eng)
            o = oracle_files(root, p)
            assert g[2] == 1, p
            assert g[1] == o[1], p
            assert g[0] == o[0], p
    finally:
        eng.close()


def wide_predicates(mins):
    """Filters past every old cap (8 stats paths, 64 ops, 4 KiB of literals): an OR of 32 equalities
    over 14 columns, '=' on 5 columns, IS_NOT_NULL on 12 columns, 10 KiB string literals."""
    cols = ["l", "i", "d", "s", "dc", "f", "g"] + ["x%d" % k for k in range(7)]

    def lit(c, k):
        vs = [v for v in mins[c] if v == v]
        v = vs[k % len(vs)]
        return {"l": Literal.ofLong, "i": Literal.ofInt, "d": Literal.ofDate, "s": Literal.ofString,
                "f": Literal.ofFloat, "g": Literal.ofDouble}.get(c, Literal.ofLong)(v) if c != "dc" \
            else Literal.ofDecimal(str(v), 12, 2)
    ors = cmp("=", col(cols[0]), lit(cols[0], 0))
    for k in range(1, 32):
        c = cols[k % len(cols)]
        ors = Or(ors, cmp("=", col(c), lit(c, 7 * k)))
    five = cmp("=", col("x0"), lit("x0", 1))
    for c in ("x1", "x2", "x3", "x4"):
        five = And(five, cmp(">=", col(c), Literal.ofLong(-150)))
    nn = Predicate("IS_NOT_NULL", col(cols[0]))
    for c in cols[1:12]:
        nn = And(nn, Predicate("IS_NOT_NULL", col(c)))
    big_z, big_a = "z" * 10240, "a" * 5000 + "\u4e2d" * 2000
    return [ors, five, nn, And(ors, nn), cmp("<", col("s"), Literal.ofString(big_z)),
            cmp(">", col("s"), Literal.ofString(big_a)), cmp("=", col("s"), Literal.ofString(big_z)),
            Or(cmp("=", col("s"), Literal.ofString(big_a)), cmp("=", col("x5"), lit("x5", 3)))]


@pytest.mark.gpu
def test_gpu_wide_filters(tmp_path):
    """The filters of wide_predicates over a checkpoint with add.stats_parsed (14 typed columns:
    k_stats_parsed with per-lane scratch) and a commit tail (k_stats_eval over the JSON, 32-path
    extraction windows): the scan files and counters equal the oracle's."""
    from delta_amd import kernel as K
    from delta_amd import programs
    root = str(tmp_path / "t")
    mins = synth.write_typed_stats_table(root, n=3000, seed=17, extra_long=7)
    eng = K.GpuEngine()
    try:
        widest = 0
        for p in wide_predicates(mins):
            schema, parts = table_metadata(root)
            leaves = sk.data_schema_leaves(schema, parts)
            widest = max(widest, len(programs.compile_skipping(sk.construct(p, leaves), leaves).paths))
            g = _gpu_files_parsed(root, p, eng)
            o = oracle_files(root, p)
            assert g[1] == o[1], p
            assert g[0] == o[0], p
            assert g[2] == 1, p                       # the checkpoint's skipping read stats_parsed
        assert widest > 32
    finally:
        eng.close()


def test_oracle_wide_filters_discriminate(tmp_path):
    root = str(tmp_path / "t")
    mins = synth.write_typed_stats_table(root, n=400, seed=17, extra_long=7)
    kept = [len(oracle_files(root, p)[0]) for p in wide_predicates(mins)]
    live = 400 + 40 - 20
    assert sum(0 < k < live for k in kept) >= 4, kept


def test_oracle_typed_stats_table(tmp_path):
    """The typed-stats fixture is a valid table for the oracle, and the predicates discriminate (each
    keeps some files and drops some)."""
    root = str(tmp_path / "t")
    mins = synth.write_typed_stats_table(root, n=400, seed=11, ts_unit="ms")
    live = 400 + 40 - 20                       # checkpoint adds + tail adds - tail removes
    kept = [len(oracle_files(root, p)[0]) for p in typed_predicates(mins, "ms")]
    assert all(k > 0 for k in kept), kept
    assert sum(k < live for k in kept) >= len(kept) - 3, kept


def test_rank_run_matches_java_compare():
    """binfloat.rank_run (the typed stats_parsed float comparison) agrees with Float.compare /
    Double.compare over random and special float / double values."""
    import math
    import random
    import struct
    from fractions import Fraction
    from tests import binfloat_ref as bf
    rnd = random.Random(5)
    for fmt, pk, bits_n in (("float", "<f", 32), ("double", "<d", 64)):
        specials = [0.0, -0.0, 1.5, -1.5, float("inf"), float("-inf"), float("nan"), 16777216.0, 0.1, 1e-45, 5e-324]
        for lit_type in ("float", "double", "long"):
            if fmt == "float" and lit_type == "double":
                continue
            for _ in range(40):
                lit = rnd.choice(specials) if rnd.random() < 0.5 else rnd.uniform(-100, 100)
                if lit_type == "long":
                    if lit != lit or math.isinf(lit):
                        continue
                    lit = int(lit)
                op = rnd.choice(["<", "<=", ">", ">=", "="])
                (a, b), (r_nan, _, _) = bf.rank_run(op, lit, lit_type, fmt, fmt)
                V = bf.literal_value(lit, lit_type, fmt)
                for _ in range(60):
                    x = rnd.choice(specials) if rnd.random() < 0.3 else rnd.uniform(-120, 120)
                    bits = struct.unpack("<I" if bits_n == 32 else "<Q", struct.pack(pk, x))[0]
                    x = struct.unpack(pk, struct.pack(pk, x))[0]
                    if x != x:
                        assert r_nan == bf._TEST[op](bf.java_compare(bf.NAN, V))
                        continue
                    xv = bf.PINF if x == float("inf") else bf.NINF if x == float("-inf") else \
                        (Fraction(x), math.copysign(1.0, x) < 0 and x == 0)
                    want = bf._TEST[op](bf.java_compare(xv, V))
                    assert (a <= bf.rank(bits, fmt) <= b) == want, (fmt, lit_type, lit, op, x)


def test_program_keeps_rank_bytes():
    """The FCMP threshold text is followed by its rank run (two int64s, NUL bytes included) in the
    program's pool."""
    leaves = {("f",): ("float", ("f",))}
    _, _, ops = _compiled(sk.construct(cmp("=", col("f"), Literal.ofFloat(0.0)), leaves), leaves)
    # min <= 0.0f: every rank up to +0.0 (-0.0 included); max >= 0.0f: from +0.0 (Float.compare: -0.0 < 0.0)
    assert [o[4] for o in ops if o[0] == sk.OP_FCMP] == [(-0x7f800001, 0), (0, 0x7f800000)]


# ---------------------------------------------------------------- planner vs the oracle's own restatement
_PLAN_SCHEMA = json.dumps({"type": "struct", "fields": [
    {"name": n, "type": t, "nullable": True, "metadata": m} for n, t, m in (
        ("l", "long", {}), ("i", "integer", {}), ("sh", "short", {}), ("b", "byte", {}), ("f", "float", {}),
        ("d", "double", {}), ("dt", "date", {}), ("ts", "timestamp", {}), ("tz", "timestamp_ntz", {}),
        ("s", "string", {"delta.columnMapping.physicalName": "col-s"}), ("dc", "decimal(10,2)", {}),
        ("bo", "boolean", {}), ("bi", "binary", {}), ("p", "integer", {}),
        ("st", {"type": "struct", "fields": [{"name": "x", "type": "long", "nullable": True, "metadata": {}},
                                             {"name": "y", "type": "boolean", "nullable": True, "metadata": {}}]},
         {}),
        ("ar", {"type": "array", "elementType": "long", "containsNull": True}, {}))]})


def _random_predicate(rnd, depth):
    cols = [col(n) for n in ("l", "i", "sh", "b", "f", "d", "dt", "ts", "tz", "s", "dc", "bo", "bi", "p", "ar",
                             "nope")] + [Column("st", "x"), Column("st", "y"), Column("st")]
    lits = [Literal.ofLong(5), Literal.ofInt(-3), Literal.ofShort(2), Literal.ofByte(1), Literal.ofFloat(1.5),
            Literal.ofDouble(-2.25), Literal.ofDate(100), Literal.ofTimestamp(10 ** 12), Literal.ofTimestampNtz(7),
            Literal.ofString("k"), Literal.ofDecimal("1.25", 10, 2), Literal.ofDecimal("1.5", 5, 1),
            Literal.ofBoolean(True), Literal.ofNull("long"), Literal.ofNull("string")]
    r = rnd.random()
    if depth > 0 and r < 0.35:
        return Predicate(rnd.choice(["AND", "OR"]), _random_predicate(rnd, depth - 1), _random_predicate(rnd, depth - 1))
    if depth > 0 and r < 0.5:
        return Predicate("NOT", _random_predicate(rnd, depth - 1))
    if r < 0.6:
        return Predicate(rnd.choice(["IS_NULL", "IS_NOT_NULL"]), rnd.choice(cols))
    if r < 0.63:
        return Predicate("STARTS_WITH", rnd.choice(cols), rnd.choice(lits))
    op = rnd.choice(["=", "<", "<=", ">", ">=", "IS NOT DISTINCT FROM"])
    a, b = rnd.choice(cols), rnd.choice(lits)
    if rnd.random() < 0.3:
        a, b = b, a
    if rnd.random() < 0.05:
        b = rnd.choice(cols)
    return Predicate(op, a, b)


def test_planner_matches_oracle_restatement():
    """delta_amd/skipping.py (construct, split_filters, check_types) against oracle/skipping_filter.py,
    an independent restatement of DataSkippingUtils.constructDataSkippingFilter / StatsSchemaHelper /
    PartitionUtils.splitMetadataAndDataPredicates / transformBinaryComparator, on 3,000 random
    predicates over every column kind (eligible, ineligible, nested, array, partition, missing)."""
    import random
    from oracle import skipping_filter as osf
    rnd = random.Random(12)
    parts = ["p"]
    leaves = sk.data_schema_leaves(_PLAN_SCHEMA, parts)
    S = osf.StatsSchema(_PLAN_SCHEMA, parts)
    n_nodes = 0
    for _ in range(3000):
        p = _random_predicate(rnd, 4)
        pf, df = sk.split_filters(p, parts)
        opf, odf = osf.split(p, parts)
        assert (pf, df) == (opf, odf), p
        if df is None:
            continue
        got, want = sk.construct(df, leaves), osf.build(df, S)
        assert got == want, (p, got, want)
        if want is None:
            continue
        n_nodes += 1
        try:
            osf.check(want, S)
            bad = None
        except osf.Incomparable as e:
            bad = e
        if bad is None:
            sk.check_types(got, leaves)
        else:
            with pytest.raises(sk.UnsupportedExpression):
                sk.check_types(got, leaves)
    assert n_nodes > 1000
