"""Partition pruning (delta_amd/partitions.py planner, k_part_eval on the GPU, oracle/partitions.py).

The oracle is cross-checked against an independent filter over the reference golden table
dv-partitioned-with-checkpoint's expected scan files (tests/golden/expected.json, integer partition
column `part`, a checkpoint plus a commit tail), then the GPU path is compared with the oracle there,
on a synthetic table with a string partition column, together with data skipping, and on
hand-written logs with null, missing, malformed and out-of-range partition values.
"""
import json
import os

import pytest

from delta_amd import partitions as pp
from delta_amd import skipping as sk
from delta_amd import synth
from delta_amd.expressions import And, Column, Literal, Or, Predicate
from tests.golden_util import TABLES, load_expected
from tests.test_skipping import oracle_skipping, table_metadata

DV_PART = os.path.join(TABLES, "dv-partitioned-with-checkpoint")


def col(n):
    return Column(n)


def cmp(op, c, v):
    return Predicate(op, c, v)


def fields_of(root):
    schema, parts = table_metadata(root)
    return pp.partition_fields(schema, parts)


def oracle_files(root, predicate, bs=1024):
    from delta_amd import skipping as sk
    from oracle import ref
    schema, parts = table_metadata(root)
    from oracle import skipping_filter as osf
    pf, df = osf.split(predicate, parts)
    part = (pf, pp.partition_fields(schema, parts)) if pf is not None else None
    skip = oracle_skipping(root, df) if df is not None else None
    r = ref.replay(root, json_batch_size=bs, with_stats=skip is not None, skipping=skip, partition=part)
    return r.scan_files(), r.counters.as_tuple()


# ---------------------------------------------------------------- planner (host logic, CPU)
def test_partition_fields_and_compile():
    schema = json.dumps({"type": "struct", "fields": [
        {"name": "P", "type": "integer", "metadata": {"delta.columnMapping.physicalName": "col-p"}},
        {"name": "s", "type": "string", "metadata": {}}, {"name": "d", "type": "date", "metadata": {}},
        {"name": "x", "type": "long", "metadata": {}}]})
    f = pp.partition_fields(schema, ["p", "S", "d"])
    assert f == {"p": ("integer", "col-p"), "s": ("string", "s"), "d": ("date", "d")}
    d = _describe(And(cmp(">=", col("P"), Literal.ofInt(3)), cmp("=", col("s"), Literal.ofString("a b"))), f)
    assert [x["name"] for x in d["fields"]] == ["col-p", "s"] and [x["type"] for x in d["fields"]] == [1, 4]
    assert [o[0] for o in d["ops"]] == [PO_FIELD, PO_LIT_INT, PO_GE, PO_FIELD, PO_LIT_STR, PO_EQ, PO_AND]
    d = _describe(cmp("<", col("d"), Literal.ofDate(10957)), f)
    assert [x["type"] for x in d["fields"]] == [5] and d["ops"][1] == [PO_LIT_INT, 0, 10957]
    # differently typed operands without an up-cast throw, as transformBinaryComparator does
    for bad in (cmp("=", col("d"), Literal.ofInt(1)), cmp("=", col("s"), Literal.ofInt(1)),
                cmp("=", col("d"), Literal.ofString("2000-01-01")), cmp("=", col("p"), Literal.ofNull("string"))):
        with pytest.raises(sk.UnsupportedExpression, match="not comparable"):
            _describe(bad, f)
    _describe(cmp("=", col("p"), Literal.ofLong(1)), f)                # integer -> long up-cast
    with pytest.raises(ValueError):
        _describe(cmp("=", col("zz"), Literal.ofInt(1)), f)
    # COALESCE / ALWAYS_TRUE / ALWAYS_FALSE compile; a predicate the device does not evaluate is refused
    _describe(Predicate("COALESCE", cmp("=", col("p"), Literal.ofInt(1)), Predicate("ALWAYS_FALSE")), f)
    _describe(Predicate("LIKE", col("s"), Literal.ofString("a%")), f)
    _describe(cmp("=", Predicate("SUBSTRING", col("s"), Literal.ofInt(2)), Literal.ofString("b")), f)
    with pytest.raises(sk.UnsupportedExpression, match="STRING"):
        _describe(Predicate("STARTS_WITH", col("p"), Literal.ofString("1")), f)
    with pytest.raises(sk.UnsupportedExpression, match="single character"):
        _describe(Predicate("LIKE", col("s"), Literal.ofString("a%"), Literal.ofString("ab")), f)
    # a per-row LIKE pattern compiles to the device's dynamic LIKE (PO_LIKE_DYN = 21, escape in arg)
    d = _describe(Predicate("LIKE", col("s"), col("s")), f)
    assert [o[0] for o in d["ops"]] == [PO_FIELD, PO_FIELD, 21] and d["ops"][2][1] == ord("\\")


(PO_FIELD, PO_LIT_INT, PO_LIT_STR, PO_LIT_NULL, PO_LT, PO_LE, PO_GT, PO_GE, PO_EQ, PO_NSEQ, PO_ISNULL,
 PO_ISNOTNULL, PO_NOT, PO_AND, PO_OR, PO_LIT_DEC, PO_FCMP, PO_COALESCE) = range(18)


def _describe(pred, fields):
    from delta_amd import programs
    return programs.compile_partition(pred, fields).describe()


def test_program_unbounded():
    """No size caps: 40 partition columns, an OR of 300 equalities (re-associated under the device
    stack), a 10 KiB string literal."""
    f = {"c%d" % i: ("integer", "c%d" % i) for i in range(40)}
    f["s"] = ("string", "s")
    big = Predicate("AND", cmp(">=", col("c0"), Literal.ofInt(0)), cmp("=", col("c39"), Literal.ofInt(5)))
    for i in range(1, 39):
        big = Predicate("AND", big, cmp("<", col("c%d" % i), Literal.ofInt(i)))
    d = _describe(big, f)
    assert len(d["fields"]) == 40 and d["stack"] <= 32
    ors = cmp("=", col("c1"), Literal.ofInt(0))
    for i in range(1, 300):
        ors = Predicate("OR", ors, cmp("=", col("c1"), Literal.ofInt(i)))
    d = _describe(ors, f)
    assert d["stack"] <= 32 and sum(o[0] == PO_OR for o in d["ops"]) == 299
    right = cmp("=", col("c1"), Literal.ofInt(0))
    for i in range(1, 300):                                    # right-deep: balanced by the compiler
        right = Predicate("OR", cmp("=", col("c1"), Literal.ofInt(i)), right)
    assert _describe(right, f)["stack"] <= 32
    lit = "x" * 10240
    d = _describe(cmp("=", col("s"), Literal.ofString(lit)), f)
    assert bytes.fromhex(d["pool"]).find(lit.encode()) >= 0


# ---------------------------------------------------------------- oracle (cross-checked)
PART_PREDICATES = [
    cmp(">=", col("part"), Literal.ofInt(7)),
    cmp("=", col("part"), Literal.ofInt(3)),
    Or(cmp("<", col("part"), Literal.ofInt(2)), cmp(">", col("part"), Literal.ofLong(8))),
    Predicate("NOT", cmp("<", col("part"), Literal.ofInt(5))),
    Predicate("IS_NULL", col("part")),
    Predicate("IS_NOT_NULL", col("part")),
    cmp("IS NOT DISTINCT FROM", col("part"), Literal.ofNull("integer")),
    cmp("IS NOT DISTINCT FROM", col("PART"), Literal.ofInt(4)),
    cmp("=", col("part"), Literal.ofNull("integer")),
]


def _pv_part(row):
    """`part` of an expected.json scan-file row (index 1 = partitionValues pairs)."""
    for k, v in row[1] or []:
        if (k["b"] if isinstance(k, dict) else k) == "part":
            return None if v is None else int(v["b"] if isinstance(v, dict) else v)
    return None


def _reference_filter(pred, part):
    """The same predicates written out directly over one integer value (None = null)."""
    n = pred.name.upper()
    c = pred.children
    if n == "OR":
        a, b = _reference_filter(c[0], part), _reference_filter(c[1], part)
        return True if (a or b) else (False if (a is False and b is False) else None)
    if n == "NOT":
        a = _reference_filter(c[0], part)
        return None if a is None else not a
    if n == "IS_NULL":
        return part is None
    if n == "IS_NOT_NULL":
        return part is not None
    lit = c[1].value
    if n == "IS NOT DISTINCT FROM":
        return part == lit
    if part is None or lit is None:
        return None
    return {"<": part < lit, ">": part > lit, ">=": part >= lit, "=": part == lit}[n]


@pytest.mark.parametrize("pred", PART_PREDICATES)
def test_oracle_partition_pruning_golden(pred):
    rows = load_expected()["dv-partitioned-with-checkpoint"]["1024-0"]["rows"]
    want = sorted(r[0]["b"] for r in rows if _reference_filter(pred, _pv_part(r)) is True)
    got, counters = oracle_files(DV_PART, pred)
    assert sorted(r[0].decode() for r in got) == want
    assert list(counters) == load_expected()["dv-partitioned-with-checkpoint"]["1024-0"]["counters"]


def _write_pv_table(root, pvs, schema_type="integer"):
    log = os.path.join(root, "_delta_log")
    os.makedirs(log)
    schema = {"type": "struct", "fields": [{"name": "p", "type": schema_type, "nullable": True, "metadata": {}},
                                           {"name": "id", "type": "long", "nullable": True, "metadata": {}}]}
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        f.write(json.dumps({"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}}) + "\n")
        f.write(json.dumps({"metaData": {"id": "t", "format": {"provider": "parquet", "options": {}},
                                         "schemaString": json.dumps(schema), "partitionColumns": ["p"],
                                         "configuration": {}, "createdTime": 0}}) + "\n")
        for i, pv in enumerate(pvs):
            f.write(json.dumps({"add": {"path": "p%d.parquet" % i, "partitionValues": pv, "size": 1,
                                        "modificationTime": 0, "dataChange": True}}) + "\n")


EDGE_PVS = [{"p": "5"}, {"p": None}, {}, {"p": "+7"}, {"p": "-3"}, {"p": "0005"}, {"q": "5"}, {"p": "2147483647"}]


def test_oracle_edge_values(tmp_path):
    root = str(tmp_path / "t")
    _write_pv_table(root, EDGE_PVS)
    got = lambda p: sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0])   # noqa: E731
    assert got(cmp("=", col("p"), Literal.ofInt(5))) == [0, 5]
    assert got(Predicate("IS_NULL", col("p"))) == [1, 2, 6]
    assert got(cmp(">", col("p"), Literal.ofInt(0))) == [0, 3, 5, 7]
    assert got(Predicate("NOT", cmp(">", col("p"), Literal.ofInt(0)))) == [4]


@pytest.mark.parametrize("bad", ["x", "", "1.0", "2147483648", " 1", "0x10"])
def test_oracle_malformed_value_raises(tmp_path, bad):
    from oracle import partitions as opp
    root = str(tmp_path / "t")
    _write_pv_table(root, [{"p": "1"}, {"p": bad}])
    with pytest.raises(opp.PartitionValueError):
        oracle_files(root, cmp("=", col("p"), Literal.ofInt(1)))


# ---------------------------------------------------------------- GPU parity
def _gpu_files(root, predicate, eng):
    from tests.test_skipping import _gpu_files as gf
    return gf(root, predicate, eng)


@pytest.mark.gpu
def test_gpu_partition_pruning_golden():
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    for pred in PART_PREDICATES + [And(cmp(">=", col("part"), Literal.ofInt(7)), cmp(">=", col("col1"), Literal.ofInt(0))),
                                   And(cmp(">=", col("part"), Literal.ofInt(7)), cmp("=", col("col1"), Literal.ofInt(28)))]:
        assert _gpu_files(DV_PART, pred, eng) == oracle_files(DV_PART, pred), pred
    eng.close()


@pytest.mark.gpu
def test_gpu_partition_pruning_synthetic(tmp_path):
    from delta_amd import kernel as K
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=30_000, n_parts=2, n_commits=5, dv_frac=0.1,
                                                     ckpt_removes=100, with_stats=True, pv_keys=2))
    eng = K.GpuEngine()
    day = Literal.ofString("2024-06-01")
    for pred in (cmp(">=", col("date"), day), cmp("=", col("date"), Literal.ofString("2024-01-01")),
                 Or(cmp("<", col("date"), day), Predicate("IS_NULL", col("date"))),
                 And(cmp("<", col("date"), day), cmp(">", col("id"), Literal.ofLong(30_000_000)))):
        g = _gpu_files(str(tmp_path), pred, eng)
        o = oracle_files(str(tmp_path), pred)
        assert g[1] == o[1] and len(g[0]) == len(o[0]) and g[0] == o[0], pred
    eng.close()


@pytest.mark.gpu
def test_gpu_partition_edge_values(tmp_path):
    from delta_amd import kernel as K
    root = str(tmp_path / "t")
    _write_pv_table(root, EDGE_PVS)
    eng = K.GpuEngine()
    for pred in (cmp("=", col("p"), Literal.ofInt(5)), Predicate("IS_NULL", col("p")),
                 cmp(">", col("p"), Literal.ofInt(0)), Predicate("NOT", cmp(">", col("p"), Literal.ofInt(0))),
                 cmp("IS NOT DISTINCT FROM", col("p"), Literal.ofNull("integer"))):
        assert _gpu_files(root, pred, eng) == oracle_files(root, pred), pred
    eng.close()


@pytest.mark.gpu
def test_gpu_malformed_value_raises(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    eng = K.GpuEngine()
    for i, bad in enumerate(["x", "", "1.0", "2147483648", " 1", "0x10"]):
        root = str(tmp_path / str(i))
        _write_pv_table(root, [{"p": "1"}, {"p": bad}])
        with pytest.raises(DkError, match="partition"):
            _gpu_files(root, cmp("=", col("p"), Literal.ofInt(1)), eng)
    eng.close()


def _days(text):
    import datetime
    return (datetime.date.fromisoformat(text) - datetime.date(1970, 1, 1)).days


# PartitionValueEvaluator.java:72-73: daysSinceEpoch(java.sql.Date.valueOf(value))
DATE_PVS = [{"p": "2000-01-01"}, {"p": None}, {"p": "2000-1-2"}, {"p": "2021-02-30"}, {"p": "2021-+3-01"},
            {}, {"p": "1999-12-31"}, {"p": "9999-12-31"}]
DATE_PREDICATES = [cmp("=", col("p"), Literal.ofDate(_days("2000-01-02"))),
                   cmp(">=", col("p"), Literal.ofDate(_days("2021-03-02"))),
                   cmp("<", col("p"), Literal.ofDate(_days("2000-01-02"))),
                   Or(Predicate("IS_NULL", col("p")), cmp("=", col("p"), Literal.ofDate(_days("2021-03-01")))),
                   cmp("IS NOT DISTINCT FROM", col("p"), Literal.ofNull("date"))]
DATE_BAD_PVS = ["2000-13-01", "1500-01-01", "2000-01", "x", "", "2000-01-01 "]


def test_oracle_date_partition_values(tmp_path):
    from oracle import partitions as opp
    root = str(tmp_path / "t")
    _write_pv_table(root, DATE_PVS, "date")
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in DATE_PREDICATES]
    assert got == [[2], [3, 7], [0, 6], [1, 4, 5], [1, 5]]    # row 3 is 2021-03-02 (lenient carry)
    for i, bad in enumerate(DATE_BAD_PVS):
        r = str(tmp_path / ("b%d" % i))
        _write_pv_table(r, [{"p": "2000-01-01"}, {"p": bad}], "date")
        with pytest.raises(opp.PartitionValueError):
            oracle_files(r, DATE_PREDICATES[0])


@pytest.mark.gpu
def test_gpu_date_partition_values(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    root = str(tmp_path / "t")
    _write_pv_table(root, DATE_PVS, "date")
    eng = K.GpuEngine()
    for pred in DATE_PREDICATES:
        assert _gpu_files(root, pred, eng) == oracle_files(root, pred), pred
    for i, bad in enumerate(DATE_BAD_PVS):
        r = str(tmp_path / ("b%d" % i))
        _write_pv_table(r, [{"p": "2000-01-01"}, {"p": bad}], "date")
        with pytest.raises(DkError, match="partition"):
            _gpu_files(r, DATE_PREDICATES[0], eng)
    eng.close()


# PartitionValueEvaluator.java:112-113: new BigDecimal(value), compared with compareTo
DEC_PVS = [{"p": "1.50"}, {"p": "1.5"}, {"p": "-0.001"}, {"p": "1E+1"}, {"p": ".5"}, {"p": None}, {"p": "0.00"},
           {"p": "+10"}, {"p": "-1e-3"}, {"p": "123456789012345678901234567890.5"}, {"p": "2."}]
# literals of the column's type decimal(38,3) (differently typed decimals are not comparable)
DEC_PREDICATES = [cmp("=", col("p"), Literal.ofDecimal("1.5", 38, 3)),
                  cmp(">", col("p"), Literal.ofDecimal("1.499", 38, 3)),
                  cmp("<", col("p"), Literal.ofDecimal("0", 38, 3)),
                  cmp("=", col("p"), Literal.ofDecimal("10", 38, 3)),
                  cmp("<=", col("p"), Literal.ofDecimal("0.5000", 38, 3)),
                  Or(Predicate("IS_NULL", col("p")), cmp(">=", col("p"), Literal.ofDecimal("1E+29", 38, 3)))]
DEC_BAD_PVS = ["x", "", "1.2.3", "1e", " 1", "e5", "1e99999999999", "\u0661"]


def test_oracle_decimal_partition_values(tmp_path):
    from oracle import partitions as opp
    root = str(tmp_path / "t")
    _write_pv_table(root, DEC_PVS, "decimal(38,3)")
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in DEC_PREDICATES]
    assert got == [[0, 1], [0, 1, 3, 7, 9, 10], [2, 8], [3, 7], [2, 4, 6, 8], [5, 9]]
    for i, bad in enumerate(DEC_BAD_PVS):
        r = str(tmp_path / ("b%d" % i))
        _write_pv_table(r, [{"p": "1"}, {"p": bad}], "decimal(38,3)")
        with pytest.raises(opp.PartitionValueError):
            oracle_files(r, DEC_PREDICATES[0])


@pytest.mark.gpu
def test_gpu_decimal_partition_values(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    root = str(tmp_path / "t")
    _write_pv_table(root, DEC_PVS, "decimal(38,3)")
    eng = K.GpuEngine()
    for pred in DEC_PREDICATES:
        assert _gpu_files(root, pred, eng) == oracle_files(root, pred), pred
    for i, bad in enumerate(DEC_BAD_PVS):
        r = str(tmp_path / ("b%d" % i))
        _write_pv_table(r, [{"p": "1"}, {"p": bad}], "decimal(38,3)")
        with pytest.raises(DkError, match="partition"):
            _gpu_files(r, DEC_PREDICATES[0], eng)
    eng.close()


# ---------------------------------------------------------------- boolean / float / double / timestamp
# PartitionPruningSuite.scala:37-97 on golden data-reader-partition-values: `col = value` keeps the one
# partition holding the value (two for date and timestamp), `col = null` keeps nothing
PV_TABLE = os.path.join(TABLES, "data-reader-partition-values")
PV_CASES = [(col("as_boolean"), Literal.ofBoolean(False), Literal.ofNull("boolean"), 1),
            (col("as_byte"), Literal.ofByte(1), Literal.ofNull("byte"), 1),
            (col("as_short"), Literal.ofShort(1), Literal.ofNull("short"), 1),
            (col("as_int"), Literal.ofInt(1), Literal.ofNull("integer"), 1),
            (col("as_long"), Literal.ofLong(1), Literal.ofNull("long"), 1),
            (col("as_float"), Literal.ofFloat(1), Literal.ofNull("float"), 1),
            (col("as_double"), Literal.ofDouble(1), Literal.ofNull("double"), 1),
            (col("as_date"), Literal.ofDate(18878), Literal.ofNull("date"), 2),
            (col("as_string"), Literal.ofString("1"), Literal.ofNull("string"), 1),
            (col("as_timestamp"), Literal.ofTimestamp(1631099471000000), Literal.ofNull("timestamp"), 2),
            (col("as_big_decimal"), Literal.ofDecimal(1, 1, 0), Literal.ofNull("decimal(1,0)"), 1)]
# :99-160 (combinations; the data-column halves only add a data filter, so the partition side decides)
PV_COMBOS = [(And(cmp(">=", col("as_float"), Literal.ofFloat(-200)), cmp("=", col("as_date"), Literal.ofDate(18878))), 2),
             (Or(cmp("=", col("as_float"), Literal.ofFloat(0)), cmp("=", col("as_int"), Literal.ofInt(1))), 2),
             (cmp("=", col("as_float"), Literal.ofFloat(0)), 1),
             (cmp("=", col("as_float"), Literal.ofFloat(234)), 0)]
# :197-255 on data-reader-timestamp_ntz[-name-mode|-id-mode]: files (not rows) per predicate
NTZ_TABLES = ["data-reader-timestamp_ntz", "data-reader-timestamp_ntz-name-mode", "data-reader-timestamp_ntz-id-mode"]
NTZ_CASES = [(cmp("=", col("tsNtzPartition"), Literal.ofTimestampNtz(1637202600123456)), 1),
             (cmp("=", col("tsNtzPartition"), Literal.ofNull("timestamp_ntz")), 0),
             (cmp(">=", col("tsNtzPartition"), Literal.ofTimestampNtz(1373043660123456)), 3),
             (Predicate("IS_NULL", col("tsNtzPartition")), 1)]


def test_oracle_partition_values_golden():
    for c, value, null, n in PV_CASES:
        assert len(oracle_files(PV_TABLE, cmp("=", c, value))[0]) == n, c
        assert oracle_files(PV_TABLE, cmp("=", c, null))[0] == [], c
    for pred, n in PV_COMBOS:
        assert len(oracle_files(PV_TABLE, pred)[0]) == n, pred
    for name in NTZ_TABLES:
        for pred, n in NTZ_CASES:
            assert len(oracle_files(os.path.join(TABLES, name), pred)[0]) == n, (name, pred)


@pytest.mark.gpu
def test_gpu_partition_values_golden():
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    preds = [cmp("=", c, v) for c, value, null, _ in PV_CASES for v in (value, null)] + [p for p, _ in PV_COMBOS]
    for pred in preds:
        assert _gpu_files(PV_TABLE, pred, eng) == oracle_files(PV_TABLE, pred), pred
    for name in NTZ_TABLES:
        root = os.path.join(TABLES, name)
        for pred, _ in NTZ_CASES:
            assert _gpu_files(root, pred, eng) == oracle_files(root, pred), (name, pred)
    eng.close()


# Float.parseFloat / Double.parseDouble values (PartitionValueEvaluator.java:93-100)
FLOAT_PVS = [{"p": "1.0"}, {"p": "-0.0"}, {"p": "0"}, {"p": "NaN"}, {"p": "Infinity"}, {"p": "-Infinity"},
             {"p": "1e50"}, {"p": "-1e-50"}, {"p": " 1.5f "}, {"p": "16777217"}, {"p": "0.1"}, {"p": None},
             {"p": "+.5e1D"}, {"p": "3.4028235677973366E38"}]
FLOAT_PREDICATES = [cmp("=", col("p"), Literal.ofFloat(1.0)), cmp("<", col("p"), Literal.ofFloat(0.0)),
                    cmp(">=", col("p"), Literal.ofFloat(-0.0)), cmp("=", col("p"), Literal.ofFloat(float("nan"))),
                    cmp(">", col("p"), Literal.ofFloat(3e38)), cmp("=", col("p"), Literal.ofFloat(16777216)),
                    cmp("=", col("p"), Literal.ofDouble(0.1)), cmp("<", Literal.ofFloat(1.25), col("p")),
                    cmp("IS NOT DISTINCT FROM", col("p"), Literal.ofFloat(float("inf"))),
                    cmp("IS NOT DISTINCT FROM", col("p"), Literal.ofNull("float")),
                    cmp("=", col("p"), Literal.ofInt(5)), Predicate("NOT", cmp("<=", col("p"), Literal.ofFloat(1.5)))]
FLOAT_BAD_PVS = ["x", "", "1e", "NaNf", ".", "1.0.0", "Inf", "--1"]


def test_oracle_float_partition_values(tmp_path):
    from oracle import partitions as opp
    root = str(tmp_path / "t")
    _write_pv_table(root, FLOAT_PVS, "float")
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in FLOAT_PREDICATES]
    # worked by hand: "-0.0" and "-1e-50" are -0.0f (below 0.0f); "1e50" overflows to Infinity while
    # 3.4028235677973366E38 stays Float.MAX_VALUE (below the overflow tie); NaN is above everything;
    # 16777217 rounds to 2^24; 0.1f widened to double is not 0.1d; the int literal 5 widens to 5.0f
    assert got == [[0], [1, 5, 7], [0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 12, 13], [3], [3, 4, 6, 13], [9], [],
                   [3, 4, 6, 8, 9, 12, 13],
                   [4, 6], [11], [12], [3, 4, 6, 9, 12, 13]]
    for i, bad in enumerate(FLOAT_BAD_PVS):
        r = str(tmp_path / ("b%d" % i))
        _write_pv_table(r, [{"p": "1"}, {"p": bad}], "float")
        with pytest.raises(opp.PartitionValueError):
            oracle_files(r, FLOAT_PREDICATES[0])


@pytest.mark.gpu
def test_gpu_float_partition_values(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    eng = K.GpuEngine()
    for typ in ("float", "double"):
        root = str(tmp_path / typ)
        _write_pv_table(root, FLOAT_PVS, typ)
        for pred in FLOAT_PREDICATES:
            assert _gpu_files(root, pred, eng) == oracle_files(root, pred), (typ, pred)
    root = str(tmp_path / "int")
    _write_pv_table(root, [{"p": "16777217"}, {"p": "16777218"}, {"p": "-3"}, {"p": None}], "integer")
    for pred in (cmp("=", col("p"), Literal.ofFloat(16777216)), cmp(">", col("p"), Literal.ofDouble(-2.5)),
                 cmp("<", col("p"), Literal.ofFloat(float("nan")))):
        assert _gpu_files(root, pred, eng) == oracle_files(root, pred), pred
    for i, bad in enumerate(FLOAT_BAD_PVS):
        r = str(tmp_path / ("b%d" % i))
        _write_pv_table(r, [{"p": "1"}, {"p": bad}], "float")
        with pytest.raises(DkError, match="partition"):
            _gpu_files(r, FLOAT_PREDICATES[0], eng)
    eng.close()


BOOL_PVS = [{"p": "true"}, {"p": "TRUE"}, {"p": "false"}, {"p": "yes"}, {"p": ""}, {"p": None}, {"p": "True "}]
BOOL_PREDICATES = [cmp("=", col("p"), Literal.ofBoolean(True)), cmp("<", col("p"), Literal.ofBoolean(True)),
                   Predicate("NOT", cmp("=", col("p"), Literal.ofBoolean(False)))]
# java.sql.Timestamp.valueOf: lenient field rollover, 1-2 digit month/day, optional 1-9 digit fraction
TS_PVS = [{"p": "2021-09-08 11:11:11"}, {"p": "2021-9-8 11:11:11.5"}, {"p": "2021-09-07 35:11:11"},
          {"p": "2021-09-08 11:11:10.999999999"}, {"p": None}, {"p": " 2021-09-08 11:11:11.000001 "},
          {"p": "1969-12-31 23:59:59.9999995"}, {"p": "2021-02-30 00:00:00"}]
TS_PREDICATES = [cmp("=", col("p"), Literal.ofTimestamp(1631099471000000)),
                 cmp(">", col("p"), Literal.ofTimestamp(1631099471000000)),
                 cmp("<", col("p"), Literal.ofTimestamp(0)),
                 cmp("=", col("p"), Literal.ofTimestamp(1614643200000000))]
TS_BAD_PVS = ["2021-09-08T11:11:11", "2021-09-08 11:11", "2021-09-08", "x", "2021-09-08 11:11:11.", "1500-01-01 00:00:00",
              "2021-13-01 00:00:00", "2021-09-08 11:11:11.1234567890"]


def test_oracle_bool_timestamp_partition_values(tmp_path):
    from oracle import partitions as opp
    root = str(tmp_path / "b")
    _write_pv_table(root, BOOL_PVS, "boolean")
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in BOOL_PREDICATES]
    assert got == [[0, 1], [2, 3, 4, 6], [0, 1]]          # "True " is not "true": parseBoolean does not trim
    root = str(tmp_path / "t")
    _write_pv_table(root, TS_PVS, "timestamp")
    got = [sorted(int(r[0].decode()[1:-8]) for r in oracle_files(root, p)[0]) for p in TS_PREDICATES]
    # row 2: 35:11:11 on the 7th rolls over to the 8th 11:11:11; row 6 truncates toward zero to 0
    assert got == [[0, 2], [1, 5], [], [7]]
    for i, bad in enumerate(TS_BAD_PVS):
        r = str(tmp_path / ("x%d" % i))
        _write_pv_table(r, [{"p": "2021-09-08 11:11:11"}, {"p": bad}], "timestamp")
        with pytest.raises(opp.PartitionValueError):
            oracle_files(r, TS_PREDICATES[0])


@pytest.mark.gpu
def test_gpu_bool_timestamp_partition_values(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    eng = K.GpuEngine()
    root = str(tmp_path / "b")
    _write_pv_table(root, BOOL_PVS, "boolean")
    for pred in BOOL_PREDICATES:
        assert _gpu_files(root, pred, eng) == oracle_files(root, pred), pred
    for typ in ("timestamp", "timestamp_ntz"):
        root = str(tmp_path / typ)
        _write_pv_table(root, TS_PVS, typ)
        lit = Literal.ofTimestamp if typ == "timestamp" else Literal.ofTimestampNtz
        for p in TS_PREDICATES:
            pred = cmp(p.name, p.children[0], lit(p.children[1].value))
            assert _gpu_files(root, pred, eng) == oracle_files(root, pred), (typ, pred)
    for i, bad in enumerate(TS_BAD_PVS):
        r = str(tmp_path / ("x%d" % i))
        _write_pv_table(r, [{"p": "2021-09-08 11:11:11"}, {"p": bad}], "timestamp")
        with pytest.raises(DkError, match="partition"):
            _gpu_files(r, TS_PREDICATES[0], eng)
    eng.close()


# ---------------------------------------------------------------- checkpoint row-group pruning
# ActionsIterator.java:336-351: the partition filter, rewritten onto add.partitionValues_parsed,
# prunes row groups of multi-part parts and sidecars by their footer statistics
# (ParquetFileReader.java:111-132, ParquetFilterUtils.toParquetFilter, parquet-mr StatisticsFilter);
# pruned rows are never read, so the ScanMetrics counters shrink too.
def _rewrite_with_parsed(root, rg_rows=700):
    """Give every checkpoint part of a synth table an integer partition column `part` (0..9 by date)
    and add.partitionValues_parsed {date, part}, sorted by part, in small row groups."""
    import glob
    import pyarrow as pa
    import pyarrow.parquet as pq
    for path in sorted(glob.glob(os.path.join(root, "_delta_log", "*.checkpoint.*.parquet"))):
        t = pq.read_table(path)
        add = t.column("add").combine_chunks()
        pvs = add.field("partitionValues").to_pylist()
        valid = add.is_valid().to_pylist()
        dates = [dict(pv).get("date") if (ok and pv is not None) else None for ok, pv in zip(valid, pvs)]
        parts = [None if d is None else int(d.replace("-", "")) % 10 for d in dates]
        new_pv = [None if not ok else (list(pv or []) + [("part", str(p))]) for ok, pv, p in zip(valid, pvs, parts)]
        parsed = pa.StructArray.from_arrays([pa.array(dates, pa.string()), pa.array(parts, pa.int32())],
                                            names=["date", "part"], mask=pa.array([not v for v in valid]))
        fields = [add.field(i) for i in range(add.type.num_fields)]
        names = [add.type[i].name for i in range(add.type.num_fields)]
        fields[names.index("partitionValues")] = pa.array(new_pv, add.type.field("partitionValues").type)
        new_add = pa.StructArray.from_arrays(fields + [parsed], names=names + ["partitionValues_parsed"],
                                             mask=pa.array([not v for v in valid]))
        t = t.set_column(t.schema.get_field_index("add"), "add", new_add)
        if "metaData" in t.schema.names:
            md = t.column("metaData").combine_chunks()
            rows = md.to_pylist()
            for r in rows:
                if r is not None:
                    sch = json.loads(r["schemaString"])
                    if not any(f["name"] == "part" for f in sch["fields"]):
                        sch["fields"].append({"name": "part", "type": "integer", "nullable": True, "metadata": {}})
                    r["schemaString"] = json.dumps(sch)
                    r["partitionColumns"] = ["date", "part"]
            t = t.set_column(t.schema.get_field_index("metaData"), "metaData", pa.array(rows, md.type))
        order = sorted(range(t.num_rows), key=lambda i: (-1 if parts[i] is None else parts[i], i))
        t = t.take(pa.array(order))
        pq.write_table(t, path, row_group_size=rg_rows, compression="snappy")


RG_PREDICATES = [cmp(">", col("part"), Literal.ofInt(6)), cmp("=", col("part"), Literal.ofInt(3)),
                 Predicate("NOT", cmp("<", col("part"), Literal.ofInt(7))),
                 Or(cmp("<", col("part"), Literal.ofInt(2)), cmp(">", col("part"), Literal.ofLong(8))),
                 Predicate("IS_NULL", col("part")), Predicate("IS_NOT_NULL", col("part")),
                 cmp("<", Literal.ofInt(5), col("part")),              # swapped without flipping: lt(part, 5)
                 And(cmp(">=", col("part"), Literal.ofInt(4)), cmp("<", col("date"), Literal.ofString("2024-07-01"))),
                 cmp("=", col("date"), Literal.ofString("2024-03-15")),
                 cmp("IS NOT DISTINCT FROM", col("part"), Literal.ofInt(2)),   # not convertible: no pruning
                 cmp(">", col("part"), Literal.ofLong(1 << 40))]           # long literal beyond int: none


@pytest.fixture(scope="module")
def rg_table(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("rgprune"))
    synth.write_table(d, synth.TableSpec(n_adds=12_000, n_parts=3, n_commits=4, compression="snappy"))
    _rewrite_with_parsed(d)
    return d


def test_oracle_row_group_pruning(rg_table):
    from oracle import ref
    full = ref.replay(rg_table).counters.as_tuple()
    seen = {}
    for p in RG_PREDICATES:
        files, counters = oracle_files(rg_table, p)
        seen[repr(p)] = counters[0]
        assert counters[0] <= full[0]
    # row groups hold one `part` value each (sorted, 700 rows): range predicates prune
    assert seen[repr(RG_PREDICATES[0])] < full[0] and seen[repr(RG_PREDICATES[1])] < seen[repr(RG_PREDICATES[0])]
    assert seen[repr(RG_PREDICATES[9])] == full[0]         # IS NOT DISTINCT FROM does not convert


@pytest.mark.gpu
def test_gpu_row_group_pruning(rg_table):
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    for p in RG_PREDICATES:
        assert _gpu_files(rg_table, p, eng) == oracle_files(rg_table, p), p
    eng.close()


def wide_partition_predicates():
    """Past the old caps (8 columns, 64 ops, 4 KiB pool): an OR of 40 equalities, a 10 KiB string
    literal, COALESCE / ALWAYS_FALSE, and the three combined."""
    ors = cmp("=", col("part"), Literal.ofInt(0))
    for k in range(1, 40):
        ors = Or(ors, cmp("=", col("part"), Literal.ofInt(k % 3 if k % 2 else 100 + k)))
    big = cmp("<", col("date"), Literal.ofString("2024-06" + "z" * 10240))
    co = Predicate("COALESCE", cmp(">", col("part"), Literal.ofInt(5)), Predicate("ALWAYS_FALSE"))
    co1 = Predicate("COALESCE", cmp(">=", col("part"), Literal.ofInt(1)), Predicate("ALWAYS_FALSE"))
    return [ors, big, co, And(And(ors, big), Or(co1, Predicate("IS_NULL", col("part"))))]


def test_oracle_wide_partition_predicates(rg_table):
    from oracle import ref
    full = ref.replay(rg_table).counters.as_tuple()
    kept = [len(oracle_files(rg_table, p)[0]) for p in wide_partition_predicates()]
    assert all(0 < k < full[2] for k in kept), (kept, full)


def string_function_predicates():
    """STARTS_WITH / LIKE / SUBSTRING over the string partition column (ExpressionVisitor.java:118-123)."""
    d = col("date")
    sub = lambda *a: Predicate("SUBSTRING", d, *[Literal.ofInt(x) for x in a])   # noqa: E731
    return [Predicate("STARTS_WITH", d, Literal.ofString("2024-0")),
            Predicate("LIKE", d, Literal.ofString("2024-_3-%")),
            Predicate("LIKE", d, Literal.ofString("%1_")),
            Predicate("LIKE", d, Literal.ofString("2024-0%!%"), Literal.ofString("!")),
            Predicate("NOT", Predicate("LIKE", d, Literal.ofString("%-0_-%"))),
            cmp("=", sub(6, 2), Literal.ofString("03")),
            cmp(">", sub(-2), Literal.ofString("15")),
            cmp("=", sub(0, 4), Literal.ofString("2024")),
            cmp("=", sub(-100, 95), Literal.ofString("")),
            And(Predicate("STARTS_WITH", d, Literal.ofString("2024-1")), cmp(">", col("part"), Literal.ofInt(3)))]


def test_oracle_string_function_predicates(rg_table):
    from oracle import ref
    full = ref.replay(rg_table).counters.as_tuple()
    kept = [len(oracle_files(rg_table, p)[0]) for p in string_function_predicates()]
    assert sum(0 < k < full[2] for k in kept) >= 6, kept
    from oracle import partitions as opp
    with pytest.raises(opp.PartitionValueError):       # an invalid escape fails the evaluation
        oracle_files(rg_table, Predicate("LIKE", col("date"), Literal.ofString("2024!-%"), Literal.ofString("!")))


@pytest.mark.gpu
def test_gpu_string_function_predicates(rg_table):
    """The string functions of string_function_predicates on the GPU equal the oracle; an invalid LIKE
    escape fails the scan as the reference's evaluator does."""
    from delta_amd import kernel as K
    from delta_amd.skipping import UnsupportedExpression
    eng = K.GpuEngine()
    for p in string_function_predicates():
        assert _gpu_files(rg_table, p, eng) == oracle_files(rg_table, p), p
    with pytest.raises(UnsupportedExpression, match="invalid escape"):
        _gpu_files(rg_table, Predicate("LIKE", col("date"), Literal.ofString("2024!-%"), Literal.ofString("!")), eng)
    eng.close()


@pytest.mark.gpu
def test_gpu_wide_partition_predicates(rg_table):
    """wide_partition_predicates on the GPU (partition pruning over add.partitionValues, and the
    checkpoint row-group predicate over partitionValues_parsed) equal the oracle."""
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    for p in wide_partition_predicates():
        assert _gpu_files(rg_table, p, eng) == oracle_files(rg_table, p), p
    eng.close()


@pytest.mark.gpu
def test_gpu_row_group_pruning_sharded(rg_table):
    """Pruned row groups are left out before the shard plan; the merged shards equal the oracle."""
    from delta_amd import kernel as K
    from delta_amd import shard as S
    from oracle import ref
    eng = K.GpuEngine()
    p = RG_PREDICATES[0]
    want = oracle_files(rg_table, p)
    outs, scans = [], []
    for r in range(3):
        snap = K.Table.forPath(eng, rg_table).getLatestSnapshot(eng)
        scan = snap.getScanBuilder().withFilter(p).withShard(3, r).build()
        batches = list(scan.getScanFiles(eng))
        o = S.ShardOutput(r, scan.tail_metrics.as_tuple(), scan.ckpt_metrics.as_tuple())
        for b in batches:
            if b.file_index < 0:
                o.tail = b
            else:
                o.files[(b.file_index, b.row_offset)] = b
        outs.append(o)
        scans.append(scan)
    counters, batches = S.merge(outs)
    rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in batches for i in b.selected_rows()]
    assert counters == want[1] and rows == want[0]
    for s in scans:
        s.close()
    eng.close()


def test_row_group_pruning_decisions_match_oracle(rg_table):
    """The product's per-file pruning (dk_parquet_prune_row_groups, host C++) against the oracle's
    independent restatement (oracle/rowgroups.py) for every predicate and part file (no GPU)."""
    import glob
    from delta_amd import kernel as K
    from delta_amd._lib import dk_rg_filter
    from oracle.rowgroups import surviving_row_groups
    schema, parts = table_metadata(rg_table)
    fields = pp.partition_fields(schema, parts)
    files = sorted(glob.glob(os.path.join(rg_table, "_delta_log", "*.checkpoint.*.parquet")))
    extra = [cmp(">=", col("date"), Literal.ofString("2024-10-01")), Predicate("NOT", cmp("=", col("part"), Literal.ofInt(0))),
             cmp("<=", col("part"), Literal.ofDate(3)), cmp("=", col("part"), Literal.ofString("3"))]
    for p in RG_PREDICATES + extra:
        packed = pp.pack_row_group_filter(pp.row_group_filter(p, fields), dk_rg_filter)
        for f in files:
            want = [g for g, k in enumerate(surviving_row_groups(f, p, fields)) if k]
            assert K.prune_row_groups(f, packed) == want, (p, f)


@pytest.mark.gpu
def test_gpu_filters_over_json_manifest_adds(tmp_path):
    """Partition pruning and data skipping over the add rows of a V2 JSON manifest (checkpoint rows
    read by the JSON handler, ActionsIterator.java:213-248) equal the oracle's."""
    from delta_amd import kernel as K
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=9_000, n_parts=2, v2_sidecars=2, v2_manifest="json",
                                                     v2_json_adds=300, n_commits=4, with_stats=True))
    eng = K.GpuEngine()
    for pred in (cmp("=", col("date"), Literal.ofString("2024-01-01")), cmp(">", col("date"), Literal.ofString("2024-01-01")),
                 cmp(">", col("id"), Literal.ofLong(30_000_000)),
                 And(cmp(">=", col("date"), Literal.ofString("2023-01-01")), cmp("<", col("id"), Literal.ofLong(1_000_000)))):
        g = _gpu_files(str(tmp_path), pred, eng)
        o = oracle_files(str(tmp_path), pred)
        assert g[1] == o[1] and g[0] == o[0], pred
    eng.close()
