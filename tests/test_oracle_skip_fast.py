"""The oracle's C fast path for integral data skipping (oracle/dk_skip.c) against the Python
restatement it stands in for (oracle/skipping.keep), row for row (CPU, test infrastructure)."""
import json

import numpy as np
import pytest

from oracle import ref
from oracle import skipping as sk

MIN_ID, MAX_ID, NULLS = ("minValues", "id"), ("maxValues", "id"), ("nullCount", "id")

EDGE = [
    '{"numRecords":10,"minValues":{"id":5},"maxValues":{"id":30000000},"nullCount":{"id":0}}',
    '{"numRecords":10,"minValues":{"id":5},"maxValues":{"id":25000000},"nullCount":{"id":0}}',
    '{"minValues":{"id":5},"maxValues":{"id":null}}',
    '{"minValues":{"id":5}}',
    '{"maxValues":null}',
    '{"maxValues":7}',                                    # not an object: decode error (Python raises)
    '{"maxValues":[1,2]}',
    '{"maxValues":{"id":"30000000"}}',                    # a string for a long: decode error
    '{"maxValues":{"id":3.0E7}}',                         # a decimal for a long: decode error
    '{"maxValues":{"id":30000000}, "maxValues":{"x":1}}', # last duplicate wins: id missing -> null
    '{"maxValues":{"x":1}, "maxValues":{"id":1}}',
    '{"maxValues":{"id":1,"id":99999999}}',
    '  \n{"maxValues":{"id":99999999}} trailing garbage',
    '{"maxValues":{"id":99999999}',                       # truncated: parse error
    '[1]',
    '"x"',
    '',
    '{"maxValues":{"id":9223372036854775807}}',
    '{"maxValues":{"id":9223372036854775808}}',           # out of range for long
    '{"maxValues":{"id":-9223372036854775808}}',
    '{"maxValues":{"id":-0}}',
    '{"maxValues":{"id":01}}',                            # leading zero: invalid JSON
    '{"maxValues":{"id":NaN}}',
    '{"maxValues":{"\\u0069d":30000000}}',                # escaped key = "id"
    '{"max\\u0056alues":{"id":30000000}}',
    '{"maxValues":{"id":30000000,"s":"a\\"b\\\\c\\u00e9\\n"}}',
    '{"maxValues":{"id":30000000,"s":"tab\there"}}',      # raw control character: invalid
    '{"maxValues":{"id":30000000,"n":[{"a":{}},[],true,false,null,-1.5e-3]}}',
    '{"maxValues":{"id":30000000}}\x00',
    '{ "maxValues" : { "id" : 30000001 } , "minValues" : { "id" : -4 } }',
    '{"maxValues":{"id":1e400}}',
    '{"maxValues":{"id":-}}',
    '{"maxValues":{"id":1.}}',
    '{"maxValues":{"id":.5}}',
    '{"maxValues":{"id":tru}}',
    '{"maxValues":{"id":true}}',
    '{"maxValues":{"id":{}}}',
    '{"maxValues":{"ID":30000000}}',
    '{"maxValues":{"id":30000000},}',
]

SHORT_EDGE = ['{"maxValues":{"s":5.0}}', '{"maxValues":{"s":5E0}}', '{"maxValues":{"s":50E-1}}',
              '{"maxValues":{"s":5.5}}', '{"maxValues":{"s":32767}}', '{"maxValues":{"s":32768}}',
              '{"maxValues":{"s":3.2768E4}}', '{"maxValues":{"s":-32768.000}}', '{"maxValues":{"s":0E-5000}}',
              '{"maxValues":{"s":0.00000}}', '{"maxValues":{"s":-0.0}}', '{"maxValues":{"s":1E5}}',
              '{"maxValues":{"s":1e-1}}', '{"maxValues":{"s":12.30E1}}', '{"maxValues":{"s":123.0E-1}}',
              '{"maxValues":{"s":0.0123E3}}', '{"maxValues":{"s":0.0120E3}}']


def _column(strings):
    """An oracle string column (row_def 2 = present, 0 = null stats) over `strings` (None = null)."""
    enc = [b"" if s is None else s.encode("utf-8", "surrogatepass") for s in strings]
    offs = np.zeros(len(enc) + 1, np.int64)
    offs[1:] = np.cumsum([len(e) for e in enc])
    return ref.Column(path="add.stats", phys=6, max_def=2, max_rep=0, rep_def=0, n_rows=len(enc),
                      row_def=np.array([0 if s is None else 2 for s in strings], np.uint8),
                      offs=offs, chars=np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy())


def _python(strings, node, types):
    out = []
    for s in strings:
        try:
            out.append(sk.keep(s, node, types))
        except sk.StatsDecodeError:
            out.append("error")
    return out


def _fast(strings, node, types):
    col = _column(strings)
    out = []
    for i in range(len(strings)):     # one row at a time so that decode errors are per row
        sel = np.zeros(len(strings), np.uint8)
        sel[i] = 1
        try:
            sk.apply_to_column(col, sel, node, types)
            out.append(bool(sel[i]))
        except sk.StatsDecodeError:
            out.append("error")
    return out


def _random_stats(rng, n):
    out = []
    for _ in range(n):
        k = rng.integers(0, 10)
        lo = int(rng.integers(-2**40, 2**40))
        hi = lo + int(rng.integers(0, 2**40))
        if k == 0:
            out.append(None)
        elif k == 1:
            out.append(json.dumps({"numRecords": 3, "minValues": {"id": lo}, "nullCount": {"id": 1}}))
        elif k == 2:
            out.append(json.dumps({"maxValues": {"id": hi, "name": "xé\"y"}, "minValues": {"id": None}}))
        else:
            out.append(json.dumps({"numRecords": int(rng.integers(1, 100)), "minValues": {"id": lo, "name": "a"},
                                   "maxValues": {"id": hi, "name": "z"}, "nullCount": {"id": 0, "name": 2}},
                                  indent=None if k < 8 else 1))
    return out


def _gt(path, v, t="long"):
    return (">", ("stat", path), ("lit", v, t))


PREDICATES = [
    (_gt(MAX_ID, 25_000_000), {MAX_ID: "long"}),
    (("<=", ("stat", MIN_ID), ("lit", 0, "long")), {MIN_ID: "long"}),
    (("AND", _gt(MAX_ID, -5), ("<", ("stat", MIN_ID), ("lit", 2**39, "long"))), {MAX_ID: "long", MIN_ID: "long"}),
    (("OR", ("=", ("stat", NULLS), ("lit", 0, "long")), ("<", ("stat", MIN_ID), ("lit", 7, "long"))),
     {NULLS: "long", MIN_ID: "long"}),
    ((">=", ("stat", MAX_ID), ("lit", 30000001, "integer")), {MAX_ID: "integer"}),
]


@pytest.mark.parametrize("pi", range(len(PREDICATES)))
def test_fast_path_equals_python(pi):
    node, types = PREDICATES[pi]
    assert sk.compile_integral(node, types) is not None
    rows = EDGE + _random_stats(np.random.default_rng(pi), 400)
    assert _fast(rows, node, types) == _python(rows, node, types)


def test_fast_path_short_decimals():
    path = ("maxValues", "s")
    for t, lit in (("short", 5), ("byte", 5), ("short", 32767), ("short", 12)):
        node, types = (">=", ("stat", path), ("lit", lit, t)), {path: t}
        assert _fast(SHORT_EDGE, node, types) == _python(SHORT_EDGE, node, types), (t, lit)


def test_fast_path_refuses_other_types():
    assert sk.compile_integral(_gt(("maxValues", "d"), 1), {("maxValues", "d"): "date"}) is None
    assert sk.compile_integral(("<", ("timeadd", ("stat", MAX_ID)), ("lit", 1, "long")), {MAX_ID: "long"}) is None
    assert sk.compile_integral(_gt(MAX_ID, 1.5), {MAX_ID: "long"}) is None


def test_fast_path_decides_clean_rows():
    """The fast path must actually decide the common rows (no deferral to Python)."""
    node, types = PREDICATES[0]
    rows = _random_stats(np.random.default_rng(7), 1000)
    col = _column(rows)
    sel = np.ones(len(rows), np.uint8)
    blob, n, ops = sk.compile_integral(node, types)
    defer = np.zeros(len(rows), np.uint8)
    import ctypes as C
    P = C.c_void_p
    nd = ref.lib().dkr_skip_eval(P(col.chars.ctypes.data), P(col.offs.ctypes.data), P(col.row_def.ctypes.data), 2,
                                 P(sel.ctypes.data), P(defer.ctypes.data), len(rows), blob, len(blob), n,
                                 P(ops.ctypes.data), len(ops) // 2)
    assert nd == 0
    assert [bool(x) for x in sel] == _python(rows, node, types)


def test_pooled_replay_with_row_group_tasks_equals_sequential(tmp_path):
    """ref.replay over a thread pool with row-group-run tasks and early data skipping gives the
    sequential replay's counters, tail rows and selection bits."""
    from delta_amd import synth
    root = str(tmp_path / "t")
    synth.write_table(root, synth.TableSpec(n_adds=60_000, n_parts=3, row_group_size=7_000, with_stats=True,
                                            dv_frac=0.2, n_commits=6, adds_per_commit=40, removes_per_commit=40))
    node, types = PREDICATES[2]
    a = ref.replay(root, with_stats=True, skipping=(node, types))
    b = ref.replay(root, with_stats=True, threads=5, keep_cols=False, skipping=(node, types))
    assert b.pool_tasks > 3
    assert a.counters.as_tuple() == b.counters.as_tuple()
    assert [r["path"] for r in a.json_rows] == [r["path"] for r in b.json_rows]
    assert [x.path for x in a.checkpoint] == [x.path for x in b.checkpoint]
    for x, y in zip(a.checkpoint, b.checkpoint):
        assert x.n_rows == y.n_rows and np.array_equal(x.selected, y.selected)
    assert 0 < sum(int(x.selected.sum()) for x in a.checkpoint) < 60_000
