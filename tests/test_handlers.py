"""Engine plugin point 1 beyond the ParquetHandler (delta_amd/handlers.py over
dk_json_parse_stats / dk_parsed_stats_eval): JsonHandler.parseJson of stats strings and the
data-skipping PredicateEvaluator, as a stock ScanImpl.applyDataSkipping calls them
(kernel-api/.../internal/ScanImpl.java:304-352), on the GPU.

Each case is one of test_skipping.py's stats edge sets (integral / date / string / timestamp /
decimal / float stats, escapes, duplicates, nulls) with its predicates. The oracle answers per row:
unselected -> not selected; null stats -> kept; else oracle/skipping.keep with the oracle's own
skipping predicate (oracle/skipping_filter.py). Parsed integral / date values are compared with the
oracle's decode_stats. Decode errors fail the parse."""
import json

import numpy as np
import pytest

from delta_amd import skipping as sk
from tests import test_skipping as T


def _schema(columns):
    return json.dumps({"type": "struct", "fields": [{"name": n, "type": t, "nullable": True, "metadata": {}}
                                                    for n, t in columns]})


def _plans(columns, predicate):
    """(product program, oracle node, oracle types) for predicate over a table of `columns`."""
    from oracle import skipping_filter as osf
    schema = _schema(columns)
    leaves = sk.data_schema_leaves(schema, [])
    node = sk.construct(predicate, leaves)
    if node is None:
        return None
    sk.check_types(node, leaves)
    prog = sk.compile_program(node, leaves)
    S = osf.StatsSchema(schema, [])
    onode = osf.build(predicate, S)
    osf.check(onode, S)
    return prog, onode, osf.stat_types(onode, S)


CASES = [
    ((("x", "short"), ("id", "long")), T.EDGE_STATS, T.EDGE_PREDICATES),
    (T.DATE_COLUMNS, T.DATE_EDGE_STATS, T.DATE_PREDICATES),
    (T.STRING_COLUMNS, T.STRING_EDGE_STATS, T.STRING_PREDICATES),
    (T.TS_COLUMNS, T.TS_EDGE_STATS, T.TS_EDGE_PREDICATES),
    (T.DEC_COLUMNS, T.DEC_EDGE_STATS, T.DEC_PREDICATES),
    (T.FP_COLUMNS, T.FP_EDGE_STATS, T.FP_EDGE_PREDICATES),
]


def test_plans_build():
    """Both planners accept every case's predicates (CPU)."""
    for columns, _, preds in CASES:
        for p in preds:
            assert _plans(columns, p) is not None, p


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_gpu_parse_json_and_predicate_evaluator(ci):
    from delta_amd import kernel as K
    from delta_amd.handlers import GpuJsonHandler, GpuPredicateEvaluator
    from oracle import skipping as osk
    columns, stats, preds = CASES[ci]
    eng = K.GpuEngine()
    rng = np.random.default_rng(ci)
    rows = list(stats) * 3
    for p in preds:
        prog, onode, otypes = _plans(columns, p)
        for trial in range(2):
            sel = np.ones(len(rows), bool) if trial == 0 else rng.random(len(rows)) < 0.6
            parsed = GpuJsonHandler(eng).parseJson(rows, prog, sel)
            got = GpuPredicateEvaluator(eng, prog).eval(parsed, sel)
            want = [bool(s) and osk.keep(st, onode, otypes) for st, s in zip(rows, sel)]
            assert list(got) == want, (p, trial)
            # parsed integral / date / timestamp values equal the oracle's decoded stats
            paths, types = prog[0], prog[1]
            for pi, (path, t) in enumerate(zip(paths, types)):
                if t not in (0, 1, 2, 3, 4, 6, 8):
                    continue
                vals, pres = parsed.column(pi)
                for r, st in enumerate(rows):
                    if not sel[r] or st is None:
                        assert not pres[r]
                        continue
                    want_v = osk.decode_stats(st, {path: otypes.get(path, "long")}).get(path) \
                        if path in otypes else None
                    if path in otypes:
                        assert (want_v is None and not pres[r]) or (pres[r] and vals[r] == want_v), (path, r, st)
            parsed.close()
    eng.close()


@pytest.mark.gpu
def test_gpu_parse_json_decode_errors():
    """A stats string the reference cannot decode fails parseJson (DefaultJsonHandler throws)."""
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    from delta_amd.handlers import GpuJsonHandler
    eng = K.GpuEngine()
    prog = _plans((("x", "short"), ("id", "long")), T.BAD_PREDICATE)[0]
    for bad in T.BAD_STATS:
        with pytest.raises(DkError, match="Parsing the JSON statistics"):
            GpuJsonHandler(eng).parseJson([T.EDGE_STATS[0], bad], prog)
        # an unselected bad row is never parsed
        GpuJsonHandler(eng).parseJson([T.EDGE_STATS[0], bad], prog, np.array([True, False])).close()
    eng.close()
