"""Debug: localize the typed stats_parsed / oracle disagreement (run with and without
DK_NO_STATS_PARSED=1)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from delta_amd import synth  # noqa: E402
from delta_amd.expressions import And, Literal, Or  # noqa: E402
from tests import test_skipping as T  # noqa: E402


def main():
    from delta_amd import kernel as K
    root = os.path.join(tempfile.mkdtemp(), "t")
    synth.write_typed_stats_table(root, n=3000, seed=11, ts_unit="us")
    eng = K.GpuEngine()
    c, col = T.cmp, T.col
    preds = {
        "and_s_ts": And(c(">=", col("s"), Literal.ofString("x")), c("<", col("ts"), Literal.ofTimestamp(0))),
        "ts_lt0": c("<", col("ts"), Literal.ofTimestamp(0)),
        "s_ge_x": c(">=", col("s"), Literal.ofString("x")),
        "and_ts_s": And(c("<", col("ts"), Literal.ofTimestamp(0)), c(">=", col("s"), Literal.ofString("x"))),
        "and_s_l": And(c(">=", col("s"), Literal.ofString("x")), c("<", col("l"), Literal.ofLong(-10 ** 15))),
        "and_l_ts": And(c(">", col("l"), Literal.ofLong(10 ** 15)), c("<", col("ts"), Literal.ofTimestamp(0))),
        "or_s_ts": Or(c(">=", col("s"), Literal.ofString("x")), c("<", col("ts"), Literal.ofTimestamp(0))),
    }
    for name, p in preds.items():
        g = T._gpu_files_parsed(root, p, eng)
        o = T.oracle_files(root, p)
        gs, os_ = {r[0].decode() for r in g[0]}, {r[0].decode() for r in o[0]}
        print(name, "parsed_files=%d" % g[2], "gpu=%d oracle=%d gpu_only=%s oracle_only=%s" % (
            len(gs), len(os_), sorted(gs - os_)[:5], sorted(os_ - gs)[:5]))
    eng.close()


if __name__ == "__main__":
    main()
