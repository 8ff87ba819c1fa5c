"""Debug: the rows where the GPU's typed stats_parsed skipping and the oracle disagree for the
typed-stats fixture's predicates (tests/test_skipping.py::typed_predicates)."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from delta_amd import synth  # noqa: E402
from tests import test_skipping as T  # noqa: E402


def main():
    from delta_amd import kernel as K
    import pyarrow.parquet as pq
    root = os.path.join(tempfile.mkdtemp(), "t")
    unit = sys.argv[1] if len(sys.argv) > 1 else "us"
    mins = synth.write_typed_stats_table(root, n=3000, seed=11, ts_unit=unit)
    t = pq.read_table(os.path.join(root, "_delta_log", "%020d.checkpoint.parquet" % 0)).column("add").to_pylist()
    byp = {r["path"]: r for r in t if r}
    eng = K.GpuEngine()
    for p in T.typed_predicates(mins, unit):
        g = T._gpu_files_parsed(root, p, eng)
        o = T.oracle_files(root, p)
        gs, os_ = {r[0].decode() for r in g[0]}, {r[0].decode() for r in o[0]}
        if gs != os_:
            print("PRED", p)
            for path in sorted(gs ^ os_)[:6]:
                r = byp.get(path)
                print("  ", path, "gpu" if path in gs else "oracle", "kept")
                if r:
                    print("     json:", r["stats"])
                    print("     typed:", r["stats_parsed"])
    eng.close()
    print("done")


if __name__ == "__main__":
    main()
