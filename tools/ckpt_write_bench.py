"""Time Table.checkpoint with the GPU encoder on a C3-shaped table and check the file it writes:
pyarrow reads it back (row count, schema), and getScanFiles over the new checkpoint gives the scan
files and counters the old one gave. Usage: python tools/ckpt_write_bench.py ROWS PARTS [--host]"""
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import pyarrow.parquet as pq
    from delta_amd import kernel as K
    from delta_amd import synth
    rows, parts = int(sys.argv[1]), int(sys.argv[2])
    encoder = "gpu"
    d = "/tmp/dk_ckw_%d_%d" % (rows, parts)
    shutil.rmtree(d, ignore_errors=True)
    spec = synth.TableSpec(n_adds=rows, n_parts=parts, compression="snappy", n_commits=100, adds_per_commit=100,
                           removes_per_commit=100, readd_frac=0.1, dup_frac=0.05, seed=20250218,
                           extra={"protocol": {"minWriterVersion": 2, "minReaderVersion": 1, "readerFeatures": None,
                                               "writerFeatures": None}})
    synth.write_table(d, spec)
    eng = K.GpuEngine()

    def scan_summary():
        snap = K.Table.forPath(eng, d).getLatestSnapshot(eng)
        sc = snap.getScanBuilder().build()
        n, size = 0, 0
        for b in sc.getScanFiles(eng):
            v = b.data["add.size"].fixed.view("<i8")
            sel = np.ones(b.size, bool) if b.selection is None else b.selection
            n += int(np.count_nonzero(sel))
            size += int(v.sum(where=sel))
        m = sc.metrics.as_tuple()
        sc.close()
        return n, size, m

    before = scan_summary()
    t0 = time.perf_counter()
    v, n_adds = K.Table.forPath(eng, d).checkpoint(eng, now_ms=1_700_000_000_000 + 10**12)
    dt = time.perf_counter() - t0
    path = os.path.join(d, "_delta_log", "%020d.checkpoint.parquet" % v)
    pf = pq.ParquetFile(path)
    after = scan_summary()
    res = {"encoder": encoder, "rows": rows, "version": v, "adds_written": n_adds, "write_s": dt,
           "file_bytes": os.path.getsize(path), "row_groups": pf.metadata.num_row_groups,
           "file_rows": pf.metadata.num_rows, "pyarrow_rows_read": pq.read_table(path, columns=["add"]).num_rows,
           "selected_before": before[0], "selected_after": after[0], "size_sum_equal": before[1] == after[1],
           "counters_after": list(after[2]), "adds_equal_selected": n_adds == before[0],
           "scan_files_equal": before[:2] == after[:2]}
    print(json.dumps(res), flush=True)
    eng.close()
    shutil.rmtree(d, ignore_errors=True)
    return 0 if res["scan_files_equal"] and res["adds_equal_selected"] else 1


if __name__ == "__main__":
    sys.exit(main())
