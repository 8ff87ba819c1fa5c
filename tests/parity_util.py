"""Shared helpers for parity tests: run the product (libdkgpu via delta_amd.kernel) and the oracle
on the same table and reduce both to ordered canonical scan-file rows + ScanMetrics counters."""
import numpy as np

from delta_amd import kernel as K
from oracle import ref


def product_scan(table_root, json_batch_size=1024, with_stats=False, engine=None):
    eng = engine or K.GpuEngine(json_batch_size=json_batch_size)
    snap = K.Table.forPath(eng, table_root).getLatestSnapshot(eng)
    scan = snap.getScanBuilder().withStats(with_stats).build()
    rows = []
    for b in scan.getScanFiles(eng):
        for r in b.selected_rows():
            rows.append(ref.canon_add_from_cols(b.data, int(r)) + (b.table_root,))
    out = (snap.getVersion(), rows, scan.metrics.as_tuple())
    scan.close()
    return out


def oracle_scan(table_root, json_batch_size=1024, with_stats=False):
    r = ref.replay(table_root, json_batch_size=json_batch_size, with_stats=with_stats)
    return r.version, r.scan_files(), r.counters.as_tuple()


def assert_same(p, o):
    assert p[0] == o[0], ("version", p[0], o[0])
    assert p[2] == o[2], ("counters", p[2], o[2])
    assert len(p[1]) == len(o[1]), ("n scan files", len(p[1]), len(o[1]))
    for i, (a, b) in enumerate(zip(p[1], o[1])):
        assert a == b, ("row", i, a, b)
