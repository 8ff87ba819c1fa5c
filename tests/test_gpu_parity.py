"""GPU parity: libdkgpu's scan files + ScanMetrics vs the CPU oracle, bit-exact, on seeded synthetic
tables across encodings / page versions / batch sizes."""
import pytest

from delta_amd import synth
from tests.parity_util import assert_same, oracle_scan, product_scan

pytestmark = pytest.mark.gpu

CASES = {
    "dict-v1": dict(),
    "plain-v1": dict(use_dictionary=False),
    "dict-v2": dict(data_page_version="2.0"),
    "plain-v2-smallpages": dict(use_dictionary=False, data_page_version="2.0", max_rows_per_page=997),
    "pv2-dv-removes": dict(pv_keys=2, dv_frac=0.3, ckpt_removes=300),
    "variable-paths": dict(variable_paths=True, dv_frac=0.2),
    "no-page-index": dict(write_page_index=False, max_rows_per_page=3000),
    "multi-rowgroup": dict(row_group_size=7000, max_rows_per_page=2500),
    "snappy-v1": dict(compression="snappy", pv_keys=2, dv_frac=0.1),
    "snappy-v2-plain": dict(compression="snappy", data_page_version="2.0", use_dictionary=False),
    "snappy-stats-variable": dict(compression="snappy", variable_paths=True, with_stats=True),
    "delta-binary-packed-v1": dict(delta_binary_packed=True, max_rows_per_page=4099),
    "delta-binary-packed-v2-snappy": dict(delta_binary_packed=True, data_page_version="2.0", compression="snappy"),
}


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("jbs", [1024, 3])
def test_scan_parity(tmp_path, name, jbs):
    spec = synth.TableSpec(n_adds=20_000, n_commits=12, adds_per_commit=40, removes_per_commit=40,
                           seed=synth.SEED + hash(name) % 1000, **CASES[name])
    synth.write_table(str(tmp_path), spec)
    assert_same(product_scan(str(tmp_path), jbs), oracle_scan(str(tmp_path), jbs))


@pytest.mark.parametrize("jbs", [1024, 7])
def test_large_tail_parity(tmp_path, jbs):
    """A commit tail of ~28k rows: the replay's action table is built in parallel over row blocks
    (dk_replay_create), and the tail's columns are concatenated from the per-commit parses."""
    spec = synth.TableSpec(n_adds=20_000, n_commits=40, adds_per_commit=400, removes_per_commit=300,
                           pv_keys=2, dv_frac=0.2, seed=synth.SEED + 31)
    synth.write_table(str(tmp_path), spec)
    assert_same(product_scan(str(tmp_path), jbs), oracle_scan(str(tmp_path), jbs))


def test_large_json_manifest_parity(tmp_path):
    """V2 JSON manifest with 9000 add rows after the commits: checkpoint adds inside the tail, across
    several of the replay's build blocks."""
    spec = synth.TableSpec(n_adds=30_000, n_commits=10, n_parts=2, v2_sidecars=2, v2_manifest="json",
                           v2_json_adds=9000, seed=synth.SEED + 32)
    synth.write_table(str(tmp_path), spec)
    assert_same(product_scan(str(tmp_path), 1024), oracle_scan(str(tmp_path), 1024))


def test_multipart_parity(tmp_path):
    spec = synth.TableSpec(n_adds=30_000, n_parts=4, n_commits=8, dv_frac=0.1)
    synth.write_table(str(tmp_path), spec)
    assert_same(product_scan(str(tmp_path)), oracle_scan(str(tmp_path)))


def test_with_stats_parity(tmp_path):
    spec = synth.TableSpec(n_adds=8_000, n_commits=5, with_stats=True)
    synth.write_table(str(tmp_path), spec)
    assert_same(product_scan(str(tmp_path), with_stats=True), oracle_scan(str(tmp_path), with_stats=True))


V2_CASES = {
    # C5 shape: V2 manifest + sidecars, snappy, v2 pages, DELTA_BINARY_PACKED, hot partition
    "v2-sidecars-c5": dict(n_parts=6, v2_sidecars=6, compression="snappy", data_page_version="2.0",
                           delta_binary_packed=True, hot_frac=0.6, ckpt_removes=200, dv_frac=0.1),
    "v2-one-sidecar-dict": dict(n_parts=1, v2_sidecars=1, pv_keys=2),
    # V2 JSON manifest carrying add rows (checkpoint adds read by the JSON handler before the
    # sidecars, ActionsIterator.java:213-248) and remove rows (ignored); the tail removes / re-adds some
    "v2-json-manifest-adds": dict(n_parts=3, v2_sidecars=3, v2_manifest="json", v2_json_adds=400, with_stats=True),
}


@pytest.mark.parametrize("name", list(V2_CASES))
@pytest.mark.parametrize("jbs", [1024, 5])
def test_v2_sidecar_parity(tmp_path, name, jbs):
    spec = synth.TableSpec(n_adds=30_000, n_commits=8, seed=synth.SEED + 7, **V2_CASES[name])
    synth.write_table(str(tmp_path), spec)
    assert_same(product_scan(str(tmp_path), jbs), oracle_scan(str(tmp_path), jbs))


@pytest.mark.parametrize("name", ["snappy-v1", "dict-v2", "delta-binary-packed-v2-snappy", "pv2-dv-removes"])
def test_repeated_runs_equal(tmp_path, name):
    """The first run after prepare reuses the prepare pass's stages (headers, snappy, runs, counts,
    positions); every later run decodes from scratch. Both must give the oracle's answer."""
    from delta_amd import kernel as K
    from oracle import ref
    spec = synth.TableSpec(n_adds=20_000, n_commits=6, adds_per_commit=40, removes_per_commit=40,
                           seed=synth.SEED + 11, **CASES[name])
    synth.write_table(str(tmp_path), spec)
    eng = K.GpuEngine()
    snap = K.Table.forPath(eng, str(tmp_path)).getLatestSnapshot(eng)
    scan = snap.getScanBuilder().build()
    runs = []
    for i in range(3):
        it = scan.getScanFiles(eng) if i == 0 else (scan.run(), scan.sync(), scan._batches())[2]
        rows = [ref.canon_add_from_cols(b.data, int(r)) + (b.table_root,) for b in it for r in b.selected_rows()]
        runs.append((rows, scan.metrics.as_tuple()))
    scan.close()
    o = oracle_scan(str(tmp_path))
    for rows, counters in runs:
        assert counters == o[2]
        assert rows == o[1]
