"""Committed golden fixtures (reference golden `_delta_log`s + expected answers): the oracle must
reproduce them (CPU), and libdkgpu must reproduce them bit-exactly (GPU)."""
import os

import pytest

from tests.golden_util import TABLES, load_expected, to_json_rows

EXPECTED = load_expected()
KEYS = [(name, key) for name in sorted(EXPECTED) for key in sorted(EXPECTED[name])]


@pytest.mark.parametrize("name,key", KEYS)
def test_oracle_matches_fixture(name, key):
    from oracle import ref
    bs, stats = map(int, key.split("-"))
    r = ref.replay(os.path.join(TABLES, name), json_batch_size=bs, with_stats=bool(stats))
    exp = EXPECTED[name][key]
    assert r.version == exp["version"]
    assert list(r.counters.as_tuple()) == exp["counters"]
    assert to_json_rows(r.scan_files()) == exp["rows"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,key", KEYS)
def test_gpu_matches_fixture(name, key):
    from tests.parity_util import product_scan
    bs, stats = map(int, key.split("-"))
    v, rows, counters = product_scan(os.path.join(TABLES, name), bs, bool(stats))
    exp = EXPECTED[name][key]
    assert v == exp["version"]
    assert list(counters) == exp["counters"]
    assert to_json_rows(rows) == exp["rows"]
