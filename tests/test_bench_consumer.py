"""bench.py's JMH-shaped consumer sums add.size over the selected rows of every batch with
masked_sum (a packed-word scan for near-uniform masks, a blocked multiply-add for irregular ones);
it must equal the plain masked sum for every mask shape and length (the headline value's size_sum
is checked against the oracle only through the counters)."""
import importlib.util
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 63, 64, 65, 1000, 65536 + 3, 300001])
@pytest.mark.parametrize("frac", [0.0, 0.0005, 0.03, 0.5, 0.97, 0.9995, 1.0])
def test_masked_sum_equals_plain(bench, n, frac):
    rng = np.random.default_rng(n * 1000 + int(frac * 997))
    v = rng.integers(-(1 << 40), 1 << 40, n).astype("<i8")
    sel = rng.random(n) < frac
    assert bench.masked_sum(v, sel) == (int(v[sel].sum()), int(sel.sum()))


def test_masked_sum_on_views(bench):
    """Batches hand out views (slices of a pinned block): odd offsets and lengths."""
    rng = np.random.default_rng(7)
    base_v = rng.integers(0, 1 << 40, 100003).astype("<i8")
    base_s = rng.random(100003) < 0.999
    for a, b in [(0, 100003), (3, 99999), (17, 50017), (1, 2)]:
        v, sel = base_v[a:b], base_s[a:b]
        assert bench.masked_sum(v, sel) == (int(v[sel].sum()), int(sel.sum()))
