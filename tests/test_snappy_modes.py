"""The snappy decoder's three paths give the same bytes (the wave-cooperative
fragment-boundary walk of k_snap_fix was only checked end to end).

  default       hybrid: speculative walk + link, k_snap_fix verifies entries, rewrites the tag-start
                bitmap and walks it to every 64 KiB fragment start; k_snap_frag decodes fragments
  DK_SNAPPY_MODE=frag  fragments without the bitmap (k_snap_fix walks to the fragment starts tag by tag)
  DK_SNAPPY_MODE=page  one wave decodes a whole page in order (no fragments)

Pages are crafted to stress the walk: long incompressible literals that cross many 2 KiB segments,
dense 2-byte / overlapping copies (runs of one or two characters), mixtures of the two, and pages of
several 64 KiB fragments (1 MiB page size, PLAIN values). Each mode runs in its own process (the mode
is read once per process); every column must equal pyarrow's decode of the same file.
"""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _strings(kind, n, rng):
    out = []
    for i in range(n):
        if kind == "literal":          # incompressible: long literals across segments
            k = int(rng.integers(200, 4000))
            out.append(rng.integers(33, 127, size=k, dtype=np.uint8).tobytes().decode())
        elif kind == "runs":           # dense short copies: offset 1 / 2 runs of every length
            k = int(rng.integers(1, 3000))
            unit = "a" if i % 3 == 0 else "ab" if i % 3 == 1 else "xyz"
            out.append((unit * (k // len(unit) + 1))[:k])
        else:                          # mixed: path-like with repeated prefixes and random tails
            tail = rng.integers(48, 58, size=int(rng.integers(1, 40)), dtype=np.uint8).tobytes().decode()
            lit = rng.integers(97, 123, size=int(rng.integers(0, 300)), dtype=np.uint8).tobytes().decode()
            out.append("date=2024-01-%02d/part-%05d-%s-c000.snappy.parquet%s%s" % (i % 28 + 1, i, tail, lit, "z" * (i % 50)))
    return out


def _write(path, seed):
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(seed)
    t = pa.table({k: pa.array(_strings(k, 3000, rng)) for k in ("literal", "runs", "mixed")})
    pq.write_table(t, path, compression="snappy", use_dictionary=False, data_page_size=1 << 20,
                   row_group_size=1500, write_statistics=False)
    return t


def _digest_expected(t):
    out = {}
    for name in t.column_names:
        h = hashlib.sha256()
        for v in t.column(name).to_pylist():
            b = v.encode()
            h.update(len(b).to_bytes(4, "little"))
            h.update(b)
        out[name] = h.hexdigest()
    return out


def _digest_product(path):
    """Run in a child process: decode the file on the GPU, digest every string column."""
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    leaves = ["literal", "runs", "mixed"]
    ps = K.ParquetSet(eng, [path], leaves).decode()
    out = {}
    for leaf in leaves:
        c = ps.column(0, leaf)
        h = hashlib.sha256()
        for i in range(c.n_rows):
            b = bytes(c.chars[c.offs[i]:c.offs[i + 1]])
            h.update(len(b).to_bytes(4, "little"))
            h.update(b)
        out[leaf] = h.hexdigest()
    ps.close()
    eng.close()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"DK_SNAPPY_MODE": "frag"}, {"DK_SNAPPY_MODE": "page"}],
                         ids=["hybrid-bitmap", "frag-no-bitmap", "page"])
def test_gpu_snappy_modes_equal_pyarrow(tmp_path, env):
    path = str(tmp_path / "s.parquet")
    want = _digest_expected(_write(path, 31))
    code = ("import sys, json; sys.path.insert(0, %r); from tests.test_snappy_modes import _digest_product; "
            "print(json.dumps(_digest_product(%r)))" % (ROOT, path))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got == want


def test_crafted_pages_span_fragments(tmp_path):
    """(CPU) the crafted file really has multi-fragment snappy pages: some page's uncompressed
    size exceeds 64 KiB several times over."""
    import pyarrow.parquet as pq
    path = str(tmp_path / "s.parquet")
    _write(path, 31)
    md = pq.ParquetFile(path).metadata
    biggest = max(md.row_group(g).column(c).total_uncompressed_size
                  for g in range(md.num_row_groups) for c in range(md.num_columns))
    assert biggest > 4 * 65536
