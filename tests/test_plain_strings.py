"""PLAIN BYTE_ARRAY pages through the string decode (k_pos_count / scan / write: length-prefix
candidates per 16 KiB chunk with the chain verified across chunks, k_pos_fallback for pages whose
chain the candidate scan cannot follow; k_string_copy: chars + key hashes per 128-value tile) against
the oracle decoder, bit for bit.

The cases are the ones that stress the chunking: values straddling chunk boundaries, values longer
than a copy tile's staging buffer and than a whole chunk, empty strings (4-byte values; runs of them
defeat the zero-run candidate test), embedded NUL runs that look like length prefixes, a value of
2^24 bytes (its length prefix has no zero high byte), nulls in between, v1 / v2 pages, snappy and
uncompressed. Reference: DefaultBinaryVector / parquet-mr's PLAIN BinaryColumnReader.
"""
import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from oracle import ref


def _values(kind, rng, n):
    if kind == "paths":              # path-like, 60-140 bytes: many values per chunk, all straddling
        return ["part-%05d-%s.c000.snappy.parquet" % (i, "x" * int(rng.integers(20, 100))) for i in range(n)]
    if kind == "mixed":              # 0 B .. 40 KiB, nulls, NUL runs
        out = []
        for i in range(n):
            r = rng.random()
            if r < 0.1:
                out.append(None)
            elif r < 0.2:
                out.append("")
            elif r < 0.3:
                out.append("\x00\x00\x00" + chr(1 + i % 100) + "\x00" * int(rng.integers(1, 9)) + "q")
            elif r < 0.35:
                out.append("L" * int(rng.integers(1500, 40000)))
            else:
                out.append("v%d-" % i + "y" * int(rng.integers(0, 300)))
        return out
    if kind == "empties":            # long runs of empty strings
        return ["" if i % 50 else "e%d" % i for i in range(n)]
    raise ValueError(kind)


def _write(path, vals, compression, version, page_size):
    t = pa.table({"add": pa.StructArray.from_arrays([pa.array(vals, pa.string())], names=["path"])})
    pq.write_table(t, path, compression=compression, use_dictionary=False, data_page_version=version,
                   data_page_size=page_size, row_group_size=len(vals))


def _read(eng, paths):
    with eng.readParquetFiles(paths, ["add.path"], window_rows=0) as rd:
        return list(rd)


def _check(batches, paths):
    from tests.test_reader import _assert_leaf, _concat
    by_file = {}
    for b in batches:
        by_file.setdefault(b.file, []).append(b)
    for fi, p in enumerate(paths):
        want = ref.ParquetFile.open(p).read("add.path")
        _assert_leaf(_concat(by_file[fi], "add.path"), want, "add.path")


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,compression,version,page_size", [
    ("paths", 60_000, "snappy", "1.0", 1 << 20),
    ("paths", 60_000, "none", "2.0", 300_000),
    ("mixed", 3_000, "snappy", "2.0", 1 << 20),
    ("mixed", 3_000, "none", "1.0", 64 << 10),
    ("empties", 50_000, "snappy", "1.0", 1 << 20),
])
def test_plain_strings_match_oracle(tmp_path, kind, n, compression, version, page_size):
    from delta_amd import kernel as K
    rng = np.random.default_rng(hash(kind) & 0xffff)
    paths = []
    for k in range(2):
        p = str(tmp_path / ("f%d.parquet" % k))
        _write(p, _values(kind, rng, n), compression, version, page_size)
        paths.append(p)
    eng = K.GpuEngine(parquet_batch_size=4096)
    _check(_read(eng, paths), paths)
    eng.close()


@pytest.mark.gpu
def test_plain_string_of_16_mib(tmp_path):
    """A 2^24-byte value: its length prefix 00 00 00 01 has no zero high byte, so the page takes the
    fallback walk; the values around it must still land in place."""
    from delta_amd import kernel as K
    vals = ["a%d" % i for i in range(100)] + ["Z" * (1 << 24)] + ["b%d" % i for i in range(100)]
    p = str(tmp_path / "big.parquet")
    _write(p, vals, "none", "1.0", 1 << 20)
    eng = K.GpuEngine(parquet_batch_size=4096)
    _check(_read(eng, [p]), [p])
    eng.close()
