"""Deletion-vector load for data reads (dk_dv_*; Scan.transformPhysicalData, Scan.java:147-230).

Known answers: DeletionVectorSuite.scala:26-58 over the reference's own DV tables (copied as data
fixtures into tests/golden/dv/: kernel-defaults test resources basic-dv-no-checkpoint and
basic-dv-with-checkpoint, golden table dv-partitioned-with-checkpoint). The oracle (oracle/dv.py) is
pinned to those answers on the CPU; the GPU bitmaps must equal the oracle's bit for bit, and the
product's end-to-end read (scan files -> data files with row index -> DV selection) must give the
suite's rows. Synthetic DVs cover every roaring container kind and the reference's error paths.
"""
import os
import shutil
import struct
import zlib

import numpy as np
import pyarrow.parquet as pq
import pytest

from oracle import dv as odv
from oracle import ref

HERE = os.path.dirname(os.path.abspath(__file__))
DV = os.path.join(HERE, "golden", "dv")

EXPECTED = {
    # DeletionVectorSuite.scala:26-31, :33-38, :40-57 (partitioned: (part, col1, col2) rows)
    "basic-dv-no-checkpoint": sorted(range(2, 10)),
    "basic-dv-with-checkpoint": [x for x in range(500) if x % 11 != 0],
    "dv-partitioned-with-checkpoint": sorted((x, "foo%d" % (x % 5)) for x in range(50)
                                             if not (x % 2 == 0 and x < 30)),
}


def _s(x):
    return x.decode() if isinstance(x, bytes) else x


def _oracle_rows(name):
    """Oracle replay -> scan files; pyarrow reads each data file; oracle DV load filters rows."""
    root = os.path.join(DV, name)
    r = ref.replay(root)
    rows = []
    for t in r.scan_files():
        path, dv = _s(t[0]), t[5]
        data = pq.read_table(os.path.join(root, path))
        deleted = set()
        if dv is not None:
            deleted = odv.load("file:" + root, _s(dv[0]), _s(dv[1]), dv[2], dv[3], dv[4])
        cols = data.column_names
        for i in range(data.num_rows):
            if i in deleted:
                continue
            if "col1" in cols:
                rows.append((data.column("col1")[i].as_py(), data.column("col2")[i].as_py()))
            else:
                rows.append(data.column("id")[i].as_py())
    return sorted(rows)


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_oracle_dv_known_answers(name):
    assert _oracle_rows(name) == EXPECTED[name]


def _portable(bitmaps):
    """Serialize {high: {key: (kind, payload)}} in RoaringBitmapArray's portable format with explicit
    container kinds (kind: 'array' values, 'bitmap' values, 'run' [(start, end incl)])."""
    out = struct.pack("<iq", 1681511377, len(bitmaps))
    for high in sorted(bitmaps):
        conts = bitmaps[high]
        keys = sorted(conts)
        hasrun = any(conts[k][0] == "run" for k in keys)
        b = bytearray()
        if hasrun:
            b += struct.pack("<I", 12347 | ((len(keys) - 1) << 16))
            rb = bytearray((len(keys) + 7) // 8)
            for i, k in enumerate(keys):
                if conts[k][0] == "run":
                    rb[i // 8] |= 1 << (i % 8)
            b += rb
        else:
            b += struct.pack("<II", 12346, len(keys))
        body = []
        for k in keys:
            kind, vals = conts[k]
            if kind == "run":
                card = sum(e - s + 1 for s, e in vals)
                body.append(struct.pack("<H", len(vals)) + b"".join(struct.pack("<HH", s, e - s) for s, e in vals))
            elif kind == "bitmap":
                card = len(vals)
                words = [0] * 1024
                for v in vals:
                    words[v >> 6] |= 1 << (v & 63)
                body.append(struct.pack("<1024Q", *words))
            else:
                card = len(vals)
                body.append(struct.pack("<%dH" % len(vals), *sorted(vals)))
            b += struct.pack("<HH", k, (card - 1) & 0xFFFF)
        if not hasrun or len(keys) >= 4:
            off = len(b) + 4 * len(keys)
            for x in body:
                b += struct.pack("<I", off)
                off += len(x)
        for x in body:
            b += x
        out += struct.pack("<i", high) + bytes(b)
    return out


def _write_dv(path, payload, offset=1):
    with open(path, "wb") as f:
        f.write(b"\x01" * offset)                         # Delta's DV files start with a version byte
        f.write(struct.pack(">i", len(payload)) + payload + struct.pack(">I", zlib.crc32(payload) & 0xFFFFFFFF))
    return offset


def _uuid_z85(u16):
    """Z85 text of 16 bytes (the 'u' storage type's encoded UUID)."""
    s = ""
    for i in range(0, 16, 4):
        v, = struct.unpack(">I", u16[i:i + 4])
        enc = ""
        for _ in range(5):
            enc = odv.Z85[v % 85] + enc
            v //= 85
        s += enc
    return s


SYNTH = {
    "arrays": {0: {0: ("array", [0, 5, 63, 64, 4095]), 3: ("array", [1, 65535])}},
    "bitmap": {0: {1: ("bitmap", list(range(0, 65536, 7)))}},
    "runs": {0: {0: ("run", [(0, 0), (10, 200), (65000, 65535)]), 2: ("array", [9]), 5: ("run", [(3, 70)]),
                 6: ("bitmap", list(range(5000, 20000, 3)))}},
    "sparse-high-key": {0: {200: ("array", [12345]), 201: ("run", [(0, 65535)])}},
}


def _synth_table(tmp_path, name):
    u = bytes(range(16 * (hash(name) % 7), 16 * (hash(name) % 7) + 16))
    enc = _uuid_z85(u)
    prefix = "ab"
    d = tmp_path / prefix
    d.mkdir(exist_ok=True)
    h = u.hex()
    fname = "deletion_vector_%s-%s-%s-%s-%s.bin" % (h[:8], h[8:12], h[12:16], h[16:20], h[20:])
    payload = _portable(SYNTH[name])
    off = _write_dv(str(d / fname), payload)
    return ("u", prefix + enc, off, len(payload), 1)


@pytest.mark.parametrize("name", sorted(SYNTH))
def test_oracle_synthetic_dv(tmp_path, name):
    dv = _synth_table(tmp_path, name)
    got = odv.load("file:" + str(tmp_path), *dv)
    want = set()
    for high, conts in SYNTH[name].items():
        for k, (kind, vals) in conts.items():
            base = (high << 32) | (k << 16)
            if kind == "run":
                for s, e in vals:
                    want.update(range(base + s, base + e + 1))
            else:
                want.update(base + v for v in vals)
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SYNTH))
def test_gpu_synthetic_dv_bitmaps(tmp_path, name):
    from delta_amd import kernel as K
    dv = _synth_table(tmp_path, name)
    eng = K.GpuEngine()
    s = K.DeletionVectors(eng, "file:" + str(tmp_path), [dv, ("u", dv[1], dv[2], dv[3], 0)])
    want = odv.load("file:" + str(tmp_path), *dv)
    deleted = s.deleted(0)
    assert s.num_bits(0) == max(want) + 1
    assert set(np.nonzero(deleted)[0].tolist()) == want
    assert s.num_bits(1) == 0                      # cardinality 0: empty, never read
    rows = np.arange(0, max(want) + 100, 3, dtype=np.int64)
    np.testing.assert_array_equal(s.selection(0, rows), [int(r) not in want for r in rows])
    np.testing.assert_array_equal(s.selection(1, rows), np.ones(rows.size, bool))
    s.close()


def _product_rows(name, batch=1024):
    from delta_amd import kernel as K
    root = os.path.join(DV, name)
    eng = K.GpuEngine(parquet_batch_size=batch)
    snap = K.Table.forPath(eng, root).getLatestSnapshot(eng)
    scan = snap.getScanBuilder().build()
    rows = []
    for path, b, sel in K.read_scan_data(eng, scan, ["id"] if "col1" not in name and "partitioned" not in name
                                         else ["col1", "col2"]):
        keep = np.ones(b.n_rows, bool) if sel is None else sel
        if "id" in b.columns:
            ids = b.columns["id"].fixed.view("<i8")
            rows.extend(int(v) for v in ids[keep])
        else:
            c1 = b.columns["col1"].fixed.view("<i4")
            c2 = b.columns["col2"]
            rows.extend((int(c1[i]), c2.string(i).decode()) for i in np.nonzero(keep)[0])
    scan.close()
    return sorted(rows)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_gpu_dv_tables_known_answers(name):
    # batch size 2 as DeletionVectorSuite.scala:42-44 sets it: many batches per data file
    assert _product_rows(name, batch=2 if "partitioned" in name else 1024) == EXPECTED[name]


@pytest.mark.gpu
def test_gpu_dv_bitmaps_match_oracle():
    from delta_amd import kernel as K
    eng = K.GpuEngine()
    for name in sorted(EXPECTED):
        root = os.path.join(DV, name)
        dvs = [t[5] for t in ref.replay(root).scan_files() if t[5] is not None]
        descs = [(_s(d[0]), _s(d[1]), d[2], d[3], d[4]) for d in dvs]
        s = K.DeletionVectors(eng, "file:" + root, descs)
        for i, d in enumerate(descs):
            want = odv.load("file:" + root, *d)
            assert set(np.nonzero(s.deleted(i))[0].tolist()) == want, (name, i)
        s.close()


@pytest.mark.gpu
def test_gpu_dv_errors(tmp_path):
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    dv = _synth_table(tmp_path, "arrays")
    eng = K.GpuEngine()
    root = "file:" + str(tmp_path)
    with pytest.raises(DkError, match="DV size mismatch"):
        K.DeletionVectors(eng, root, [(dv[0], dv[1], dv[2], dv[3] - 4, 1)])
    # corrupt one payload byte: the CRC-32 no longer matches
    path = [os.path.join(dp, f) for dp, _, fs in os.walk(str(tmp_path)) for f in fs if f.endswith(".bin")][0]
    raw = bytearray(open(path, "rb").read())
    raw[10] ^= 0x40
    open(path, "wb").write(bytes(raw))
    with pytest.raises(DkError, match="DV checksum mismatch"):
        K.DeletionVectors(eng, root, [dv])
    # an inline DV fails as in the reference (isInline() compares by reference)
    with pytest.raises(DkError, match="cannot be turned into a relative path"):
        K.DeletionVectors(eng, root, [("i", "wi5b=000010000siXQKl0rr91000f55c8Xg0@@D72lkbi5=-{L", None, 40, 6)])
    # bad magic number
    bad = str(tmp_path / "ab" / "bad.bin")
    shutil.copy(path, bad)
    payload = struct.pack("<iq", 1234, 0)
    off = _write_dv(bad, payload)
    with pytest.raises(DkError, match="Unexpected RoaringBitmapArray magic number 1234"):
        K.DeletionVectors(eng, root, [("p", "file:" + bad, off, len(payload), 1)])
    with pytest.raises(odv.DvError, match="magic number 1234"):
        odv.load(root, "p", "file:" + bad, off, len(payload), 1)
