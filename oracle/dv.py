"""Oracle (test infrastructure): deletion-vector load, restated from the reference.

  DeletionVectorUtils.loadNewDvAndBitmap     kernel-api/.../internal/deletionvectors/DeletionVectorUtils.java:27-37
  DeletionVectorStoredBitmap.load / loadFromStream   DeletionVectorStoredBitmap.java:50-129
  DeletionVectorDescriptor.isInline / getAbsolutePath  internal/actions/DeletionVectorDescriptor.java:176-231
  Base85Codec.decodeBlocks / decodeUUID       deletionvectors/Base85Codec.java
  RoaringBitmapArray.readFrom / deserialize   deletionvectors/RoaringBitmapArray.java:100-229
  org.roaringbitmap:RoaringBitmap 0.9.25 (build.sbt:573; not in /root/reference): the published portable
  serialization (RoaringArray.deserialize): cookie 12346 (no run containers, then a u32 size) or
  12347 | (size - 1) << 16 (then a run-container bitmap); per container key u16, cardinality - 1 u16;
  an offset header unless (runs present and size < 4); containers: run (u16 count, (start, length - 1)
  pairs), bitmap (cardinality > 4096: 1024 little-endian u64), else array (sorted u16 values).
Pinned by DeletionVectorSuite.scala's expected rows over the reference's own DV tables
(tests/test_dv.py). Returns Python sets of deleted row indices.
"""
import struct
import zlib

Z85 = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#"


class DvError(Exception):
    pass


def z85_decode(s):
    if len(s) % 5:
        raise DvError("input should be 5 character aligned")
    out = bytearray()
    for i in range(0, len(s), 5):
        v = 0
        for ch in s[i:i + 5]:
            k = Z85.find(ch)
            if k < 0:
                raise DvError("Input is not valid Z85: " + s)
            v = v * 85 + k
        out += struct.pack(">I", v & 0xFFFFFFFF)
    return bytes(out)


def dv_path(table_root, storage_type, path_or_inline):
    """getAbsolutePath as the reference reaches it (isInline() is a reference comparison that a
    descriptor read from the log never satisfies, so "i" also lands here and fails)."""
    if storage_type == "u":
        prefix, enc = path_or_inline[:-20], path_or_inline[-20:]
        u = z85_decode(enc)[:16].hex()
        name = "deletion_vector_%s-%s-%s-%s-%s.bin" % (u[:8], u[8:12], u[12:16], u[16:20], u[20:])
        base = table_root.rstrip("/") + ("/" + prefix if prefix else "")
        return base + "/" + name
    if storage_type == "p":
        if ":" not in path_or_inline:
            raise DvError("Relative URIs are not supported for DVs")
        return path_or_inline
    raise DvError("A uri %s which cannot be turned into a relative path as found in the transaction log"
                  % path_or_inline)


def _local(p):
    if p.startswith("file://") and p[7:8] == "/":
        return p[7:]
    return p[5:] if p.startswith("file:") else p


def _roaring32(buf, at, high, out):
    cookie, = struct.unpack_from("<I", buf, at)
    at += 4
    hasrun = (cookie & 0xFFFF) == 12347
    if not hasrun and cookie != 12346:
        raise DvError("I failed to find one of the right cookies.")
    if hasrun:
        size = (cookie >> 16) + 1
    else:
        size, = struct.unpack_from("<I", buf, at)
        at += 4
    runbits = b""
    if hasrun:
        runbits = buf[at:at + (size + 7) // 8]
        at += (size + 7) // 8
    hdr = [struct.unpack_from("<HH", buf, at + 4 * k) for k in range(size)]
    at += 4 * size
    if not hasrun or size >= 4:
        at += 4 * size
    for k, (key, card1) in enumerate(hdr):
        base = (high << 32) | (key << 16)
        if hasrun and runbits[k // 8] >> (k % 8) & 1:
            nr, = struct.unpack_from("<H", buf, at)
            at += 2
            for r in range(nr):
                st, ln = struct.unpack_from("<HH", buf, at + 4 * r)
                out.update(range(base + st, base + st + ln + 1))
            at += 4 * nr
        elif card1 + 1 > 4096:
            words = struct.unpack_from("<1024Q", buf, at)
            for w, v in enumerate(words):
                while v:
                    b = v & -v
                    out.add(base + 64 * w + b.bit_length() - 1)
                    v ^= b
            at += 8192
        else:
            vals = struct.unpack_from("<%dH" % (card1 + 1), buf, at)
            out.update(base + v for v in vals)
            at += 2 * (card1 + 1)
    return at


def read_bitmap_array(buf):
    """RoaringBitmapArray.readFrom over the bitmap bytes -> set of row indices."""
    magic, = struct.unpack_from("<i", buf, 0)
    out = set()
    if magic == 1681511377:                       # portable
        n, = struct.unpack_from("<q", buf, 4)
        at = 12
        for _ in range(n):
            key, = struct.unpack_from("<i", buf, at)
            at = _roaring32(buf, at + 4, key, out)
    elif magic == 1681511376:                     # native
        n, = struct.unpack_from("<i", buf, 4)
        at = 8
        for k in range(n):
            size, = struct.unpack_from("<i", buf, at)
            _roaring32(buf, at + 4, k, out)
            at += 4 + size
    else:
        raise DvError("Unexpected RoaringBitmapArray magic number %d" % magic)
    return out


def load(table_root, storage_type, path_or_inline, offset, size_in_bytes, cardinality):
    if cardinality == 0:
        return set()
    path = dv_path(table_root, storage_type, path_or_inline)
    with open(_local(path), "rb") as f:
        f.seek(offset or 0)
        raw = f.read(size_in_bytes + 8)
    if len(raw) < size_in_bytes + 8:
        raise DvError("EOF")
    size, = struct.unpack(">i", raw[:4])
    if size != size_in_bytes:
        raise DvError("DV size mismatch")
    body = raw[4:4 + size]
    crc, = struct.unpack(">i", raw[4 + size:8 + size])
    if (zlib.crc32(body) & 0xFFFFFFFF) != (crc & 0xFFFFFFFF):
        raise DvError("DV checksum mismatch")
    return read_bitmap_array(body)
