"""Back-reference distance profile of the snappy pages of a checkpoint (CPU, no GPU): for every
column chunk, the share of copy tags / copied bytes whose offset falls in each distance bucket.
Sizes k_snap_frag's LDS ring.

    python tools/snap_offsets.py CHECKPOINT.parquet [--leaf add.path]
"""
import argparse
import collections

import pyarrow.parquet as pq


def varint(b, i):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7f) << s
        s += 7
        if c < 0x80:
            return r, i


def zz(v):
    return (v >> 1) ^ -(v & 1)


def skip(b, i, t):
    if t in (1, 2):
        return i
    if t == 3:
        return i + 1
    if t in (4, 5, 6):
        return varint(b, i)[1]
    if t == 7:
        return i + 8
    if t == 8:
        n, i = varint(b, i)
        return i + n
    if t in (9, 10):
        h = b[i]
        i += 1
        n, et = h >> 4, h & 15
        if n == 15:
            n, i = varint(b, i)
        for _ in range(n):
            i = skip(b, i, et)
        return i
    if t == 12:
        return struct_fields(b, i, None)[1]
    raise ValueError("thrift type %d" % t)


def struct_fields(b, i, want):
    """Top-level i32 fields of a compact struct (ids in `want`); returns (dict, end)."""
    out, fid = {}, 0
    while True:
        h = b[i]
        i += 1
        if h == 0:
            return out, i
        t, d = h & 15, h >> 4
        if d:
            fid += d
        else:
            v, i = varint(b, i)
            fid = zz(v)
        if want is not None and fid in want and t == 5:
            v, i = varint(b, i)
            out[fid] = zz(v)
        else:
            i = skip(b, i, t)


def snappy_tags(buf):
    _, i = varint(buf, 0)
    o = 0
    while i < len(buf):
        tag = buf[i]
        k = tag & 3
        if k == 0:
            ln = (tag >> 2) + 1
            i += 1
            if ln > 60:
                nb = ln - 60
                ln = int.from_bytes(buf[i:i + nb], "little") + 1
                i += nb
            yield 0, ln, 0
            i += ln
        elif k == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | buf[i + 1]
            i += 2
            yield 1, ln, off
        elif k == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[i + 1:i + 3], "little")
            i += 3
            yield 1, ln, off
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[i + 1:i + 5], "little")
            i += 5
            yield 1, ln, off
        o += ln


BUCKETS = [64, 256, 1024, 2048, 4096, 8192, 16384, 32768, 65536, 1 << 40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--leaf", default=None)
    a = ap.parse_args()
    data = open(a.path, "rb").read()
    md = pq.ParquetFile(a.path).metadata
    tot = collections.Counter()
    for rg in range(md.num_row_groups):
        for c in range(md.num_columns):
            cc = md.row_group(rg).column(c)
            if cc.compression != "SNAPPY" or (a.leaf and cc.path_in_schema != a.leaf):
                continue
            start = cc.dictionary_page_offset or cc.data_page_offset
            i, end = start, start + cc.total_compressed_size
            while i < end:
                h, j = struct_fields(data, i, {1, 2, 3})
                body = data[j:j + h[3]]
                i = j + h[3]
                if h[1] == 3:   # DATA_PAGE_V2: levels stored uncompressed before the snappy block
                    continue
                for kind, ln, off in snappy_tags(body):
                    if kind == 0:
                        tot["lit_tags"] += 1
                        tot["lit_bytes"] += ln
                    else:
                        bkt = next(x for x in BUCKETS if off <= x)
                        tot["cp_tags", bkt] += 1
                        tot["cp_bytes", bkt] += ln
                        tot["cp_tags"] += 1
                        tot["cp_bytes"] += ln
    out = tot["lit_bytes"] + tot["cp_bytes"]
    print("output %d B: literal %.3f, copy %.3f; tags: %d literal, %d copy"
          % (out, tot["lit_bytes"] / out, tot["cp_bytes"] / out, tot["lit_tags"], tot["cp_tags"]))
    acc_t = acc_b = 0
    for x in BUCKETS:
        acc_t += tot["cp_tags", x]
        acc_b += tot["cp_bytes", x]
        print("offset <= %-8s copy tags %.4f (cum %.4f)  copy bytes %.4f (cum %.4f)"
              % (x if x < 1 << 40 else "inf", tot["cp_tags", x] / max(1, tot["cp_tags"]), acc_t / max(1, tot["cp_tags"]),
                 tot["cp_bytes", x] / max(1, tot["cp_bytes"]), acc_b / max(1, tot["cp_bytes"])))


if __name__ == "__main__":
    main()
