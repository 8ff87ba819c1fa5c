"""Oracle (test infrastructure): projected-column resolution of ParquetSchemaUtils.

Restates `ParquetSchemaUtils.findSubFieldType` / `getParquetFieldToTypeMap` / `pruneFields`
(kernel/kernel-defaults/src/main/java/io/delta/kernel/defaults/internal/parquet/ParquetSchemaUtils.java:
92-138, 189-205) over pyarrow's reading of the footer schema (independent of the product's Thrift
parser): a Kernel field resolves by its parquet.field.id when a sibling carries that id, then by exact
name, then by the first case-insensitive name; every struct group visited builds the id map and two
children with one id fail (IllegalStateException). Map key_value / key / value levels are structural.

Returns the leaf's dotted *file* path, which the oracle decoder (oracle/ref.py) then reads.
"""
import pyarrow as pa
import pyarrow.parquet as pq


class DuplicateFieldId(Exception):
    pass


def _fid(f):
    md = f.metadata or {}
    v = md.get(b"PARQUET:field_id")
    return int(v) if v is not None else None


def resolve(path, dotted, ids=None):
    """File leaf path for the Kernel leaf `dotted` (components with optional field ids), or None."""
    comps = dotted.split(".")
    ids = list(ids or []) + [None] * len(comps)
    fields = list(pq.read_schema(path))          # the root group's children
    out = []
    map_level = 0                                # 1: in a map, next is key_value; 2: next is key / value
    cur_type = None
    for i, name in enumerate(comps):
        if map_level == 1:
            out.append(name if name else "key_value")   # the repeated group (structural)
            map_level = 2
            continue
        if map_level == 2:
            if name not in ("key", "value"):
                return None
            out.append(name)
            cur_type = cur_type.key_type if name == "key" else cur_type.item_type
            map_level = 0
            if i + 1 < len(comps):
                if not pa.types.is_struct(cur_type):
                    return None
                fields = list(cur_type)
            continue
        by_id = {}
        for f in fields:
            fid = _fid(f)
            if fid is not None:
                if fid in by_id:
                    raise DuplicateFieldId("Parquet file contains multiple columns (%s, %s) with the same field id"
                                           % (by_id[fid].name, f.name))
                by_id[fid] = f
        hit = by_id.get(ids[i]) if ids[i] is not None and ids[i] >= 0 else None
        if hit is None:
            hit = next((f for f in fields if f.name == name), None)
        if hit is None:
            hit = next((f for f in fields if f.name.lower() == name.lower()), None)
        if hit is None:
            return None
        out.append(hit.name)
        t = hit.type
        if pa.types.is_map(t):
            cur_type = t
            map_level = 1
        elif pa.types.is_struct(t):
            fields = list(t)
        elif pa.types.is_list(t) or pa.types.is_large_list(t):
            fields = [t.value_field]
        elif i + 1 < len(comps):
            return None
    return ".".join(out)
