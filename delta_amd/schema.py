"""Kernel StructType JSON and the scan state's schemas (Scan.getScanState, KA/internal/ScanImpl.java:189-218).

* ``parse`` / ``to_json`` restate DataTypeJsonSerDe (KA/internal/types/DataTypeJsonSerDe.java:173-344
  parse, :445-555 write): primitive names, ``decimal`` -> decimal(10,0), ``decimal( p , s )`` ->
  ``decimal(p,s)``, struct / array / map objects, field metadata typed as FieldMetadata holds it
  (integral -> long, double, boolean, string, nested metadata, arrays typed by their head; the
  ``__COLLATIONS`` key is not kept in a struct field's metadata). Writing is Jackson's compact output:
  a field is {"name","type","nullable","metadata"}, and metadata entries come out in the iteration
  order of the java.util.HashMap FieldMetadata.Builder fills (KA/types/FieldMetadata.java:189):
  bucket (String.hashCode spread over the table size), then insertion order.
* ``scan_state`` is ScanImpl.getScanState: the logical read schema, its physical equivalent under the
  table's column mapping mode (ColumnMapping.convertToPhysicalSchema, KA/internal/util/
  ColumnMapping.java:102-115,201-259: physical names; under "id" each field's metadata is
  {parquet.field.id[, parquet.field.nested.ids]}), the physical data read schema without the partition
  columns (PartitionUtils.physicalSchemaWithoutPartitionColumns, KA/internal/util/PartitionUtils.java:
  59-79) plus ``_metadata.row_index`` when ``deletionVectors`` is a reader feature
  (StructField.METADATA_ROW_INDEX_COLUMN, KA/types/StructField.java:44-50), as JSON text.
"""
from __future__ import annotations

import json
import math
import re

PRIMITIVES = {"boolean", "byte", "short", "integer", "long", "float", "double", "date", "timestamp",
              "timestamp_ntz", "string", "binary", "variant"}
_DECIMAL = re.compile(r"decimal\(\s*(\d+)\s*,\s*(-?\d+)\s*\)\Z")
COLLATIONS_KEY = "__COLLATIONS"
PHYSICAL_NAME_KEY = "delta.columnMapping.physicalName"
COLUMN_ID_KEY = "delta.columnMapping.id"
NESTED_IDS_KEY = "delta.columnMapping.nested.ids"
PARQUET_FIELD_ID_KEY = "parquet.field.id"
PARQUET_NESTED_IDS_KEY = "parquet.field.nested.ids"
ROW_INDEX_COLUMN = "_metadata.row_index"


class SchemaError(ValueError):
    """The reference's IllegalArgumentException / KernelException for a schema it cannot parse."""


# ---- java.util.HashMap iteration order --------------------------------------------------------
def java_string_hash(s: str) -> int:
    """String.hashCode over UTF-16 code units, as a signed 32-bit int."""
    h = 0
    for ch in s:
        cp = ord(ch)
        units = [cp] if cp < 0x10000 else [0xD800 + ((cp - 0x10000) >> 10), 0xDC00 + ((cp - 0x10000) & 0x3FF)]
        for u in units:
            h = (31 * h + u) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


class MetaMap:
    """FieldMetadata's entries: a java.util.HashMap filled by put() in parse order; items() iterates as
    HashMap does -- by bucket of the final table (16 slots, doubled each time the size passes 3/4),
    then insertion order inside a bucket (resizes split buckets without reordering)."""

    def __init__(self, pairs=()):
        self._d = {}
        for k, v in pairs:
            self.put(k, v)

    def put(self, k, v):
        self._d[k] = v                   # a re-put keeps the key's place, as HashMap.put does

    def get(self, k, default=None):
        return self._d.get(k, default)

    def __contains__(self, k):
        return k in self._d

    def __len__(self):
        return len(self._d)

    def items(self):
        n = len(self._d)
        cap = 16
        while n > cap * 3 // 4:
            cap *= 2

        def bucket(k):
            h = java_string_hash(k) & 0xFFFFFFFF
            return (h ^ (h >> 16)) & (cap - 1)
        keys = list(self._d)
        order = sorted(range(len(keys)), key=lambda i: (bucket(keys[i]), i))
        return [(keys[i], self._d[keys[i]]) for i in order]


# ---- types ------------------------------------------------------------------------------------
class Field:
    def __init__(self, name, dtype, nullable=True, metadata=None):
        self.name, self.type, self.nullable = name, dtype, bool(nullable)
        self.metadata = metadata if metadata is not None else MetaMap()


class Struct:
    def __init__(self, fields):
        self.fields = list(fields)

    def get(self, name):
        for f in self.fields:
            if f.name == name:
                return f
        raise SchemaError("Field with name %s not found" % name)


class Array:
    def __init__(self, element, contains_null):
        self.element, self.contains_null = element, bool(contains_null)


class Map:
    def __init__(self, key, value, value_contains_null):
        self.key, self.value, self.value_contains_null = key, value, bool(value_contains_null)


def _meta(obj, include_collations=True):
    """parseFieldMetadata (DataTypeJsonSerDe.java:278-344)."""
    m = MetaMap()
    if obj is None:
        return m
    if not isinstance(obj, dict):
        raise SchemaError("Expected JSON object for struct field metadata")
    for k, v in obj.items():
        if not include_collations and k == COLLATIONS_KEY:
            continue
        if v is None or isinstance(v, (bool, int, float, str)):
            m.put(k, v)
        elif isinstance(v, dict):
            m.put(k, _meta(v))
        elif isinstance(v, list):
            if not v:
                m.put(k, ("long[]", []))
            elif isinstance(v[0], bool):
                m.put(k, ("boolean[]", [bool(x) for x in v]))
            elif isinstance(v[0], int):
                m.put(k, ("long[]", [int(x) for x in v]))
            elif isinstance(v[0], float):
                m.put(k, ("double[]", [float(x) for x in v]))
            elif isinstance(v[0], str):
                m.put(k, ("string[]", list(v)))
            elif isinstance(v[0], dict):
                m.put(k, ("metadata[]", [_meta(x) for x in v]))
            else:
                raise SchemaError("Unsupported type for Array as field metadata value: %s" % (v,))
        else:
            raise SchemaError("Unsupported type for field metadata value: %s" % (v,))
    return m


def _type(node):
    if isinstance(node, str):
        if node in PRIMITIVES:
            return node
        if node == "decimal":
            return "decimal(10,0)"
        if node.lower() == "void":
            raise SchemaError("void type encountered")
        m = _DECIMAL.match(node)
        if m:
            return "decimal(%d,%d)" % (int(m.group(1)), int(m.group(2)))
        raise SchemaError("%s is not a supported delta data type" % node)
    if isinstance(node, dict):
        t = node.get("type")
        if t == "struct":
            if len(node) != 2 or not isinstance(node.get("fields"), list):
                raise SchemaError("Expected JSON object with 2 fields for struct data type")
            return Struct([_field(f) for f in node["fields"]])
        if t == "array":
            if len(node) != 3:
                raise SchemaError("Expected JSON object with 3 fields for array data type")
            return Array(_type(node["elementType"]), node["containsNull"])
        if t == "map":
            if len(node) != 4:
                raise SchemaError("Expected JSON object with 4 fields for map data type")
            return Map(_type(node["keyType"]), _type(node["valueType"]), node["valueContainsNull"])
    raise SchemaError("Could not parse the following JSON as a valid Delta data type:\n%s" % json.dumps(node))


def _field(node):
    if not isinstance(node, dict):
        raise SchemaError("Expected JSON object for struct field")
    nullable = node.get("nullable")
    if not isinstance(nullable, bool):
        raise SchemaError("Expected boolean for fieldName=nullable")
    return Field(node["name"], _type(node["type"]), nullable, _meta(node.get("metadata"), include_collations=False))


def parse(text: str) -> Struct:
    """DataTypeJsonSerDe.deserializeStructType."""
    t = _type(json.loads(text))
    if not isinstance(t, Struct):
        raise SchemaError("Expected a struct type")
    return t


# ---- JSON writing (Jackson compact output) ----------------------------------------------------
def _jstr(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif o < 0x20:
            out.append({8: "\\b", 9: "\\t", 10: "\\n", 12: "\\f", 13: "\\r"}.get(o, "\\u%04X" % o))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _jdouble(x: float) -> str:
    """Double.toString (Jackson writeNumber(double)): plain notation in [1e-3, 1e7), else d.dddE<n>,
    from the shortest decimal digits that round-trip."""
    import decimal
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "-0.0" if math.copysign(1, x) < 0 else "0.0"
    sign, digits, exp = decimal.Decimal(repr(x)).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    e10 = exp + len(digits) - 1                       # x = d.ddd * 10^e10
    neg = "-" if sign else ""
    if -3 <= e10 < 7:
        if e10 >= 0:
            whole = (ds[:e10 + 1]).ljust(e10 + 1, "0")
            frac = ds[e10 + 1:] or "0"
        else:
            whole, frac = "0", "0" * (-e10 - 1) + ds
        return "%s%s.%s" % (neg, whole, frac)
    return "%s%s.%sE%d" % (neg, ds[0], ds[1:] or "0", e10)


def _jmeta(m: MetaMap) -> str:
    parts = []
    for k, v in m.items():
        if v is None:
            s = "null"
        elif isinstance(v, bool):
            s = "true" if v else "false"
        elif isinstance(v, int):
            s = str(v)
        elif isinstance(v, float):
            s = _jdouble(v)
        elif isinstance(v, str):
            s = _jstr(v)
        elif isinstance(v, MetaMap):
            s = _jmeta(v)
        else:
            kind, vals = v
            conv = {"long[]": str, "double[]": _jdouble, "boolean[]": lambda b: "true" if b else "false",
                    "string[]": _jstr, "metadata[]": _jmeta}[kind]
            s = "[" + ",".join(conv(x) for x in vals) + "]"
        parts.append(_jstr(k) + ":" + s)
    return "{" + ",".join(parts) + "}"


def type_json(t) -> str:
    if isinstance(t, str):
        return _jstr(t)
    if isinstance(t, Struct):
        return '{"type":"struct","fields":[' + ",".join(
            '{"name":%s,"type":%s,"nullable":%s,"metadata":%s}' % (
                _jstr(f.name), type_json(f.type), "true" if f.nullable else "false", _jmeta(f.metadata))
            for f in t.fields) + "]}"
    if isinstance(t, Array):
        return '{"type":"array","elementType":%s,"containsNull":%s}' % (
            type_json(t.element), "true" if t.contains_null else "false")
    if isinstance(t, Map):
        return '{"type":"map","keyType":%s,"valueType":%s,"valueContainsNull":%s}' % (
            type_json(t.key), type_json(t.value), "true" if t.value_contains_null else "false")
    raise SchemaError("not a data type: %r" % (t,))


to_json = type_json


# ---- column mapping and the scan state -------------------------------------------------------
def column_mapping_mode(configuration) -> str:
    """ColumnMapping.getColumnMappingMode / ColumnMappingMode.fromTableConfig."""
    v = (configuration or {}).get("delta.columnMapping.mode")
    if v is None:
        return "none"
    for mode in ("none", "id", "name"):
        if v.lower() == mode:
            return mode
    raise SchemaError("Invalid value for table property 'delta.columnMapping.mode': '%s'" % v)


def _physical_type(lt, pt, with_ids):
    if isinstance(lt, Struct):
        return physical_struct(lt, pt, with_ids)
    if isinstance(lt, Array):
        return Array(_physical_type(lt.element, pt.element, with_ids), lt.contains_null)
    if isinstance(lt, Map):
        return Map(_physical_type(lt.key, pt.key, with_ids), _physical_type(lt.value, pt.value, with_ids),
                   lt.value_contains_null)
    return lt


def physical_struct(logical: Struct, physical: Struct, with_ids: bool) -> Struct:
    """ColumnMapping.convertToPhysicalSchema (ColumnMapping.java:201-233)."""
    out = []
    for lf in logical.fields:
        pf = physical.get(lf.name)
        name = pf.metadata.get(PHYSICAL_NAME_KEY)
        if not isinstance(name, str):
            raise SchemaError("Expected '%s' to be of type 'String' but was missing" % PHYSICAL_NAME_KEY)
        ptype = _physical_type(lf.type, pf.type, with_ids)
        md = MetaMap()
        if with_ids:
            fid = pf.metadata.get(COLUMN_ID_KEY)
            if not isinstance(fid, int) or isinstance(fid, bool):
                raise SchemaError("Expected '%s' to be of type 'Long'" % COLUMN_ID_KEY)
            md.put(PARQUET_FIELD_ID_KEY, fid)
            if NESTED_IDS_KEY in pf.metadata:
                md.put(PARQUET_NESTED_IDS_KEY, pf.metadata.get(NESTED_IDS_KEY))
        out.append(Field(name, ptype, lf.nullable, md))
    return Struct(out)


def scan_state(metadata: dict, protocol: dict, table_path: str, read_schema: str | None = None) -> dict:
    """ScanImpl.getScanState (ScanImpl.java:189-218) as a dict with ScanStateRow's field names
    (KA/internal/data/ScanStateRow.java:35-44)."""
    snapshot_schema = parse(metadata["schemaString"])
    logical = parse(read_schema) if read_schema is not None else snapshot_schema
    mode = column_mapping_mode(metadata.get("configuration"))
    physical = logical if mode == "none" else physical_struct(logical, snapshot_schema, mode == "id")
    parts = set(metadata.get("partitionColumns") or [])
    if parts:
        phys_to_logical = {p.name: l.name for l, p in zip(logical.fields, physical.fields)}
        data = Struct([f for f in physical.fields if phys_to_logical.get(f.name) not in parts])
    else:
        data = physical
    if "deletionVectors" in ((protocol or {}).get("readerFeatures") or []):
        data = Struct(data.fields + [Field(ROW_INDEX_COLUMN, "long", False, MetaMap([("isMetadataColumn", True)]))])
    return {"configuration": dict(metadata.get("configuration") or {}),
            "logicalSchemaString": to_json(logical),
            "physicalSchemaString": to_json(physical),
            "physicalDataReadSchemaString": to_json(data),
            "partitionColumns": list(metadata.get("partitionColumns") or []),
            "minReaderVersion": (protocol or {}).get("minReaderVersion"),
            "minWriterVersion": (protocol or {}).get("minWriterVersion"),
            "tablePath": table_path}
