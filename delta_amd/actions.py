"""Protocol and Metadata actions of the snapshot-load pass, and the read-support check.

Reference (paths under /root/reference/kernel/kernel-api/src/main/java/io/delta/kernel/internal/):
  Protocol.fromColumnVector / FULL_SCHEMA        actions/Protocol.java:33-54 (null feature arrays
                                                 read as empty lists)
  Metadata.fromColumnVector / FULL_SCHEMA        actions/Metadata.java:35-71 (id, format,
                                                 schemaString, partitionColumns, configuration are
                                                 required; name, description, createdTime optional)
  TableFeatures.validateReadSupportedTable       TableFeatures.java:47-98
  ColumnMapping.getColumnMappingMode             util/ColumnMapping.java:41-51,78-92
  DeltaErrors.unsupportedReader*                 DeltaErrors.java:144-162
  LogReplay.loadTableProtocolAndMetadata         replay/LogReplay.java:220-314 (validates once both
                                                 are found)

The commit-JSON side decodes with DefaultJsonRow's rules for the P&M read schema
(kernel-defaults/.../internal/data/DefaultJsonRow.java:136-357): an int field needs an integral
JSON number in int range, a long field an integral number, strings must be JSON strings, a missing
or null required field is an error.
"""
from __future__ import annotations

from ._lib import DkError

SUPPORTED_READER_FEATURES = frozenset([
    "columnMapping", "deletionVectors", "timestampNtz", "typeWidening-preview", "typeWidening",
    "vacuumProtocolCheck", "variantType", "variantType-preview", "v2Checkpoint"])
COLUMN_MAPPING_MODE_KEY = "delta.columnMapping.mode"
COLUMN_MAPPING_MODES = ("none", "id", "name")


class KernelException(DkError):
    pass


def _int(v, name, bits=32):
    if isinstance(v, bool) or not isinstance(v, int) or not -(1 << (bits - 1)) <= v < (1 << (bits - 1)):
        raise KernelException("Couldn't decode %r for field %s, expected a%s" % (v, name, "n int" if bits == 32 else " long"))
    return v


def _str(v, name):
    if not isinstance(v, str):
        raise KernelException("Couldn't decode %r for field %s, expected a string" % (v, name))
    return v


def _str_list(v, name):
    if v is None:
        return None
    if not isinstance(v, list):
        raise KernelException("Couldn't decode %r for field %s, expected an array" % (v, name))
    return [None if x is None else _str(x, name) for x in v]


def _str_map(v, name):
    if v is None:
        return None
    if not isinstance(v, dict):
        raise KernelException("Couldn't decode %r for field %s, expected a map" % (v, name))
    return {_str(k, name): (None if x is None else _str(x, name)) for k, x in v.items()}


def _required(obj, key, action):
    if obj.get(key) is None:
        raise KernelException("Field `%s` in `%s` is not nullable, but it is missing or null" % (key, action))
    return obj[key]


def protocol_from_json(obj: dict) -> dict:
    """A commit-JSON protocol action as Protocol.fromColumnVector builds it."""
    return {"minReaderVersion": _int(_required(obj, "minReaderVersion", "protocol"), "minReaderVersion"),
            "minWriterVersion": _int(_required(obj, "minWriterVersion", "protocol"), "minWriterVersion"),
            "readerFeatures": _str_list(obj.get("readerFeatures"), "readerFeatures") or [],
            "writerFeatures": _str_list(obj.get("writerFeatures"), "writerFeatures") or []}


def metadata_from_json(obj: dict) -> dict:
    """A commit-JSON metaData action as Metadata.fromColumnVector builds it."""
    fmt = _required(obj, "format", "metaData")
    if not isinstance(fmt, dict):
        raise KernelException("Couldn't decode %r for field format, expected a struct" % (fmt,))
    created = obj.get("createdTime")
    return {"id": _str(_required(obj, "id", "metaData"), "id"),
            "name": None if obj.get("name") is None else _str(obj["name"], "name"),
            "description": None if obj.get("description") is None else _str(obj["description"], "description"),
            "format": {"provider": _str(_required(fmt, "provider", "format"), "provider"),
                       "options": _str_map(fmt.get("options"), "options") or {}},
            "schemaString": _str(_required(obj, "schemaString", "metaData"), "schemaString"),
            "partitionColumns": _str_list(_required(obj, "partitionColumns", "metaData"), "partitionColumns"),
            "createdTime": None if created is None else _int(created, "createdTime", 64),
            "configuration": _str_map(_required(obj, "configuration", "metaData"), "configuration")}


def column_mapping_mode(metadata: dict) -> str:
    """ColumnMapping.getColumnMappingMode: absent -> none; otherwise one of none/id/name, any case."""
    v = (metadata.get("configuration") or {}).get(COLUMN_MAPPING_MODE_KEY)
    if v is None:
        return "none"
    for m in COLUMN_MAPPING_MODES:
        if m.lower() == v.lower():
            return m
    raise KernelException("Invalid value for table property '%s': '%s'. Needs to be one of: [%s]."
                          % (COLUMN_MAPPING_MODE_KEY, v, ", ".join(COLUMN_MAPPING_MODES)))


def validate_read_supported(protocol: dict, table_path: str, metadata: dict | None):
    """TableFeatures.validateReadSupportedTable (TableFeatures.java:76-98)."""
    rv = protocol["minReaderVersion"]
    if rv == 1:
        return
    if rv == 2:
        if metadata is not None:
            column_mapping_mode(metadata)
        return
    if rv == 3:
        feats = protocol.get("readerFeatures") or []
        bad = [f for f in feats if f not in SUPPORTED_READER_FEATURES]
        if bad:
            raise KernelException(
                "Unsupported Delta reader features: table `%s` requires reader table features [%s] which is "
                "unsupported by this version of Delta Kernel." % (table_path, ", ".join(sorted(set(bad)))))
        if "columnMapping" in feats and metadata is not None:
            column_mapping_mode(metadata)
        return
    raise KernelException(
        "Unsupported Delta protocol reader version: table `%s` requires reader version %d which is unsupported "
        "by this version of Delta Kernel." % (table_path, rv))
