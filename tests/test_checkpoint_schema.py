"""The checkpoint writer's Parquet schema against SingleAction.CHECKPOINT_SCHEMA (CPU).

Expected field order and nullability are restated from the reference's schema definitions
(kernel-api/.../internal/actions/: SingleAction.java:30-37, AddFile.java:42-70, RemoveFile.java:23-38,
DeletionVectorDescriptor.java:84-90, Metadata.java:57-72, Format.java:42-48, Protocol.java:49-54,
SetTransaction.java:28-32, DomainMetadata.java:34-38). When /root/reference is present the restatement
is itself checked against the Java text (`.add("name", TYPE, nullable)` lines)."""
import os
import re

import pytest


# ---- CHECKPOINT_SCHEMA as Arrow types -----------------------------------------------------------
# Field order and nullability follow the reference definitions (paths under kernel-api/.../internal/
# actions/): SingleAction.CHECKPOINT_SCHEMA (SingleAction.java:30-37), AddFile.FULL_SCHEMA =
# SCHEMA_WITHOUT_STATS + stats (AddFile.java:42-70), RemoveFile.FULL_SCHEMA (RemoveFile.java:23-38),
# DeletionVectorDescriptor.READ_SCHEMA (:84-90), Metadata.FULL_SCHEMA (Metadata.java:57-72) with
# Format.FULL_SCHEMA (Format.java:42-48), Protocol.FULL_SCHEMA (Protocol.java:49-54),
# SetTransaction.FULL_SCHEMA (SetTransaction.java:28-32), DomainMetadata.FULL_SCHEMA
# (DomainMetadata.java:34-38). `nullable=False` becomes a REQUIRED Parquet field.
def checkpoint_schema():
    import pyarrow as pa
    S, L, B, I = pa.string(), pa.int64(), pa.bool_(), pa.int32()

    def F(name, t, nullable=True):
        return pa.field(name, t, nullable=nullable)

    def M(value_nullable=True):                 # MapType(string, string, valueContainsNull)
        return pa.map_(F("key", S, False), F("value", S, value_nullable))

    def A(contains_null):                       # ArrayType(string, containsNull)
        return pa.list_(F("element", S, contains_null))

    dv = pa.struct([F("storageType", S, False), F("pathOrInlineDv", S, False), F("offset", I),
                    F("sizeInBytes", I, False), F("cardinality", L, False)])
    add = pa.struct([F("path", S, False), F("partitionValues", M(), False), F("size", L, False),
                     F("modificationTime", L, False), F("dataChange", B, False), F("deletionVector", dv),
                     F("tags", M()), F("baseRowId", L), F("defaultRowCommitVersion", L), F("stats", S)])
    rm = pa.struct([F("path", S, False), F("deletionTimestamp", L), F("dataChange", B, False),
                    F("extendedFileMetadata", B), F("partitionValues", M()), F("size", L), F("stats", S),
                    F("tags", M()), F("deletionVector", dv), F("baseRowId", L), F("defaultRowCommitVersion", L)])
    fmt = pa.struct([F("provider", S, False), F("options", M(False))])
    meta = pa.struct([F("id", S, False), F("name", S), F("description", S), F("format", fmt, False),
                      F("schemaString", S, False), F("partitionColumns", A(False), False), F("createdTime", L),
                      F("configuration", M(False), False)])
    proto = pa.struct([F("minReaderVersion", I, False), F("minWriterVersion", I, False),
                       F("readerFeatures", A(False)), F("writerFeatures", A(False))])
    txn = pa.struct([F("appId", S, False), F("version", L, False), F("lastUpdated", L)])
    dm = pa.struct([F("domain", S, False), F("configuration", S, False), F("removed", B, False)])
    return pa.schema([("txn", txn), ("add", add), ("remove", rm), ("metaData", meta), ("protocol", proto),
                      ("domainMetadata", dm)])


_ADD_KEYS = ("path", "partitionValues", "size", "modificationTime", "dataChange", "stats", "tags", "deletionVector",
             "baseRowId", "defaultRowCommitVersion")
_RM_KEYS = ("path", "deletionTimestamp", "dataChange", "extendedFileMetadata", "partitionValues", "size", "stats",
            "tags", "deletionVector", "baseRowId", "defaultRowCommitVersion")
_DV_KEYS = ("storageType", "pathOrInlineDv", "offset", "sizeInBytes", "cardinality")



ACT = "/root/reference/kernel/kernel-api/src/main/java/io/delta/kernel/internal/actions"

# struct -> [(field, nullable)] in declaration order
EXPECTED = {
    "add": [("path", False), ("partitionValues", False), ("size", False), ("modificationTime", False),
            ("dataChange", False), ("deletionVector", True), ("tags", True), ("baseRowId", True),
            ("defaultRowCommitVersion", True), ("stats", True)],
    "remove": [("path", False), ("deletionTimestamp", True), ("dataChange", False), ("extendedFileMetadata", True),
               ("partitionValues", True), ("size", True), ("stats", True), ("tags", True),
               ("deletionVector", True), ("baseRowId", True), ("defaultRowCommitVersion", True)],
    "deletionVector": [("storageType", False), ("pathOrInlineDv", False), ("offset", True),
                       ("sizeInBytes", False), ("cardinality", False)],
    "metaData": [("id", False), ("name", True), ("description", True), ("format", False),
                 ("schemaString", False), ("partitionColumns", False), ("createdTime", True),
                 ("configuration", False)],
    "format": [("provider", False), ("options", True)],
    "protocol": [("minReaderVersion", False), ("minWriterVersion", False), ("readerFeatures", True),
                 ("writerFeatures", True)],
    "txn": [("appId", False), ("version", False), ("lastUpdated", True)],
    "domainMetadata": [("domain", False), ("configuration", False), ("removed", False)],
}
JAVA = {"add": ("AddFile.java", "SCHEMA_WITHOUT_STATS"), "remove": ("RemoveFile.java", "FULL_SCHEMA"),
        "deletionVector": ("DeletionVectorDescriptor.java", "READ_SCHEMA"), "metaData": ("Metadata.java", "FULL_SCHEMA"),
        "format": ("Format.java", "FULL_SCHEMA"), "protocol": ("Protocol.java", "FULL_SCHEMA"),
        "txn": ("SetTransaction.java", "FULL_SCHEMA"), "domainMetadata": ("DomainMetadata.java", "FULL_SCHEMA")}


def _struct_fields(t):
    return [(t.field(i).name, t.field(i).nullable) for i in range(t.num_fields)]


def test_arrow_schema_matches_reference_order_and_nullability():
    s = checkpoint_schema()
    assert s.names == ["txn", "add", "remove", "metaData", "protocol", "domainMetadata"]   # SingleAction.java:30-37
    for top in ("add", "remove", "metaData", "protocol", "txn", "domainMetadata"):
        assert _struct_fields(s.field(top).type) == EXPECTED[top], top
    add = s.field("add").type
    assert _struct_fields(add.field("deletionVector").type) == EXPECTED["deletionVector"]
    assert _struct_fields(s.field("remove").type.field("deletionVector").type) == EXPECTED["deletionVector"]
    assert _struct_fields(s.field("metaData").type.field("format").type) == EXPECTED["format"]
    # map keys are never null; metaData.configuration / format.options values are non-null
    # (MapType(string, string, false)); array elements of features / partitionColumns are non-null
    pv = add.field("partitionValues").type
    assert not pv.key_field.nullable and pv.item_field.nullable
    conf = s.field("metaData").type.field("configuration").type
    assert not conf.key_field.nullable and not conf.item_field.nullable
    assert not s.field("protocol").type.field("readerFeatures").type.value_field.nullable


def test_parquet_repetition_of_written_schema(tmp_path):
    import pyarrow as pa
    import pyarrow.parquet as pq
    s = checkpoint_schema()
    pq.write_table(pa.table({n: pa.array([], type=s.field(n).type) for n in s.names}, schema=s),
                   str(tmp_path / "x.parquet"))
    ps = pq.ParquetFile(str(tmp_path / "x.parquet")).schema
    rep = {ps.column(i).path: ps.column(i).max_definition_level for i in range(len(ps))}
    # add optional (1) -> path required: def 1; deletionVector optional (2) -> storageType required: 2,
    # offset optional: 3; partitionValues required map: key def 2 (key_value repeated), value def 3
    assert rep["add.path"] == 1
    assert rep["add.deletionVector.storageType"] == 2
    assert rep["add.deletionVector.offset"] == 3
    assert rep["add.stats"] == 2
    assert rep["add.partitionValues.key_value.key"] == 2
    assert rep["add.partitionValues.key_value.value"] == 3
    assert rep["remove.path"] == 1
    assert rep["protocol.minReaderVersion"] == 1


@pytest.mark.skipif(not os.path.isdir(ACT), reason="reference sources not present")
def test_restatement_matches_reference_java():
    for struct, (fname, const) in JAVA.items():
        text = open(os.path.join(ACT, fname)).read()
        at = text.index(const + " =")
        end = text.index(";", at)
        body = text[at:end]
        fields = []
        for seg in body.split(".add(")[1:]:
            # top-level arguments of .add(name, type[, nullable]); StructType.add(name, type)
            # defaults to nullable
            args, depth, cur = [], 0, ""
            for ch in seg:
                if ch == ")" and depth == 0:
                    break
                depth += (ch == "(") - (ch == ")")
                if ch == "," and depth == 0:
                    args.append(cur)
                    cur = ""
                else:
                    cur += ch
            args.append(cur)
            args = [re.sub(r"/\*.*?\*/", "", a).strip() for a in args]
            name = re.match(r'"(\w+)"', args[0]).group(1)
            fields.append((name, args[2] == "true" if len(args) > 2 else True))
        exp = EXPECTED[struct]
        if struct == "add":
            exp = exp[:-1]            # stats: SCHEMA_WITH_STATS = SCHEMA_WITHOUT_STATS.add(JSON_STATS_FIELD)
        assert fields == exp, (struct, fields)
