"""The checkpoint writer's Parquet schema against SingleAction.CHECKPOINT_SCHEMA (CPU).

Expected field order and nullability are restated from the reference's schema definitions
(kernel-api/.../internal/actions/: SingleAction.java:30-37, AddFile.java:42-70, RemoveFile.java:23-38,
DeletionVectorDescriptor.java:84-90, Metadata.java:57-72, Format.java:42-48, Protocol.java:49-54,
SetTransaction.java:28-32, DomainMetadata.java:34-38). When /root/reference is present the restatement
is itself checked against the Java text (`.add("name", TYPE, nullable)` lines)."""
import os
import re

import pytest

from delta_amd.checkpoint import checkpoint_schema

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
