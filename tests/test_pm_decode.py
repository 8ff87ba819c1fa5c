"""Commit-side protocol / metaData decode (dk_json_pm_decode: host C++ in libdkgpu, DefaultJsonRow's
rules for Protocol / Metadata FULL_SCHEMA, kernel-defaults/.../internal/data/DefaultJsonRow.java:
136-357) against the oracle's restatement (oracle/ref.py _pm_json_protocol / _pm_json_metadata):
the same values for every accepted line, an error for every line either rejects. Host logic only:
no device call."""
import ctypes as C
import json

import pytest

from delta_amd._lib import DkError, check, lib
from oracle import ref

META = {"id": "t1", "name": None, "format": {"provider": "parquet", "options": {}},
        "schemaString": '{"type":"struct","fields":[]}', "partitionColumns": ["date"],
        "createdTime": 1700000000000, "configuration": {"delta.appendOnly": "true"}}
PROTO = {"minReaderVersion": 3, "minWriterVersion": 7, "readerFeatures": ["deletionVectors"],
         "writerFeatures": ["deletionVectors", "appendOnly"]}


def _variants():
    good = [("protocol", PROTO), ("protocol", {"minReaderVersion": 1, "minWriterVersion": 2}),
            ("metaData", META), ("metaData", dict(META, name="né", description="d\"q\\", createdTime=None)),
            ("metaData", dict(META, format={"provider": "parquet"}, configuration={}, partitionColumns=[])),
            ("metaData", dict(META, id="☃😀"))]
    bad = [("protocol", dict(PROTO, minReaderVersion=1.0)), ("protocol", dict(PROTO, minReaderVersion=1 << 31)),
           ("protocol", dict(PROTO, minWriterVersion=None)), ("protocol", {k: v for k, v in PROTO.items() if k != "minReaderVersion"}),
           ("protocol", dict(PROTO, readerFeatures=["a", None])), ("protocol", dict(PROTO, writerFeatures="x")),
           ("protocol", dict(PROTO, minReaderVersion="3")), ("protocol", dict(PROTO, readerFeatures=[1])),
           ("metaData", dict(META, id=None)), ("metaData", dict(META, id=7)), ("metaData", dict(META, createdTime=1.5)),
           ("metaData", dict(META, createdTime=1 << 63)), ("metaData", dict(META, configuration={"k": None})),
           ("metaData", dict(META, partitionColumns=None)), ("metaData", dict(META, partitionColumns=["a", None])),
           ("metaData", dict(META, format={"options": {}})), ("metaData", dict(META, format="parquet")),
           ("metaData", dict(META, format={"provider": "p", "options": {"a": None}})),
           ("metaData", dict(META, name=5))]
    return [(k, v, True) for k, v in good] + [(k, v, False) for k, v in bad]


def _product(tmp_path, kind, value):
    line = json.dumps({kind: value}).encode()
    p = tmp_path / "00000000000000000001.json"
    p.write_bytes(b'{"commitInfo":{}}\n' + line + b"\n")
    n = C.c_int64()
    buf = C.create_string_buffer(64)
    rc = lib().dk_json_pm_decode(str(p).encode(), 18, len(line), 0 if kind == "protocol" else 1, buf, len(buf), C.byref(n))
    if rc == 2:
        buf = C.create_string_buffer(n.value + 16)
        rc = lib().dk_json_pm_decode(str(p).encode(), 18, len(line), 0 if kind == "protocol" else 1, buf, len(buf), C.byref(n))
    check(rc)
    return json.loads(buf.raw[:n.value].decode("utf-8"))


def _oracle(kind, value):
    return ref._pm_json_protocol(value) if kind == "protocol" else ref._pm_json_metadata(value)


@pytest.mark.parametrize("case", range(len(_variants())))
def test_pm_decode_matches_oracle(tmp_path, case):
    kind, value, ok = _variants()[case]
    if ok:
        got = _product(tmp_path, kind, value)
        want = _oracle(kind, value)
        if kind == "protocol":
            got = dict(got, readerFeatures=got["readerFeatures"] or [], writerFeatures=got["writerFeatures"] or [])
        else:
            got = dict(got, format={"provider": got["format"]["provider"], "options": got["format"]["options"] or {}})
        assert got == want
    else:
        with pytest.raises(DkError):
            _product(tmp_path, kind, value)
        with pytest.raises(ref.OracleError):
            _oracle(kind, value)
