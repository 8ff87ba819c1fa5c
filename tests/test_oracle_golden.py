"""Pins the oracle against the reference's own golden tables and the answers its tests assert
(SURVEY.md App. E). Runs where /root/reference exists (this container); skipped elsewhere."""
import os
import urllib.parse

import numpy as np
import pyarrow.parquet as pq
import pytest

from oracle import ref


def _names(sf):
    return {os.path.basename(urllib.parse.unquote(s[0].decode())) for s in sf}


def _data_ids(root, sf, col="id"):
    out = []
    for s in sf:
        p = urllib.parse.unquote(s[0].decode())
        t = pq.read_table(os.path.join(root, p))
        out.extend(t.column(col).to_pylist())
    return sorted(out)


def _dir_data_files(root):
    return {f for f in os.listdir(root) if f.endswith("snappy.parquet") and os.path.isfile(os.path.join(root, f))}


@pytest.mark.parametrize("bs", [2, 1024])
def test_checkpoint(golden_root, bs):
    # KDT/LogReplaySuite.scala:131-136
    r = ref.replay(os.path.join(golden_root, "checkpoint"), json_batch_size=bs)
    assert r.version == 14 and len(r.scan_files()) == 1


def test_snapshot_sequence(golden_root):
    # KDT/LogReplaySuite.scala:139-219
    g = lambda n: os.path.join(golden_root, n)
    d0 = _dir_data_files(g("snapshot-data0"))
    r = ref.replay(g("snapshot-data0"), json_batch_size=2)
    assert r.version == 0 and _names(r.scan_files()) == d0
    d01 = _dir_data_files(g("snapshot-data1"))
    r = ref.replay(g("snapshot-data1"), json_batch_size=2)
    assert r.version == 1 and _names(r.scan_files()) == d01
    d2 = _dir_data_files(g("snapshot-data2")) - d01
    r = ref.replay(g("snapshot-data2"), json_batch_size=2)
    assert r.version == 2 and _names(r.scan_files()) == d2
    r = ref.replay(g("snapshot-data3"), json_batch_size=2)
    assert r.version == 3 and _names(r.scan_files()) == _dir_data_files(g("snapshot-data3")) - d01
    r = ref.replay(g("snapshot-data2-deleted"), json_batch_size=2)
    assert r.version == 4 and _names(r.scan_files()) == _dir_data_files(g("snapshot-data2-deleted")) - d01 - d2
    r = ref.replay(g("snapshot-repartitioned"), json_batch_size=2)
    assert r.version == 5 and len(r.scan_files()) == 2
    r = ref.replay(g("snapshot-vacuumed"), json_batch_size=2)
    assert r.version == 5 and _names(r.scan_files()) == _dir_data_files(g("snapshot-vacuumed"))


def test_dv_key_cases(golden_root):
    # KDT/LogReplaySuite.scala:221-229
    sf = ref.replay(os.path.join(golden_root, "log-replay-dv-key-cases"), json_batch_size=2).scan_files()
    assert len(sf) == 1 and sf[0][5][4] == 3


def test_special_characters(golden_root):
    # KDT/LogReplaySuite.scala:231-245
    assert ref.replay(os.path.join(golden_root, "log-replay-special-characters-a")).scan_files() == []
    sf = ref.replay(os.path.join(golden_root, "log-replay-special-characters-b")).scan_files()
    assert len(sf) == 1 and _names(sf) == {"special p@#h"}


def test_delete_re_add(golden_root):
    # KDT/LogReplaySuite.scala:279-293
    r = ref.replay(os.path.join(golden_root, "delete-re-add-same-file-different-transactions"), json_batch_size=2)
    sf = r.scan_files()
    assert {s[0].split(b"/")[-1] for s in sf} == {b"foo", b"bar"}
    assert [s[3] for s in sf if s[0].endswith(b"foo")] == [1700000000000]


@pytest.mark.parametrize("name,expected", [
    ("basic-with-inserts-deletes-checkpoint",  # KDT/LogReplaySuite.scala:46-55
     list(range(0, 5)) + list(range(10, 15)) + list(range(20, 25)) + list(range(30, 35)) +
     list(range(40, 45)) + list(range(50, 66))),
    ("only-checkpoint-files", list(range(5, 10)) + list(range(0, 20))),   # :83-90
    ("multi-part-checkpoint", [0] + list(range(0, 30))),                   # KDT/DeltaTableReadsSuite.scala:271-276
    ("basic-with-inserts-overwrite-restore", list(range(0, 200))),          # :74-81
])
def test_data_answers(golden_root, name, expected):
    root = os.path.join(golden_root, name)
    for bs in (2, 1024):
        sf = ref.replay(root, json_batch_size=bs).scan_files()
        assert _data_ids(root, sf) == sorted(expected)


@pytest.mark.parametrize("name", ["v2-checkpoint-json", "v2-checkpoint-parquet"])
def test_v2_checkpoint(golden_root, name):
    # kernel/examples/.../ReadIntegrationTestSuite.java:99-115: 10 rows
    root = os.path.join(golden_root, name)
    sf = ref.replay(root).scan_files()
    n = sum(pq.read_metadata(os.path.join(root, urllib.parse.unquote(s[0].decode()))).num_rows for s in sf)
    assert n == 10


def test_uri_key_semantics():
    """java.net.URI.equals semantics."""
    k = lambda s: ref.action_key(s.encode(), None)
    assert k("a/b%2Fc") == k("a/b%2fc")             # %XX hex case-insensitive
    assert k("a/b") != k("a/B")
    assert k("S3://Bucket/x") == k("s3://bucket/x")  # scheme + server host case-insensitive
    assert k("s3://bucket:080/x") == k("s3://bucket:80/x")
    assert k("file:///foo") == k("file:/foo")         # empty authority is undefined
    assert k("/a/b") != k("file:/a/b")               # no canonicalisation
    assert k("s3://my_bucket/x") != k("s3://MY_bucket/x")   # registry authority: case-sensitive
    for bad in ["a b", "a%zz", "a|b", "a#b#c", "a[b]", "s3://", ":x"]:
        with pytest.raises(ref.OracleError):
            k(bad)
    assert k("a#b") != k("a")
    assert k("x?") != k("x")
    dv = ref.action_key(b"p", (b"u", b"ab", 1))
    assert dv.endswith(b"\x01uab@Optional[1]")
    assert ref.action_key(b"p", (b"u", b"ab", None)).endswith(b"\x01uab")
    assert ref.java_utf8(b"a\xffb") == "a�b".encode()
    assert ref.java_utf8(b"\xe2\x82") == "�".encode()
    assert ref.java_utf8("é€😀".encode()) == "é€😀".encode()
