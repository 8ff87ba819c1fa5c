"""tableRoot (scan-file column 1): dataPath.toUri().toString() of the resolved table path
(ActiveAddFilesIterator.java:251; DefaultFileSystemClient.resolvePath, DefaultFileSystemClient.java:82-86).

CPU: the product's restatement (delta_amd.kernel.table_root_uri) against known answers derived from
java.net.URI's multi-argument-constructor quoting, and against the oracle's restatement.
GPU: a scan of a table whose directory name needs quoting returns that tableRoot on every batch."""
import os

import pytest

from delta_amd import kernel as K
from oracle import ref

KNOWN = {
    "/tmp/t": "file:/tmp/t",
    "/tmp/t/": "file:/tmp/t",                       # Path.normalizePath drops the trailing slash
    "/tmp//a///b": "file:/tmp/a/b",                 # ... and collapses "//"
    "/tmp/./a/../b": "file:/tmp/b",                 # URI.normalize
    "/tmp/a b": "file:/tmp/a%20b",
    "/tmp/x%y": "file:/tmp/x%25y",                  # '%' is always quoted
    "/tmp/a#b?c": "file:/tmp/a%23b%3Fc",
    "/tmp/[v]{w}|\\^`\"<>": "file:/tmp/%5Bv%5D%7Bw%7D%7C%5C%5E%60%22%3C%3E",
    "/tmp/keep-_.!~*'()@,;:$&+=": "file:/tmp/keep-_.!~*'()@,;:$&+=",
    "/tmp/café/日本": "file:/tmp/café/日本",   # non-ASCII "other" chars stay
    "/tmp/nb sp": "file:/tmp/nb%C2%A0sp",       # Character.isSpaceChar -> UTF-8 escaped
    "/tmp/c1\u0085x": "file:/tmp/c1%C2%85x",         # ISO control
    "/tmp/tab\tx": "file:/tmp/tab%09x",
}


@pytest.mark.parametrize("path", sorted(KNOWN))
def test_known_answers(path):
    assert K.table_root_uri(path) == KNOWN[path]
    assert ref.table_root_uri(path) == KNOWN[path]


def test_relative_path_resolves_against_cwd(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    assert K.table_root_uri("t") == "file:" + str(tmp_path) + "/t"
    assert ref.table_root_uri("t") == K.table_root_uri("t")


@pytest.mark.gpu
def test_gpu_scan_table_root_quoted(tmp_path):
    from delta_amd import synth
    from tests.parity_util import assert_same, oracle_scan, product_scan
    d = os.path.join(str(tmp_path), "my table %x é")
    synth.write_table(d, synth.TableSpec(n_adds=3_000, n_commits=3))
    p, o = product_scan(d), oracle_scan(d)
    assert_same(p, o)
    want = "file:" + str(tmp_path) + "/my%20table%20%25x%20é"
    assert {r[-1] for r in p[1]} == {want}
