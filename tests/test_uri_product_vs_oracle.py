"""The product's URI canonical-key code (dk_uri.h, compiled for the host here) must induce exactly
the oracle's java.net.URI equivalence classes and accept/reject exactly the same strings."""
import ctypes as C
import itertools
import os
import random
import subprocess

import pytest

from oracle import ref

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "_uri_shim.so")


@pytest.fixture(scope="module")
def shim():
    src = os.path.join(HERE, "native", "uri_shim.cpp")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(
            os.path.join(HERE, "..", "delta_amd", "csrc", "dk_uri.h"))):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO, src])
    L = C.CDLL(SO)
    L.prod_uri_canon.restype = C.c_int64
    L.prod_uri_canon.argtypes = [C.c_char_p, C.c_int32, C.c_char_p, C.c_int64]
    L.prod_path_hash.argtypes = [C.c_char_p, C.c_int32, C.c_uint32, C.POINTER(C.c_uint64)]
    return L


def prod(L, s: bytes):
    buf = C.create_string_buffer(len(s) + 128)
    n = L.prod_uri_canon(s, len(s), buf, len(buf))
    return None if n < 0 else buf.raw[:n]


def orac(s: bytes):
    try:
        return ref.action_key(s, None)
    except ref.OracleError:
        return None


ALPHABET = list("aZ09/-._~%:@?#[]!$&'()*+,;= |\\^`{}\"<>") + ["%2F", "%2f", "%4a", "%zz", "//", "s3:", "file:",
                                                             "é", "\u00a0", "\u0085", "😀", "[::1]", ":8080",
                                                             "HOST", "host", "@", "my_b", "1.2.3.4"]


def _strings(rng, n):
    out = set()
    fixed = ["a/b", "a/B", "s3://Bucket/x", "s3://bucket/x", "S3://bucket:080/x", "s3://bucket:80/x",
             "file:///foo", "file:/foo", "/a/b", "file:/a/b", "s3://my_bucket/x", "s3://MY_bucket/x",
             "a#b", "a", "x?", "x", "special%20p@%23h", "special p@#h", "a%2Fb", "a%2fb", "//h", "//H/",
             "mailto:Joe@x", "MAILTO:Joe@x", "http://[::1]:80/a", "http://[::1]/a", "http://u@h/a",
             "http://U@h/a", "http://h:/a", "http://h/a", "date=2024-01-01/part-00000.parquet", "",
             "a:b", "A:b", "1:b", "#f", "?q", "http://1.2.3.4.5/x", "http://a-/x", "http://-a/x"]
    out.update(fixed)
    while len(out) < n:
        k = rng.randint(1, 8)
        out.add("".join(rng.choice(ALPHABET) for _ in range(k)))
    return [s.encode() for s in sorted(out)]


def test_accept_reject_and_classes(shim):
    rng = random.Random(20250218)
    strs = _strings(rng, 4000)
    P = {s: prod(shim, s) for s in strs}
    O = {s: orac(s) for s in strs}
    for s in strs:
        assert (P[s] is None) == (O[s] is None), (s, P[s], O[s])
    ok = [s for s in strs if P[s] is not None]
    # equivalence classes must coincide
    by_p, by_o = {}, {}
    for s in ok:
        by_p.setdefault(P[s], set()).add(s)
        by_o.setdefault(O[s][:-2], set()).add(s)   # strip the oracle's "\0\0" (no-DV) suffix
    assert sorted(map(sorted, by_p.values())) == sorted(map(sorted, by_o.values()))


def test_fast_path_hash_matches_slow_stream(shim):
    # the fast path must hash exactly the stream the generic emitter produces
    for s in [b"date=2024-01-01/part-00000-abc.c000.snappy.parquet", b"a/b/c", b"x" * 200]:
        h = C.c_uint64()
        assert shim.prod_path_hash(s, len(s), 0, C.byref(h)) == 0
        assert h.value != 0


def test_simple_word_hash_equals_generic(shim):
    shim.prod_simple_hash.argtypes = [C.c_char_p, C.c_int32, C.c_uint32, C.POINTER(C.c_uint64)]
    rng = random.Random(7)
    simple = "abcXYZ019-_.!~*'()/@&=+$,;"
    for n in list(range(0, 40)) + [83, 87, 200]:
        for _ in range(5):
            s = "".join(rng.choice(simple) for _ in range(n)).encode()
            if s.startswith(b"//"):
                continue
            a, b = C.c_uint64(), C.c_uint64()
            assert shim.prod_simple_hash(s, len(s), 3, C.byref(a)) == 1
            assert shim.prod_path_hash(s, len(s), 3, C.byref(b)) == 0
            assert a.value == b.value, s
    for s in [b"a:b", b"a%20", b"//x", b"a b", "é".encode()]:
        a = C.c_uint64()
        assert shim.prod_simple_hash(s, len(s), 3, C.byref(a)) == 0


def test_simple8_nibble_tables_match_uri_class(shim):
    """simple8 (v_perm nibble-table classifier) agrees with uri_class()&CC_SIMPLE for every byte value
    in every byte position of the 8-byte word (other positions padded with a simple char)."""
    shim.prod_simple8.argtypes = [C.c_uint64]
    shim.prod_uri_class_simple.argtypes = [C.c_uint32]
    for pos in range(8):
        for c in range(256):
            w = 0x6161616161616161 & ~(0xff << (8 * pos)) | (c << (8 * pos))
            want = 1 if (0 < c < 128 and shim.prod_uri_class_simple(c)) else 0
            assert shim.prod_simple8(w) == want, (pos, c)
