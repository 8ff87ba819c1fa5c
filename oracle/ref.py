"""CPU ORACLE (test infrastructure only) — Delta Kernel log replay restated in Python over the C
oracle ``oracle/_ref/libdk_ref.so``.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module, and only as the checker / CPU baseline. The product (``delta_amd``) never imports it.

Restates, for the ``getScanFiles`` path:

* log-segment selection and ordering: ``SnapshotManager.getLogSegmentForVersion``
  (kernel-api/.../internal/snapshot/SnapshotManager.java:311-566, latest version only),
  ``Checkpointer.getLatestCompleteCheckpointFromList`` (internal/checkpoints/Checkpointer.java:46-73),
  ``LogSegment.allLogFilesReversed`` (internal/snapshot/LogSegment.java:166-178);
* file sequencing: ``ActionsIterator.getNextActionsIter`` (internal/replay/ActionsIterator.java:291-362),
  multi-part grouping ``retrieveRemainingCheckpointFiles`` (:395-417), V2 sidecars
  ``extractSidecarsFromBatch`` (:256-283);
* commit JSON decode: ``DefaultJsonHandler.readJsonFiles`` (kernel-defaults/.../engine/
  DefaultJsonHandler.java:79-157, one batch = up to ``json_batch_size`` lines of ONE file) and
  ``DefaultJsonRow.decodeElement/decodeField`` (internal/data/DefaultJsonRow.java:136-357);
* reconciliation: ``ActiveAddFilesIterator.prepareNext`` (internal/replay/ActiveAddFilesIterator.java:146-275)
  and ``ScanMetrics`` (internal/metrics/ScanMetrics.java:28-40);
* keys: ``LogReplayUtils.pathToUri`` (internal/replay/LogReplayUtils.java:83-89) +
  ``DeletionVectorDescriptor.getUniqueId`` (internal/actions/DeletionVectorDescriptor.java:167-174)
  via the C restatement ``dkr_action_key``.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import re
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_ref", "libdk_ref.so")
_lib = None


class OracleError(RuntimeError):
    pass


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.dkr_open.restype = C.c_void_p
        L.dkr_open.argtypes = [C.c_char_p, C.c_int64]
        L.dkr_errmsg.restype = C.c_char_p
        L.dkr_num_rows.restype = C.c_int64
        L.dkr_num_rows.argtypes = [C.c_void_p]
        L.dkr_num_leaves.argtypes = [C.c_void_p]
        L.dkr_num_row_groups.argtypes = [C.c_void_p]
        L.dkr_select_row_groups.argtypes = [C.c_void_p, C.c_char_p]
        L.dkr_leaf_path.restype = C.c_char_p
        L.dkr_leaf_path.argtypes = [C.c_void_p, C.c_int]
        L.dkr_leaf_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.dkr_chunk_info.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int64)]
        L.dkr_read_leaf.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.dkr_col_free.argtypes = [C.c_void_p]
        L.dkr_close.argtypes = [C.c_void_p]
        L.dkr_uri_key.restype = C.c_int64
        L.dkr_uri_key.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64]
        L.dkr_java_utf8.restype = C.c_int64
        L.dkr_java_utf8.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64]
        L.dkr_action_key.restype = C.c_int64
        L.dkr_action_key.argtypes = [C.c_char_p, C.c_int64, C.c_int, C.c_char_p, C.c_int64,
                                     C.c_char_p, C.c_int64, C.c_int, C.c_int32, C.c_char_p, C.c_int64]
        L.dkr_keyset_new.restype = C.c_void_p
        L.dkr_keyset_free.argtypes = [C.c_void_p]
        L.dkr_keyset_or.argtypes = [C.c_void_p, C.c_char_p, C.c_int64, C.c_int]
        L.dkr_keyset_get.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
        P = C.c_void_p
        L.dkr_probe_checkpoint.argtypes = [P, C.c_int64, P, P, P, P, P, P, P, P, P, P, C.c_int, P, P, P]
        L.dkr_skip_eval.restype = C.c_int64
        L.dkr_skip_eval.argtypes = [P, P, P, C.c_int, P, P, C.c_int64, C.c_char_p, C.c_int64, C.c_int, P, C.c_int]
        _lib = L
    return _lib


class _Col(C.Structure):
    _fields_ = [("n_rows", C.c_int64), ("n_entries", C.c_int64), ("n_chars", C.c_int64),
                ("phys", C.c_int32), ("width", C.c_int32), ("max_def", C.c_int32),
                ("max_rep", C.c_int32), ("rep_def", C.c_int32), ("_pad", C.c_int32),
                ("row_def", C.c_void_p), ("row_offs", C.c_void_p), ("entry_def", C.c_void_p),
                ("fixed", C.c_void_p), ("offs", C.c_void_p), ("chars", C.c_void_p)]


def _np(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    itemsize = np.dtype(dtype).itemsize
    return np.frombuffer(C.string_at(ptr, n * itemsize), dtype=dtype).copy()


@dataclass
class Column:
    """Assembled leaf column (same layout the product's dk_column uses)."""
    path: str
    phys: int
    max_def: int
    max_rep: int
    rep_def: int
    n_rows: int
    row_def: np.ndarray
    row_offs: np.ndarray | None = None
    entry_def: np.ndarray | None = None
    fixed: np.ndarray | None = None   # raw bytes (n * width)
    width: int = 0
    offs: np.ndarray | None = None
    chars: np.ndarray | None = None

    def values(self, dtype):
        return self.fixed.view(dtype)

    def string(self, i):
        return bytes(self.chars[self.offs[i]:self.offs[i + 1]])


class ParquetFile:
    PHYS = {0: "BOOLEAN", 1: "INT32", 2: "INT64", 3: "INT96", 4: "FLOAT", 5: "DOUBLE",
            6: "BYTE_ARRAY", 7: "FIXED_LEN_BYTE_ARRAY"}

    def __init__(self, data):
        import mmap
        if isinstance(data, mmap.mmap):
            # a private mapping of the file: the page cache is shared, nothing is copied
            self._mm = data
            self._buf = (C.c_char * len(data)).from_buffer(data)
        else:
            self._buf = C.create_string_buffer(data, len(data))
        self._h = lib().dkr_open(self._buf, len(data))
        if not self._h:
            raise OracleError(lib().dkr_errmsg().decode())
        self.num_rows = lib().dkr_num_rows(self._h)
        self.leaves = [lib().dkr_leaf_path(self._h, i).decode() for i in range(lib().dkr_num_leaves(self._h))]

    @classmethod
    def open(cls, path):
        import mmap
        with open(path, "rb") as f:
            if os.fstat(f.fileno()).st_size == 0:
                return cls(b"")
            return cls(mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_COPY))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().dkr_close(self._h)
            self._h = None

    def select_row_groups(self, keep):
        """Read only the row groups with keep[g] true (the reader's row-group filter)."""
        lib().dkr_select_row_groups(self._h, bytes(1 if k else 0 for k in keep))
        self.num_rows = lib().dkr_num_rows(self._h)

    def leaf_index(self, path):
        """Field matching by exact name, then case-insensitive (ParquetSchemaUtils.java:92-119)."""
        if path in self.leaves:
            return self.leaves.index(path)
        low = [p.lower() for p in self.leaves]
        if path.lower() in low:
            return low.index(path.lower())
        return -1

    def read(self, path) -> Column | None:
        i = self.leaf_index(path)
        if i < 0:
            return None
        c = _Col()
        if lib().dkr_read_leaf(self._h, i, C.byref(c)) != 0:
            raise OracleError("Error reading Parquet file: " + lib().dkr_errmsg().decode())
        try:
            n_val = c.n_entries if c.max_rep > 0 else c.n_rows
            col = Column(path=path, phys=c.phys, max_def=c.max_def, max_rep=c.max_rep,
                         rep_def=c.rep_def, n_rows=c.n_rows, width=c.width,
                         row_def=_np(c.row_def, c.n_rows, np.uint8))
            if c.max_rep > 0:
                col.row_offs = _np(c.row_offs, c.n_rows + 1, np.int64)
                col.entry_def = _np(c.entry_def, c.n_entries, np.uint8)
            if c.phys == 6:
                col.offs = _np(c.offs, n_val + 1, np.int64)
                col.chars = _np(c.chars, c.n_chars, np.uint8)
            else:
                col.fixed = _np(c.fixed, n_val * c.width, np.uint8)
            return col
        finally:
            lib().dkr_col_free(C.byref(c))


def java_utf8(b: bytes) -> bytes:
    out = C.create_string_buffer(len(b) * 3 + 8)
    n = lib().dkr_java_utf8(b, len(b), out, len(out))
    return out.raw[:n]


def action_key(path: bytes, dv) -> bytes:
    """dv: None or (storageType bytes, pathOrInlineDv bytes, offset int|None)."""
    cap = len(path) * 3 + 256 + (0 if dv is None else 3 * (len(dv[0]) + len(dv[1])) + 64)
    out = C.create_string_buffer(cap)
    if dv is None:
        n = lib().dkr_action_key(path, len(path), 0, None, 0, None, 0, 0, 0, out, cap)
    else:
        st, pid, off = dv
        n = lib().dkr_action_key(path, len(path), 1, st, len(st), pid, len(pid),
                                 0 if off is None else 1, 0 if off is None else off, out, cap)
    if n < 0:
        raise OracleError("java.net.URISyntaxException: " + path.decode("utf-8", "replace"))
    return out.raw[:n]


# --------------------------------------------------------------------------------------------
# Log segment (SnapshotManager / Checkpointer / LogSegment restated for the latest snapshot)
# --------------------------------------------------------------------------------------------
DELTA_RE = re.compile(r"^(\d{20})\.json$")
CLASSIC_RE = re.compile(r"^(\d{20})\.checkpoint\.parquet$")
MULTI_RE = re.compile(r"^(\d{20})\.checkpoint\.(\d{10})\.(\d{10})\.parquet$")
V2_RE = re.compile(r"^(\d{20})\.checkpoint\.([^.]+)\.(json|parquet)$")


@dataclass
class LogFile:
    path: str
    kind: str          # commit | classic | multipart | v2 | sidecar
    version: int
    part: int = 0
    num_parts: int = 0


@dataclass
class LogSegment:
    log_path: str
    version: int
    deltas: list
    checkpoints: list

    def all_files_reversed(self):
        """LogSegment.java:171-177: sorted by file name, descending."""
        return sorted(self.deltas + self.checkpoints, key=lambda f: os.path.basename(f.path), reverse=True)


def _classify(name, full):
    m = DELTA_RE.match(name)
    if m:
        return LogFile(full, "commit", int(m.group(1)))
    m = CLASSIC_RE.match(name)
    if m:
        return LogFile(full, "classic", int(m.group(1)))
    m = MULTI_RE.match(name)
    if m:
        return LogFile(full, "multipart", int(m.group(1)), int(m.group(2)), int(m.group(3)))
    m = V2_RE.match(name)
    if m:
        return LogFile(full, "v2", int(m.group(1)))
    return None


def load_log_segment(table_root: str) -> LogSegment:
    log = os.path.join(table_root, "_delta_log")
    files = []
    for name in os.listdir(log):
        f = _classify(name, os.path.join(log, name))
        if f:
            files.append(f)
    # complete checkpoints grouped by version (CheckpointInstance / Checkpointer.java:46-73)
    ck = {}
    for f in files:
        if f.kind in ("classic", "multipart", "v2"):
            ck.setdefault((f.version, f.kind, f.num_parts), []).append(f)
    complete = []
    for (v, kind, nparts), fs in ck.items():
        if kind == "multipart":
            if sorted(x.part for x in fs) == list(range(1, nparts + 1)):
                complete.append((v, kind, fs))
        else:
            complete.append((v, kind, fs[:1]))
    deltas = sorted([f for f in files if f.kind == "commit"], key=lambda f: f.version)
    if not deltas and not complete:
        raise OracleError("No delta files found in the directory: " + log)
    latest = max([d.version for d in deltas] + [c[0] for c in complete])
    cks = [c for c in complete if c[0] <= latest]
    # preference at equal version: v2 > multipart(more parts) > classic (CheckpointInstance.compareTo)
    rank = {"classic": 0, "multipart": 1, "v2": 2}
    ckpt = max(cks, key=lambda c: (c[0], rank[c[1]], len(c[2])), default=None)
    ck_version = ckpt[0] if ckpt else -1
    tail = [d for d in deltas if d.version > ck_version]
    expect = ck_version + 1
    for d in tail:
        if d.version != expect:
            raise OracleError("Versions are not contiguous")
        expect += 1
    if ckpt is None and (not tail or tail[0].version != 0):
        raise OracleError("Cannot compute snapshot. Missing delta file version 0.")
    version = tail[-1].version if tail else ck_version
    return LogSegment(log, version, tail, list(ckpt[2]) if ckpt else [])


# --------------------------------------------------------------------------------------------
# JSON decode (DefaultJsonRow semantics for the add/remove read schema)
# --------------------------------------------------------------------------------------------
def _is_long(v):
    return isinstance(v, int) and not isinstance(v, bool) and -(1 << 63) <= v < (1 << 63)


def _is_int(v):
    return isinstance(v, int) and not isinstance(v, bool) and -(1 << 31) <= v < (1 << 31)


def _dec(node, typ, name):
    if node is None:
        return None
    if typ == "string":
        if not isinstance(node, str):
            raise OracleError("Couldn't decode %r, expected a string" % (node,))
        return node
    if typ == "long":
        if not _is_long(node):
            raise OracleError("Couldn't decode %r, expected a long" % (node,))
        return node
    if typ == "int":
        if not _is_int(node):
            raise OracleError("Couldn't decode %r, expected a integer" % (node,))
        return node
    if typ == "boolean":
        if not isinstance(node, bool):
            raise OracleError("Couldn't decode %r, expected a boolean" % (node,))
        return node
    if typ == "map":
        if not isinstance(node, dict):
            raise OracleError("Couldn't decode %r, expected a map" % (node,))
        return [(k, _dec(v, "string", k)) for k, v in node.items()]
    if isinstance(typ, list):
        if not isinstance(node, dict):
            raise OracleError("Couldn't decode %r, expected a object" % (node,))
        return _dec_struct(node, typ)
    raise OracleError("unsupported type " + str(typ))


def _dec_struct(obj, schema):
    out = {}
    for name, typ, nullable in schema:
        v = obj.get(name)
        if v is None:
            if not nullable:
                raise OracleError("Root node at key %s is null but field isn't nullable. Root node: %s"
                                  % (name, json.dumps(obj)))
            out[name] = None
        else:
            out[name] = _dec(v, typ, name)
    return out


DV_SCHEMA = [("storageType", "string", False), ("pathOrInlineDv", "string", False),
             ("offset", "int", True), ("sizeInBytes", "int", False), ("cardinality", "long", False)]
ADD_SCHEMA = [("path", "string", False), ("partitionValues", "map", False), ("size", "long", False),
              ("modificationTime", "long", False), ("dataChange", "boolean", False),
              ("deletionVector", DV_SCHEMA, True), ("tags", "map", True), ("baseRowId", "long", True),
              ("defaultRowCommitVersion", "long", True)]
ADD_SCHEMA_STATS = ADD_SCHEMA + [("stats", "string", True)]
REMOVE_SCHEMA = [("path", "string", False), ("deletionVector", DV_SCHEMA, True)]
SIDECAR_SCHEMA = [("path", "string", False), ("sizeInBytes", "long", False),
                  ("modificationTime", "long", False)]


def read_json_batches(path, batch_size, with_stats=False, sidecars=False):
    """Yields lists of rows {'add':..., 'remove':...} of at most batch_size lines of this file."""
    add_s = ADD_SCHEMA_STATS if with_stats else ADD_SCHEMA
    schema = [("add", add_s, True), ("remove", REMOVE_SCHEMA, True)]
    if sidecars:
        schema.append(("sidecar", SIDECAR_SCHEMA, True))
    with open(path, "rb") as f:
        data = f.read().decode("utf-8", errors="replace")
    lines = data.splitlines()  # BufferedReader.readLine: \n, \r, \r\n
    batch = []
    for ln in lines:
        obj = json.loads(ln)
        batch.append(_dec_struct(obj, schema))
        if len(batch) == batch_size:
            yield batch
            batch = []
    if batch:
        yield batch


# --------------------------------------------------------------------------------------------
# Replay
# --------------------------------------------------------------------------------------------
ADD_LEAVES = ["add.path", "add.partitionValues.key_value.key", "add.partitionValues.key_value.value",
              "add.size", "add.modificationTime", "add.dataChange",
              "add.deletionVector.storageType", "add.deletionVector.pathOrInlineDv",
              "add.deletionVector.offset", "add.deletionVector.sizeInBytes",
              "add.deletionVector.cardinality", "add.tags.key_value.key", "add.tags.key_value.value",
              "add.baseRowId", "add.defaultRowCommitVersion"]
STATS_LEAF = "add.stats"
SIDECAR_LEAVES = ["sidecar.path", "sidecar.sizeInBytes", "sidecar.modificationTime"]


@dataclass
class Counters:
    addFilesSeen: int = 0
    addFilesSeenFromDeltaFiles: int = 0
    activeAddFiles: int = 0
    duplicateAddFiles: int = 0
    removeFilesSeenFromDeltaFiles: int = 0

    def as_tuple(self):
        return (self.addFilesSeen, self.addFilesSeenFromDeltaFiles, self.activeAddFiles,
                self.duplicateAddFiles, self.removeFilesSeenFromDeltaFiles)


# java.net.URI (multi-argument constructors) path-component quoting: the ASCII characters left as
# they are -- unreserved (alphanum "_-!.~'()*"), punct (",;:$&+="), "/" and "@" (URI.java L_PATH /
# H_PATH); every other ASCII character, '%' included, is quoted.
_URI_PATH_LEGAL = set(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_-!.~'()*,;:$&+=/@")


def table_root_uri(table_root: str) -> str:
    """dataPath.toUri().toString() for a local table (ActiveAddFilesIterator.java:251).

    Table.forPath -> DefaultFileSystemClient.resolvePath (DefaultFileSystemClient.java:82-86):
    fs.makeQualified(new Path(p)).toString() on the local file system is "file:" + the absolute,
    normalized path (Path.normalizePath: no "//", no trailing "/"; relative paths against the
    working directory), unquoted. TableImpl wraps it in a Path again (TableImpl.java:81-85), whose
    URI comes from new URI(scheme, authority, path, null, fragment), and toUri().toString() prints
    the quoted form: an ASCII byte outside _URI_PATH_LEGAL becomes %XX (upper-case); a non-ASCII
    character is kept unless Character.isSpaceChar or isISOControl, in which case its UTF-8 bytes
    are %XX-encoded (URI.quote)."""
    import unicodedata
    parts = [x for x in os.path.abspath(table_root).split("/") if x not in ("", ".")]
    norm = "/" + "/".join(parts)
    out = []
    for ch in norm:
        o = ord(ch)
        if o < 0x80:
            out.append(ch if o in _URI_PATH_LEGAL else "%" + format(o, "02X"))
        elif 0x80 <= o <= 0x9F or unicodedata.category(ch) in ("Zs", "Zl", "Zp"):
            out.append("".join("%" + format(b, "02X") for b in ch.encode("utf-8", "surrogatepass")))
        else:
            out.append(ch)
    return "file:" + "".join(out)


@dataclass
class CheckpointBatch:
    """One decoded checkpoint / sidecar file (all rows) with its selection."""
    path: str
    cols: dict
    n_rows: int
    selected: np.ndarray = None
    file_index: int = 0          # position among the checkpoint files in replay order
    skipped: bool = False        # data skipping already applied to `selected`


@dataclass
class ReplayResult:
    version: int
    json_rows: list = field(default_factory=list)      # selected add dicts, in order
    checkpoint: list = field(default_factory=list)     # CheckpointBatch in order
    counters: Counters = field(default_factory=Counters)
    table_root: str = ""
    tail_counters: Counters = field(default_factory=Counters)   # commit-tail part of `counters`
    ckpt_counters: Counters = field(default_factory=Counters)   # checkpoint part (this shard's)

    def scan_files(self):
        """Ordered scan-file rows (App. B ordering): the add struct as canonical python tuples plus
        the tableRoot column (InternalScanFileUtils.SCAN_FILE_SCHEMA, ordinal 1)."""
        root = (self.table_root,)
        out = [canon_add_from_json(r) + root for r in self.json_rows]
        for b in self.checkpoint:
            idx = np.nonzero(b.selected)[0]
            out.extend(canon_add_from_cols(b.cols, int(i)) + root for i in idx)
        return out


def _dv_tuple(dv):
    if dv is None:
        return None
    return (dv["storageType"].encode(), dv["pathOrInlineDv"].encode(), dv["offset"])


def json_key(action):
    return action_key(action["path"].encode("utf-8", "surrogatepass"), _dv_tuple(action["deletionVector"]))


def canon_add_from_json(a):
    dv = a["deletionVector"]
    return (a["path"].encode("utf-8", "surrogatepass"),
            tuple((k.encode(), None if v is None else v.encode()) for k, v in a["partitionValues"]),
            a["size"], a["modificationTime"], a["dataChange"],
            None if dv is None else (dv["storageType"].encode(), dv["pathOrInlineDv"].encode(), dv["offset"],
                                     dv["sizeInBytes"], dv["cardinality"]),
            None if a["tags"] is None else tuple((k.encode(), None if v is None else v.encode()) for k, v in a["tags"]),
            a["baseRowId"], a["defaultRowCommitVersion"]) + ((a["stats"].encode() if a["stats"] is not None else None,) if "stats" in a else ())


def _str_at(col, r, maxdef):
    if col is None or col.row_def[r] < maxdef:
        return None
    return col.string(r)


def _fixed_at(col, r, dtype):
    if col is None or col.row_def[r] < col.max_def:
        return None
    w = np.dtype(dtype).itemsize
    return col.fixed[r * w:(r + 1) * w].view(dtype)[0].item()


def _map_at(kc, vc, r):
    if kc is None:
        return None
    if kc.row_def[r] < kc.rep_def - 1:
        return None
    b, e = kc.row_offs[r], kc.row_offs[r + 1]
    out = []
    for j in range(b, e):
        k = bytes(kc.chars[kc.offs[j]:kc.offs[j + 1]])
        v = None
        if vc is not None and vc.entry_def[j] == vc.max_def:
            v = bytes(vc.chars[vc.offs[j]:vc.offs[j + 1]])
        out.append((k, v))
    return tuple(out)


def canon_add_from_cols(cols, r):
    g = cols.get
    dvst = g("add.deletionVector.storageType")
    dv = None
    if dvst is not None and dvst.row_def[r] >= 2:
        pid = g("add.deletionVector.pathOrInlineDv")
        dv = (_str_at(dvst, r, dvst.max_def), _str_at(pid, r, pid.max_def if pid is not None else 0),
              _fixed_at(g("add.deletionVector.offset"), r, np.int32),
              _fixed_at(g("add.deletionVector.sizeInBytes"), r, np.int32),
              _fixed_at(g("add.deletionVector.cardinality"), r, np.int64))
    dc = g("add.dataChange")
    pc = g("add.path")
    # levels from the file: Spark writes every checkpoint field optional (add.path max_def 2), Kernel's
    # writer marks path / size / ... required (max_def 1, AddFile.FULL_SCHEMA)
    row = (_str_at(pc, r, pc.max_def if pc is not None else 0),
           _map_at(g("add.partitionValues.key_value.key"), g("add.partitionValues.key_value.value"), r),
           _fixed_at(g("add.size"), r, np.int64), _fixed_at(g("add.modificationTime"), r, np.int64),
           None if dc is None or dc.row_def[r] < dc.max_def else bool(dc.fixed[r]),
           dv,
           _map_at(g("add.tags.key_value.key"), g("add.tags.key_value.value"), r),
           _fixed_at(g("add.baseRowId"), r, np.int64), _fixed_at(g("add.defaultRowCommitVersion"), r, np.int64))
    if STATS_LEAF in cols:
        sc = cols[STATS_LEAF]
        row = row + (_str_at(sc, r, sc.max_def if sc is not None else 0),)
    return row


def decode_checkpoint_file(path, with_stats=False, extra_leaves=(), keep=None):
    pf = ParquetFile.open(path)
    if keep is not None:
        pf.select_row_groups(keep)
    cols = {}
    for leaf in ADD_LEAVES + ([STATS_LEAF] if with_stats else []) + list(extra_leaves):
        cols[leaf] = pf.read(leaf)
    return pf, cols


def probe_checkpoint(cols, n_rows, keyset, counters: Counters):
    """Checkpoint-batch branch of ActiveAddFilesIterator.prepareNext (isFromCheckpoint=true)."""
    L = lib()
    path = cols["add.path"]
    sel = np.zeros(n_rows, dtype=np.uint8)
    cnt = np.zeros(5, dtype=np.int64)
    bad = np.zeros(1, dtype=np.int64)
    if path is None:
        return sel
    st = cols.get("add.deletionVector.storageType")
    pid = cols.get("add.deletionVector.pathOrInlineDv")
    off = cols.get("add.deletionVector.offset")

    def ptr(a):
        return None if a is None else a.ctypes.data

    if st is not None:
        offv = off.fixed.view(np.int32) if off is not None else np.zeros(n_rows, np.int32)
        offd = off.row_def if off is not None else np.zeros(n_rows, np.uint8)
        args = (ptr(st.row_def), ptr(st.offs), ptr(st.chars), ptr(pid.offs), ptr(pid.chars),
                ptr(offd), ptr(offv), off.max_def if off is not None else 3)
    else:
        args = (None, None, None, None, None, None, None, 3)
    rc = L.dkr_probe_checkpoint(keyset, n_rows, ptr(path.row_def), ptr(path.offs), ptr(path.chars),
                                *args, ptr(sel), ptr(cnt), ptr(bad))
    if rc != 0:
        raise OracleError("java.net.URISyntaxException at checkpoint row %d" % bad[0])
    counters.addFilesSeen += int(cnt[0])
    counters.activeAddFiles += int(cnt[4])
    counters.duplicateAddFiles += int(cnt[3])
    return sel


def replay(table_root: str, json_batch_size=1024, with_stats=False, shard=None, skipping=None,
           partition=None, threads=1, keep_cols=True, extra_leaves=()) -> ReplayResult:
    """getLatestSnapshot + getScanFiles restated; returns the ordered active scan files + counters.

    shard=(world, rank): reconcile only the checkpoint files whose replay-order index i has
    i % world == rank (every rank still reads the commit tail and any V2 manifest to discover
    sidecars); res.tail_counters / res.ckpt_counters hold the two parts of the counters.

    skipping=(predicate node, {stats path: type}): ScanImpl.applyDataSkipping on the reconciled
    rows (oracle/skipping.py); implies with_stats, leaves the counters unchanged.
    partition=(predicate, {lower name: (type, physical name)}): ScanImpl.applyPartitionPruning
    (oracle/partitions.py), applied before data skipping, on every add row of every batch.

    threads > 1: multi-part / classic checkpoint files are decoded and probed on a thread pool
    (the C decoder releases the GIL); a checkpoint file's selection depends only on the commit-tail
    key sets, which are final before any checkpoint file is read (App. A, R4), so the result is
    the sequential one. keep_cols=False drops each file's decoded columns after its probe (full-size
    runs); extra_leaves are decoded too (timing the whole projected read schema)."""
    if skipping is not None:
        with_stats = True
    world, rank = shard if shard else (1, 0)
    seg = load_log_segment(table_root)
    res = ReplayResult(version=seg.version, table_root=table_root_uri(table_root))
    c = res.tail_counters
    cc = res.ckpt_counters
    ckpt_idx = 0
    tomb = set()
    added = set()
    files = seg.all_files_reversed()
    tail_adds = []          # every add row of the tail's batches (partition filters see them all)
    queue = list(files)
    L = lib()
    keyset = None
    pool_items = []         # (file, replay-order index) decoded on the thread pool (threads > 1)
    while queue:
        f = queue.pop(0)
        if f.kind == "commit":
            for batch in read_json_batches(f.path, json_batch_size, with_stats):
                for row in batch:                                  # :164-183
                    rm = row["remove"]
                    if rm is None:
                        continue
                    tomb.add(json_key(rm))
                    c.removeFilesSeenFromDeltaFiles += 1
                for row in batch:                                  # :192-234
                    a = row["add"]
                    if a is None:
                        continue
                    tail_adds.append(a)
                    c.addFilesSeen += 1
                    c.addFilesSeenFromDeltaFiles += 1
                    k = json_key(a)
                    if k not in added:
                        added.add(k)
                        if k not in tomb:
                            res.json_rows.append(a)
                            c.activeAddFiles += 1
                    else:
                        c.duplicateAddFiles += 1
            continue
        # checkpoint files: JSON sets are final from here on (checkpoint files come last)
        if keyset is None:
            keyset = L.dkr_keyset_new()
            for k in added:
                L.dkr_keyset_or(keyset, k, len(k), 1)
            for k in tomb:
                L.dkr_keyset_or(keyset, k, len(k), 2)
        group = [f]
        if f.kind in ("multipart", "sidecar"):
            while queue and queue[0].kind == f.kind and queue[0].version == f.version:
                group.append(queue.pop(0))
        for g in group:
            idx = ckpt_idx
            ckpt_idx += 1
            mine = idx % world == rank
            if g.kind == "v2" and g.path.endswith(".json"):
                # V2 JSON manifest: rows are checkpoint rows (isFromCheckpoint=true)
                for batch in read_json_batches(g.path, json_batch_size, with_stats, sidecars=True):
                    for row in batch:
                        sc = row.get("sidecar")
                        if sc is not None:
                            queue.append(LogFile(os.path.join(seg.log_path, "_sidecars", sc["path"]),
                                                 "sidecar", g.version))
                        a = row["add"]
                        if a is None or not mine:
                            continue
                        tail_adds.append(a)
                        cc.addFilesSeen += 1
                        k = json_key(a)
                        if k in added:
                            cc.duplicateAddFiles += 1
                        elif k not in tomb:
                            res.json_rows.append(a)   # manifest rows precede sidecars
                            cc.activeAddFiles += 1
                continue
            if not mine and g.kind != "v2":
                continue
            if threads > 1 and g.kind in ("classic", "multipart", "sidecar") and partition is None:
                pool_items.append((g, idx))
                continue
            extra = tuple(SIDECAR_LEAVES if g.kind == "v2" else ()) + tuple(extra_leaves)
            keep = None
            if partition is not None and g.kind in ("multipart", "sidecar"):
                # the checkpoint predicate prunes row groups of parts and sidecars (oracle/rowgroups.py)
                from .rowgroups import surviving_row_groups
                keep = surviving_row_groups(g.path, *partition)
            pf, cols = decode_checkpoint_file(g.path, with_stats, extra, keep)
            if g.kind == "v2":
                sp = cols.get("sidecar.path")
                if sp is not None:
                    for r in range(pf.num_rows):
                        if sp.row_def[r] >= 2:
                            queue.append(LogFile(os.path.join(seg.log_path, "_sidecars",
                                                              sp.string(r).decode()), "sidecar", g.version))
            if not mine:
                continue
            b = CheckpointBatch(g.path, cols, pf.num_rows, file_index=idx)
            b.selected = probe_checkpoint(cols, pf.num_rows, keyset, cc)
            if skipping is not None and partition is None:
                _skip_file(b, cols, skipping)
            if not keep_cols:
                b.cols = {}
            res.checkpoint.append(b)
    if pool_items:
        import concurrent.futures as cf
        # tasks: whole files, or (keep_cols=False) runs of row groups so that a wide pool has work
        tasks = []
        n_rgs = [1 if keep_cols else lib().dkr_num_row_groups(ParquetFile.open(g.path)._h) for g, _ in pool_items]
        per = max(1, sum(n_rgs) // max(1, threads))          # row groups per task
        for (g, idx), n_rg in zip(pool_items, n_rgs):
            for r0 in range(0, n_rg, per):
                tasks.append((g, idx, None if per >= n_rg else [r0 <= r < r0 + per for r in range(n_rg)]))

        def work(item):
            g, idx, keep = item
            pf, cols = decode_checkpoint_file(g.path, with_stats, extra_leaves, keep)
            part = Counters()
            b = CheckpointBatch(g.path, cols, pf.num_rows, file_index=idx)
            b.selected = probe_checkpoint(cols, pf.num_rows, keyset, part)
            if skipping is not None:
                _skip_file(b, cols, skipping)
            if not keep_cols:
                b.cols = {}
            return b, part

        with cf.ThreadPoolExecutor(min(threads, len(tasks))) as ex:
            for b, part in ex.map(work, tasks):
                last = res.checkpoint[-1] if res.checkpoint else None
                if last is not None and last.file_index == b.file_index:     # the next run of row groups
                    last.selected = np.concatenate([last.selected, b.selected])
                    last.n_rows += b.n_rows
                else:
                    res.checkpoint.append(b)
                cc.addFilesSeen += part.addFilesSeen
                cc.activeAddFiles += part.activeAddFiles
                cc.duplicateAddFiles += part.duplicateAddFiles
        res.pool_tasks = len(tasks)
    if keyset is not None:
        L.dkr_keyset_free(keyset)
    res.counters = Counters(*[a + b for a, b in zip(c.as_tuple(), cc.as_tuple())])
    if partition is not None:
        from . import partitions as pp
        pred, fields = partition
        keep = {id(a): pp.evaluate(pred, pp.json_map(a), fields) is True for a in tail_adds}
        res.json_rows = [a for a in res.json_rows if keep[id(a)]]
        for b in res.checkpoint:
            kc, vc, pc = b.cols.get(ADD_LEAVES[1]), b.cols.get(ADD_LEAVES[2]), b.cols.get("add.path")
            for i in range(b.n_rows):
                if pc is None or pc.row_def[i] < 1:
                    continue                    # no add in this row: its map is null
                pv = _map_at(kc, vc, i) if kc is not None else None
                if pp.evaluate(pred, pv, fields) is not True:
                    b.selected[i] = False
    if skipping is not None:
        from . import skipping as sk
        node, types = skipping
        res.json_rows = [a for a in res.json_rows if sk.keep(a.get("stats"), node, types)]
        for b in res.checkpoint:
            if not b.skipped:
                _skip_file(b, b.cols, skipping)
    return res


def replay_tail_keyset(table_root: str, json_batch_size=1024, with_stats=False):
    """The commit-tail half of replay(): the JSON add (A) and tombstone (T) key sets that every
    checkpoint row is probed against (ActiveAddFilesIterator.java:164-234, App. A R2-R4), as a C
    keyset (flag 1 = in A, 2 = in T). The caller frees it with dkr_keyset_free."""
    seg = load_log_segment(table_root)
    tomb, added = set(), set()
    for f in seg.all_files_reversed():
        if f.kind != "commit":
            continue
        for batch in read_json_batches(f.path, json_batch_size, with_stats):
            for row in batch:
                if row["remove"] is not None:
                    tomb.add(json_key(row["remove"]))
            for row in batch:
                if row["add"] is not None:
                    added.add(json_key(row["add"]))
    L = lib()
    ks = L.dkr_keyset_new()
    for k in added:
        L.dkr_keyset_or(ks, k, len(k), 1)
    for k in tomb:
        L.dkr_keyset_or(ks, k, len(k), 2)
    return ks


def _skip_file(b, cols, skipping):
    """ScanImpl.applyDataSkipping over one checkpoint file's selected rows (oracle/skipping.py; the
    integral fast path in oracle/dk_skip.c)."""
    from . import skipping as sk
    node, types = skipping
    sk.apply_to_column(cols.get(STATS_LEAF), b.selected, node, types)
    b.skipped = True


def _pm_json_protocol(p):
    """Protocol.fromColumnVector over a commit-JSON protocol (Protocol.java:33-47): null feature
    lists read as empty; the versions are required ints."""
    for k in ("minReaderVersion", "minWriterVersion"):
        if not _is_int(p.get(k)):
            raise OracleError("protocol.%s: expected an int, got %r" % (k, p.get(k)))
    for k in ("readerFeatures", "writerFeatures"):
        if p.get(k) is not None:
            _json_str_array(p[k], "protocol." + k)
    return {"minReaderVersion": p["minReaderVersion"], "minWriterVersion": p["minWriterVersion"],
            "readerFeatures": list(p.get("readerFeatures") or []), "writerFeatures": list(p.get("writerFeatures") or [])}


def _json_str(v, what):
    """DefaultJsonRow StringType: a JSON string (isTextual)."""
    if not isinstance(v, str):
        raise OracleError("%s: expected a string, got %r" % (what, v))
    return v


def _json_str_array(v, what):
    """ArrayType(string, containsNull = false) (DefaultJsonRow.java:265-290)."""
    if not isinstance(v, list):
        raise OracleError("%s: expected an array" % what)
    if any(x is None for x in v):
        raise OracleError("%s: Array type expects no nulls as elements" % what)
    return [_json_str(x, what) for x in v]


def _json_str_map(v, what):
    """MapType(string, string, valueContainsNull = false) (DefaultJsonRow.java:298-320)."""
    if not isinstance(v, dict):
        raise OracleError("%s: expected a map" % what)
    if any(x is None for x in v.values()):
        raise OracleError("%s: Map type expects no nulls in values" % what)
    return {k: _json_str(x, what) for k, x in v.items()}


def _pm_json_metadata(m):
    """Metadata.fromColumnVector over a commit-JSON metaData (Metadata.java:35-72, Format.java:42-48)
    decoded with DefaultJsonRow's rules (DefaultJsonRow.java:136-357)."""
    for k in ("id", "format", "schemaString", "partitionColumns", "configuration"):
        if m.get(k) is None:
            raise OracleError("metaData.%s is required" % k)
    if m.get("createdTime") is not None and not _is_long(m["createdTime"]):
        raise OracleError("metaData.createdTime: expected a long")
    for k in ("id", "schemaString"):
        _json_str(m[k], "metaData." + k)
    for k in ("name", "description"):
        if m.get(k) is not None:
            _json_str(m[k], "metaData." + k)
    if not isinstance(m["format"], dict) or m["format"].get("provider") is None:
        raise OracleError("metaData.format.provider is required")
    _json_str(m["format"]["provider"], "format.provider")
    if m["format"].get("options") is not None:
        _json_str_map(m["format"]["options"], "format.options")
    _json_str_array(m["partitionColumns"], "metaData.partitionColumns")
    _json_str_map(m["configuration"], "metaData.configuration")
    fmt = m["format"]
    return {"id": m["id"], "name": m.get("name"), "description": m.get("description"),
            "format": {"provider": fmt.get("provider"), "options": dict(fmt.get("options") or {})},
            "schemaString": m["schemaString"], "partitionColumns": list(m["partitionColumns"]),
            "createdTime": m.get("createdTime"), "configuration": dict(m["configuration"])}


def _first_defined(col, min_def=1):
    idx = np.nonzero(col.row_def >= min_def)[0] if col is not None else []
    return int(idx[0]) if len(idx) else -1


def _list_value(col, r):
    if col is None or col.row_def[r] < col.rep_def - 1:
        return None
    a, b = int(col.row_offs[r]), int(col.row_offs[r + 1])
    return [bytes(col.chars[col.offs[i]:col.offs[i + 1]]).decode() if col.entry_def[i] >= col.max_def else None
            for i in range(a, b)]


def _map_value(kc, vc, r):
    pairs = _map_at(kc, vc, r)
    return None if pairs is None else {k.decode(): (None if v is None else v.decode()) for k, v in pairs}


def _scalar(pf, leaf, r, dtype=None):
    c = pf.read(leaf)
    if c is None or c.row_def[r] < c.max_def:
        return None
    if dtype is None:
        return bytes(c.chars[c.offs[r]:c.offs[r + 1]]).decode()
    w = np.dtype(dtype).itemsize
    return int(c.fixed[r * w:(r + 1) * w].view(dtype)[0])


SUPPORTED_READER_FEATURES = {"columnMapping", "deletionVectors", "timestampNtz", "typeWidening-preview",
                             "typeWidening", "vacuumProtocolCheck", "variantType", "variantType-preview",
                             "v2Checkpoint"}                 # TableFeatures.java:47-61


def validate_read_supported(prot, table_path, meta):
    """TableFeatures.validateReadSupportedTable (TableFeatures.java:76-98) with
    ColumnMapping.getColumnMappingMode (util/ColumnMapping.java:41-51,78-92)."""
    def cm_mode():
        v = (meta.get("configuration") or {}).get("delta.columnMapping.mode")
        if v is not None and v.lower() not in ("none", "id", "name"):
            raise OracleError("Invalid value for table property 'delta.columnMapping.mode': '%s'." % v)
    rv = prot["minReaderVersion"]
    if rv == 1:
        return
    if rv == 2:
        cm_mode()
        return
    if rv == 3:
        bad = set(prot["readerFeatures"]) - SUPPORTED_READER_FEATURES
        if bad:
            raise OracleError("Unsupported Delta reader features: table `%s` requires reader table features [%s]"
                              % (table_path, ", ".join(sorted(bad))))
        if "columnMapping" in prot["readerFeatures"]:
            cm_mode()
        return
    raise OracleError("Unsupported Delta protocol reader version: table `%s` requires reader version %d"
                      % (table_path, rv))


def _crc_file(path):
    """ChecksumReader.readChecksumFile (ChecksumReader.java:98-127): one row, non-null protocol and
    metadata, decodable -- else None."""
    try:
        with open(path, "rb") as fh:
            lines = fh.read().decode("utf-8", "replace").splitlines()
        if len(lines) != 1:
            return None
        obj = json.loads(lines[0])
        if obj.get("protocol") is None or obj.get("metadata") is None:
            return None
        return (int(os.path.basename(path).split(".")[0]), _pm_json_protocol(obj["protocol"]),
                _pm_json_metadata(obj["metadata"]))
    except Exception:
        return None


def crc_info(log_path, version, lower):
    """ChecksumReader.getCRCInfo (ChecksumReader.java:40-96)."""
    lower = min(lower, version)
    got = _crc_file(os.path.join(log_path, "%020d.crc" % version))
    if got is not None or version in (0, lower):
        return got
    cands = []
    for n in sorted(os.listdir(log_path)):
        if n < "%020d.crc" % lower or not re.fullmatch(r"\d+\.crc", n):
            continue
        if int(n.split(".")[0]) > version:
            break
        cands.append(n)
    return _crc_file(os.path.join(log_path, cands[-1])) if cands else None


def load_protocol_metadata(table_root: str, json_batch_size=1024, parquet_batch_size=1024):
    """``LogReplay.loadTableProtocolAndMetadata`` (internal/replay/LogReplay.java:220-314) behind
    ``maybeGetNewerSnapshotHintAndCurrentCrcInfo`` (:384-426) for a fresh table (no snapshot hint):
    the newest checksum file in [max(checkpoint version, version - 100, 0), version] is the hint; a
    hint at the snapshot version answers directly. Otherwise files newest first
    (``LogSegment.allLogFilesReversed``), batch by batch: the first non-null ``protocol`` row, then
    the first non-null ``metaData`` row; ``TableFeatures.validateReadSupportedTable`` runs only when
    the metadata is found with the protocol already known; after the commit at hint version + 1 the
    hint fills the rest. Returns (protocol dict, metadata dict, validated) -- every field of Protocol /
    Metadata -- with the checkpoint decoded by the C oracle."""
    seg = load_log_segment(table_root)
    ckv = max([f.version for f in seg.all_files_reversed() if f.kind != "commit"], default=0)
    hint = crc_info(os.path.join(table_root, "_delta_log"), seg.version, max(ckv, seg.version - 100, 0))
    if hint is not None and hint[0] == seg.version:
        return hint[1], hint[2], False
    st = {"p": None, "m": None}
    path = "file:" + os.path.abspath(table_root)

    def batch(prot, meta):
        if st["p"] is None and prot is not None:
            st["p"] = prot()
            if st["m"] is not None:
                return "done"
        if st["m"] is None and meta is not None:
            st["m"] = meta()
            if st["p"] is not None:
                validate_read_supported(st["p"], path, st["m"])
                return "validated"
        return None

    for f in seg.all_files_reversed():
        if hint is not None and f.version <= hint[0]:
            break
        if f.kind == "commit" or f.path.endswith(".json"):      # commits and V2 JSON manifests
            with open(f.path, "rb") as fh:
                lines = fh.read().decode("utf-8", "replace").splitlines()
            for b0 in range(0, len(lines), json_batch_size):
                objs = [json.loads(x) for x in lines[b0:b0 + json_batch_size] if x.strip()]
                po = next((o["protocol"] for o in objs if o.get("protocol") is not None), None)
                mo = next((o["metaData"] for o in objs if o.get("metaData") is not None), None)
                r = batch(None if po is None else (lambda po=po: _pm_json_protocol(po)),
                          None if mo is None else (lambda mo=mo: _pm_json_metadata(mo)))
                if r:
                    return st["p"], st["m"], r == "validated"
        else:
            pf = ParquetFile.open(f.path)
            rp = _first_defined(pf.read("protocol.minReaderVersion")) if st["p"] is None else -1
            rm = _first_defined(pf.read("metaData.id")) if st["m"] is None else -1

            def prot(r=rp):
                return {"minReaderVersion": _scalar(pf, "protocol.minReaderVersion", r, np.int32),
                        "minWriterVersion": _scalar(pf, "protocol.minWriterVersion", r, np.int32),
                        "readerFeatures": _list_value(pf.read("protocol.readerFeatures.list.element"), r) or [],
                        "writerFeatures": _list_value(pf.read("protocol.writerFeatures.list.element"), r) or []}

            def meta(r=rm):
                return {"id": _scalar(pf, "metaData.id", r), "name": _scalar(pf, "metaData.name", r),
                        "description": _scalar(pf, "metaData.description", r),
                        "format": {"provider": _scalar(pf, "metaData.format.provider", r),
                                   "options": _map_value(pf.read("metaData.format.options.key_value.key"),
                                                         pf.read("metaData.format.options.key_value.value"), r) or {}},
                        "schemaString": _scalar(pf, "metaData.schemaString", r),
                        "partitionColumns": _list_value(pf.read("metaData.partitionColumns.list.element"), r),
                        "createdTime": _scalar(pf, "metaData.createdTime", r, np.int64),
                        "configuration": _map_value(pf.read("metaData.configuration.key_value.key"),
                                                    pf.read("metaData.configuration.key_value.value"), r)}
            bp = rp // parquet_batch_size if rp >= 0 else None
            bm = rm // parquet_batch_size if rm >= 0 else None
            order = sorted({b for b in (bp, bm) if b is not None})
            for b in order:
                r = batch(prot if bp == b else None, meta if bm == b else None)
                if r:
                    return st["p"], st["m"], r == "validated"
        if hint is not None and f.kind == "commit" and f.version == hint[0] + 1:
            break
    if hint is not None:
        return st["p"] or hint[1], st["m"] or hint[2], False
    raise OracleError("No %s found at version %d" % ("protocol" if st["p"] is None else "metadata", seg.version))
