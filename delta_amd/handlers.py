"""Engine plugin point 1 beyond the ParquetHandler: the JsonHandler.parseJson and
ExpressionHandler.getPredicateEvaluator hooks a stock ScanImpl calls for data skipping
(kernel-api/.../internal/ScanImpl.java:304-352), on the GPU through the C ABI (dk_json_parse /
dk_parsed_column_get / dk_parsed_eval, dk_skip_compile; include/dkgpu.h).

    batch = GpuJsonHandler(engine).parseJson(statsVector, prunedStatsSchema, selection)
    newSel = GpuExpressionHandler(engine).getPredicateEvaluator(prunedStatsSchema, filterToEval).eval(batch, selection)

`prunedStatsSchema` is Kernel StructType JSON (a str or a dict), `filterToEval` the predicate as
ScanImpl builds it (=(COALESCE(skip, true), ALWAYS_TRUE)) in the ABI's predicate JSON (a str or a
dict; delta_amd/programs.py writes it from skipping.construct's output). The string vector is a
Column (offs / chars / row_def, e.g. a scan-file batch's add.stats) or a list of str / None.
"""
from __future__ import annotations

import ctypes as C
import json
import struct
from decimal import Decimal

import numpy as np

from ._lib import check, dk_parsed_column, lib

TYPES = ["long", "integer", "short", "byte", "date", "string", "timestamp", "decimal", "timestamp_ntz",
         "float", "double"]


def _strings(vec):
    """(offs int64[n + 1], chars uint8, isnull uint8[n]) of a string vector."""
    if isinstance(vec, (list, tuple)):
        enc = [b"" if s is None else (s.encode("utf-8", "surrogatepass") if isinstance(s, str) else bytes(s))
               for s in vec]
        offs = np.zeros(len(enc) + 1, np.int64)
        offs[1:] = np.cumsum([len(e) for e in enc]) if enc else []
        chars = np.frombuffer(b"".join(enc) + b"\0", np.uint8).copy()
        isnull = np.array([s is None for s in vec], np.uint8)
        return offs, chars, isnull
    n = vec.n_rows
    offs = np.ascontiguousarray(vec.offs[:n + 1], dtype=np.int64)
    chars = np.ascontiguousarray(np.asarray(vec.chars, np.uint8))
    if not chars.size:
        chars = np.zeros(1, np.uint8)
    isnull = (np.asarray(vec.row_def[:n]) < vec.max_def).astype(np.uint8)
    return offs, chars, isnull


def _json_text(x):
    return x if isinstance(x, str) else json.dumps(x)


class ParsedBatch:
    """JsonHandler.parseJson's ColumnarBatch: one row per input string (null where unselected or
    null), one typed column per leaf of the output schema, in schema order."""

    def __init__(self, handle, n):
        self._h = handle
        self.n = n
        self.leaves = []
        for i in range(lib().dk_parsed_num_leaves(handle)):
            m = lib().dk_parsed_leaf_path(handle, i, None, 0)
            buf = C.create_string_buffer(m + 1)
            lib().dk_parsed_leaf_path(handle, i, buf, m + 1)
            self.leaves.append(tuple(json.loads(buf.raw[:m].decode("utf-8"))))

    def leaf_index(self, path):
        return self.leaves.index(tuple(path))

    def column(self, leaf):
        """dk_parsed_column_get of a leaf (index or path) as numpy arrays: type, valid (bool),
        values (int64), and for strings / decimals offs + chars, for decimals hi / scale / wide."""
        i = leaf if isinstance(leaf, int) else self.leaf_index(leaf)
        c = dk_parsed_column()
        check(lib().dk_parsed_column_get(self._h, i, C.byref(c)))
        n = self.n

        def arr(ptr, count, dt):
            if not ptr or count <= 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(count,)).copy()
        out = {"type": TYPES[c.type], "valid": arr(c.validity, n, np.uint8).astype(bool),
               "values": arr(c.values, n, np.int64)}
        if c.offs:
            offs = arr(c.offs, n + 1, np.int32)
            out["offs"] = offs
            out["chars"] = arr(c.chars, int(offs[-1]) if n else 0, np.uint8)
        if c.type == 7:
            out["hi"] = arr(c.values_hi, n, np.int64)
            out["scale"] = arr(c.scale, n, np.int32)
            out["wide"] = arr(c.wide, n, np.uint8).astype(bool)
        return out

    def values(self, leaf):
        """The leaf's values as Python objects (None where null): int (integral, date days,
        timestamp micros), bytes (strings, UTF-8), Decimal, float (float32 values for float)."""
        c = self.column(leaf)
        t = c["type"]
        out = []
        for r in range(self.n):
            if not c["valid"][r]:
                out.append(None)
            elif t == "string":
                out.append(bytes(c["chars"][c["offs"][r]:c["offs"][r + 1]]))
            elif t == "decimal":
                if c["wide"][r]:
                    out.append(Decimal(bytes(c["chars"][c["offs"][r]:c["offs"][r + 1]]).decode()))
                else:
                    u = (int(c["hi"][r]) << 64) | (int(c["values"][r]) & ((1 << 64) - 1))
                    digits = tuple(int(d) for d in str(abs(u)))     # exact: no context rounding
                    out.append(Decimal((1 if u < 0 else 0, digits, -int(c["scale"][r]))))
            elif t == "float":
                out.append(struct.unpack("<f", struct.pack("<I", int(c["values"][r]) & 0xffffffff))[0])
            elif t == "double":
                out.append(struct.unpack("<d", struct.pack("<q", int(c["values"][r])))[0])
            else:
                out.append(int(c["values"][r]))
        return out

    def close(self):
        if self._h:
            lib().dk_parsed_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GpuJsonHandler:
    """JsonHandler.parseJson (kernel-api/.../engine/JsonHandler.java:68-71) for stats strings."""

    def __init__(self, engine):
        self.engine = engine

    def parseJson(self, json_vector, output_schema, selection=None) -> ParsedBatch:
        offs, chars, isnull = _strings(json_vector)
        n = len(offs) - 1
        sel = None if selection is None else np.ascontiguousarray(selection, dtype=np.uint8)
        h = C.c_void_p()
        check(lib().dk_json_parse(self.engine._h, _json_text(output_schema).encode(), n, offs.ctypes.data,
                                  chars.ctypes.data, isnull.ctypes.data, None if sel is None else sel.ctypes.data, 0,
                                  C.byref(h)))
        return ParsedBatch(h, n)


class GpuPredicateEvaluator:
    """PredicateEvaluator over parsed stats: eval(batch, selection) -> new selection, the existing
    selection ANDed in (DefaultPredicateEvaluator.java:42-72)."""

    def __init__(self, engine, program):
        self.engine = engine
        self.program = program                     # a programs.Program (dk_skip_compile)

    def eval(self, parsed: ParsedBatch, selection=None):
        sel = np.ones(parsed.n, np.uint8) if selection is None else np.array(selection, dtype=np.uint8, copy=True)
        check(lib().dk_parsed_eval(parsed._h, self.program.handle, sel.ctypes.data if parsed.n else None))
        return sel.astype(bool)


class GpuExpressionHandler:
    """ExpressionHandler.getPredicateEvaluator(inputSchema, predicate) (kernel-api/.../engine/
    ExpressionHandler.java:58) for the data-skipping predicate ScanImpl evaluates over the parsed stats."""

    def __init__(self, engine):
        self.engine = engine

    def getPredicateEvaluator(self, input_schema, predicate) -> GpuPredicateEvaluator:
        from . import programs
        from .skipping import UnsupportedSkipping
        h = C.c_void_p()
        rc = lib().dk_skip_compile(_json_text(input_schema).encode(), _json_text(predicate).encode(), C.byref(h))
        if rc:
            programs._raise(rc, UnsupportedSkipping)
        return GpuPredicateEvaluator(self.engine, programs.Program(h))
