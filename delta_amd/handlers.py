"""Engine plugin point 1 beyond the ParquetHandler: the JsonHandler.parseJson and
ExpressionHandler.getPredicateEvaluator hooks a stock ScanImpl calls for data skipping
(kernel-api/.../internal/ScanImpl.java:304-352), on the GPU through the C ABI
(dk_json_parse_stats / dk_parsed_stats_eval, include/dkgpu.h).

    parsed = GpuJsonHandler(engine).parseJson(statsVector, statsProgram, selection)
    newSel = GpuPredicateEvaluator(engine, statsProgram).eval(parsed, selection)

`statsProgram` is the planner's compiled data-skipping filter (delta_amd/skipping.compile_program:
the pruned stats schema's paths and types, and COALESCE(skip, true)'s postfix program), the pair
ScanImpl builds as prunedStatsSchema + filterToEval. The string vector is a Column (offs / chars /
row_def, e.g. a scan-file batch's add.stats) or a list of str / None.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dk_skip_program, lib


def _program(program):
    from . import skipping as sk
    return sk.pack(program, dk_skip_program)


def _strings(vec):
    """(offs int64[n + 1], chars uint8, isnull uint8[n]) of a string vector."""
    if isinstance(vec, (list, tuple)):
        enc = [b"" if s is None else (s.encode("utf-8", "surrogatepass") if isinstance(s, str) else bytes(s))
               for s in vec]
        offs = np.zeros(len(enc) + 1, np.int64)
        offs[1:] = np.cumsum([len(e) for e in enc]) if enc else []
        chars = np.frombuffer(b"".join(enc) + b"\0" * 16, np.uint8).copy()
        isnull = np.array([s is None for s in vec], np.uint8)
        return offs, chars, isnull
    n = vec.n_rows
    offs = np.ascontiguousarray(vec.offs[:n + 1], dtype=np.int64)
    chars = np.concatenate([np.asarray(vec.chars, np.uint8), np.zeros(16, np.uint8)])
    isnull = (np.asarray(vec.row_def[:n]) < vec.max_def).astype(np.uint8)
    return offs, chars, isnull


class ParsedStats:
    """JsonHandler.parseJson's result: one row per input string, null where unselected / null."""

    def __init__(self, handle, n, n_paths):
        self._h = handle
        self.n = n
        self.n_paths = n_paths

    def column(self, path_index):
        """(values int64[n], present bool[n]) of stats path `path_index` (dk_parsed_stats_column)."""
        vals = np.zeros(max(1, self.n), np.int64)
        pres = np.zeros(max(1, self.n), np.uint8)
        check(lib().dk_parsed_stats_column(self._h, path_index, vals.ctypes.data, pres.ctypes.data))
        return vals[:self.n], pres[:self.n].astype(bool)

    def close(self):
        if self._h:
            lib().dk_parsed_stats_free(self._h)
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

    def parseJson(self, json_vector, stats_program, selection=None):
        offs, chars, isnull = _strings(json_vector)
        n = len(offs) - 1
        sel = None if selection is None else np.ascontiguousarray(selection, dtype=np.uint8)
        prog = _program(stats_program)
        h = C.c_void_p()
        check(lib().dk_json_parse_stats(self.engine._h, C.byref(prog), n, offs.ctypes.data, chars.ctypes.data,
                                        isnull.ctypes.data, None if sel is None else sel.ctypes.data, 0, C.byref(h)))
        return ParsedStats(h, n, prog.n_paths)


class GpuPredicateEvaluator:
    """ExpressionHandler.getPredicateEvaluator(prunedStatsSchema, COALESCE(skip, true))
    (kernel-api/.../engine/ExpressionHandler.java:58): eval(parsed, selection) -> new selection,
    the existing selection ANDed in (DefaultPredicateEvaluator.java:42-72)."""

    def __init__(self, engine, stats_program):
        self.engine = engine
        self._prog = _program(stats_program)

    def eval(self, parsed: ParsedStats, selection=None):
        sel = np.ones(parsed.n, np.uint8) if selection is None else np.array(selection, dtype=np.uint8, copy=True)
        check(lib().dk_parsed_stats_eval(parsed._h, C.byref(self._prog), sel.ctypes.data if parsed.n else None))
        return sel.astype(bool)
