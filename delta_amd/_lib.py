"""ctypes binding of libdkgpu.so (include/dkgpu.h). The library is built in-tree by
delta_amd/build.py. There is no CPU fallback: if the library or a HIP device is missing, every
entry point raises."""
import ctypes as C
import os

import numpy as np


def put_bytes(obj, field, data: bytes):
    """Copy ``data`` into the char-array field of a ctypes structure byte for byte (an assignment
    ``obj.field = data`` stops at the first NUL byte)."""
    f = getattr(type(obj), field)
    if len(data) > f.size:
        raise ValueError("%s: %d bytes do not fit %d" % (field, len(data), f.size))
    C.memset(C.addressof(obj) + f.offset, 0, f.size)
    C.memmove(C.addressof(obj) + f.offset, data, len(data))

_HERE = os.path.dirname(os.path.abspath(__file__))
# DK_LIB_PATH: load another build of the same ABI (A/B of kernel variants; tools/build_variant.py)
LIB_PATH = os.environ.get("DK_LIB_PATH") or os.path.join(_HERE, "libdkgpu.so")
_lib = None


class DkError(RuntimeError):
    """Mirrors io.delta.kernel.exceptions.KernelEngineException for errors raised by the engine."""


class dk_config(C.Structure):
    _fields_ = [("parquet_batch_size", C.c_int32), ("json_batch_size", C.c_int32),
                ("device", C.c_int32), ("flags", C.c_int32)]


class dk_rg_filter(C.Structure):
    _fields_ = [("n_cols", C.c_int32), ("col_off", C.c_void_p), ("col_len", C.c_void_p), ("n_ops", C.c_int32),
                ("op", C.c_void_p), ("arg", C.c_void_p), ("lit", C.c_void_p), ("pool", C.c_void_p),
                ("pool_len", C.c_int64)]


class dk_column(C.Structure):
    _fields_ = [("n_rows", C.c_int64), ("n_entries", C.c_int64), ("n_chars", C.c_int64),
                ("phys", C.c_int32), ("width", C.c_int32), ("max_def", C.c_int32), ("max_rep", C.c_int32),
                ("rep_def", C.c_int32), ("present", C.c_int32),
                ("row_def", C.c_void_p), ("row_offs", C.c_void_p), ("entry_def", C.c_void_p),
                ("fixed", C.c_void_p), ("offs", C.c_void_p), ("chars", C.c_void_p)]


class dk_parsed_column(C.Structure):
    _fields_ = [("type", C.c_int32), ("n", C.c_int64), ("validity", C.c_void_p), ("values", C.c_void_p),
                ("values_hi", C.c_void_p), ("scale", C.c_void_p), ("wide", C.c_void_p), ("offs", C.c_void_p),
                ("chars", C.c_void_p)]


class dk_read_options(C.Structure):
    _fields_ = [("field_ids", C.c_void_p), ("predicate", C.c_void_p), ("row_index", C.c_int32),
                ("window_rows", C.c_int32)]


class dk_batch_column(C.Structure):
    _fields_ = [("present", C.c_int32), ("phys", C.c_int32), ("width", C.c_int32), ("max_def", C.c_int32),
                ("max_rep", C.c_int32), ("rep_def", C.c_int32), ("n_values", C.c_int64), ("value_offset", C.c_int64),
                ("row_def", C.c_void_p), ("row_offs", C.c_void_p), ("validity", C.c_void_p),
                ("entry_def", C.c_void_p), ("fixed", C.c_void_p), ("offs", C.c_void_p), ("chars", C.c_void_p)]


class dk_batch(C.Structure):
    _fields_ = [("file", C.c_int32), ("n_cols", C.c_int32), ("n_rows", C.c_int64),
                ("cols", C.POINTER(dk_batch_column)), ("row_index", C.c_void_p)]


class dk_dv_descriptor(C.Structure):
    _fields_ = [("storage_type", C.c_char_p), ("path_or_inline", C.c_char_p), ("has_offset", C.c_int32),
                ("offset", C.c_int32), ("size_in_bytes", C.c_int32), ("cardinality", C.c_int64)]


MAX_LEAF_DEPTH = 8

# dk_comm (include/dkgpu.h): the owner exchange's collectives behind the C ABI
COMM_ID_BYTES = 128
STATUS_PEER = 6
A2A_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), C.c_void_p, C.POINTER(C.c_int64))
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_int32, C.c_int32)


class dk_comm_callbacks(C.Structure):
    _fields_ = [("user", C.c_void_p), ("alltoallv", A2A_FN), ("allreduce_i64", ALLREDUCE_FN)]


_U = C.c_void_p
SIDE_FNS = [
    ("begin", C.CFUNCTYPE(C.c_int, _U)),
    ("tail_counts", C.CFUNCTYPE(C.c_int, _U, C.POINTER(C.c_int64), C.POINTER(C.c_int64))),
    ("tail_pack", C.CFUNCTYPE(C.c_int, _U, C.c_void_p, C.c_void_p)),
    ("tail_resolve", C.CFUNCTYPE(C.c_int, _U, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p,
                                 C.POINTER(C.c_int32))),
    ("reseed", C.CFUNCTYPE(C.c_int, _U)),
    ("tail_finish", C.CFUNCTYPE(C.c_int, _U, C.c_void_p)),
    ("run", C.CFUNCTYPE(C.c_int, _U)),
    ("ckpt_counts", C.CFUNCTYPE(C.c_int, _U, C.POINTER(C.c_int64))),
    ("ckpt_pack", C.CFUNCTYPE(C.c_int, _U, C.c_void_p)),
    ("ckpt_lookup", C.CFUNCTYPE(C.c_int, _U, C.c_void_p, C.c_int64, C.c_void_p)),
    ("ckpt_apply", C.CFUNCTYPE(C.c_int, _U, C.c_void_p)),
    ("cand_counts", C.CFUNCTYPE(C.c_int, _U, C.POINTER(C.c_int64), C.POINTER(C.c_int64))),
    ("cand_pack", C.CFUNCTYPE(C.c_int, _U, C.c_void_p, C.c_void_p)),
    ("cand_verify", C.CFUNCTYPE(C.c_int, _U, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p)),
    ("cand_finish", C.CFUNCTYPE(C.c_int, _U, C.c_void_p)),
]


class dk_owner_side(C.Structure):
    _fields_ = [("user", C.c_void_p), ("device_buffers", C.c_int32)] + SIDE_FNS

EXPORTS = ["dk_last_error", "dk_version", "dk_engine_create", "dk_engine_destroy", "dk_parquet_open",
           "dk_parquet_decode", "dk_parquet_sync", "dk_parquet_num_rows", "dk_parquet_column",
           "dk_parquet_first_row", "dk_parquet_column_rows",
           "dk_parquet_traffic", "dk_parquet_kernel_traffic", "dk_parquet_close", "dk_json_tail_parse", "dk_json_tail_rows",
           "dk_json_tail_parse_parts", "dk_json_tail_checkpoint_row0",
           "dk_replay_set_exchange", "dk_replay_exchange_counts", "dk_replay_exchange_pack", "dk_replay_exchange_filter",
           "dk_replay_exchange_finish", "dk_json_pm_decode",
           "dk_ckpt_writer_open", "dk_ckpt_writer_add_json", "dk_ckpt_writer_add_checkpoint_adds", "dk_ckpt_writer_close",
           "dk_json_tail_column", "dk_json_tail_free", "dk_replay_create", "dk_replay_set_skipping", "dk_replay_set_partition_filter", "dk_replay_run",
           "dk_replay_run_grouped", "dk_replay_wait_file", "dk_replay_prefetch_leaf", "dk_parquet_open_async",
           "dk_replay_sync",
           "dk_replay_counters", "dk_replay_counters_split", "dk_replay_json_selection", "dk_replay_ckpt_selection",
           "dk_replay_kernel_stats", "dk_replay_free", "dk_parquet_open_rg", "dk_parquet_row_groups",
           "dk_parquet_row_offset", "dk_replay_ckpt_selection_bits", "dk_parquet_open_sel",
           "dk_parquet_prune_row_groups", "dk_parquet_nonnull_row_groups",
           "dk_reader_open", "dk_reader_next", "dk_reader_num_rows", "dk_batch_release", "dk_reader_close",
           "dk_dv_load", "dk_dv_num_bits", "dk_dv_bitmap", "dk_dv_selection", "dk_dv_free", "dk_log_pm_scan",
           "dk_replay_stats_parsed_files", "dk_replay_ckpt_selection_bits_all",
           "dk_replay_ckpt_selection_host", "dk_parquet_open_ms", "dk_replay_attach_checkpoint",
           "dk_json_tail_file_steps", "dk_json_tail_file_row0", "dk_json_tail_rebase_steps", "dk_replay_set_owner", "dk_replay_owner_begin",
           "dk_replay_owner_tail_counts", "dk_replay_owner_tail_pack", "dk_replay_owner_tail_resolve",
           "dk_replay_owner_reseed", "dk_replay_owner_tail_finish", "dk_replay_owner_ckpt_counts",
           "dk_replay_owner_ckpt_pack", "dk_replay_owner_ckpt_lookup", "dk_replay_owner_ckpt_apply",
           "dk_replay_owner_cand_counts", "dk_replay_owner_cand_pack", "dk_replay_owner_cand_verify",
           "dk_replay_owner_cand_finish", "dk_skip_compile", "dk_part_compile", "dk_program_describe",
           "dk_program_free", "dk_json_parse", "dk_parsed_num_leaves", "dk_parsed_leaf_path", "dk_parsed_column_get",
           "dk_parsed_eval", "dk_parsed_free", "dk_comm_unique_id", "dk_comm_create", "dk_comm_create_callbacks",
           "dk_comm_create_local", "dk_comm_world", "dk_comm_rank", "dk_comm_allreduce_i64", "dk_comm_alltoallv",
           "dk_comm_abort", "dk_comm_last_run", "dk_comm_last_steps", "dk_comm_destroy", "dk_replay_owner_run", "dk_owner_protocol_run"]


def lib(build_if_missing=True):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not build_if_missing:
            raise DkError("libdkgpu.so is not built (run delta_amd/build.py)")
        from . import build
        build.build()
    L = C.CDLL(LIB_PATH)
    P, I32, I64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "dk_last_error": (C.c_char_p, []), "dk_version": (C.c_char_p, []),
        "dk_engine_create": (C.c_int, [C.POINTER(dk_config), C.POINTER(P)]),
        "dk_engine_destroy": (None, [P]),
        "dk_parquet_open": (C.c_int, [P, C.POINTER(C.c_char_p), I32, C.POINTER(C.c_char_p), I32, C.POINTER(P)]),
        "dk_parquet_open_rg": (C.c_int, [P, C.POINTER(C.c_char_p), I32, C.POINTER(C.c_char_p), I32, P, P,
                                         C.POINTER(P)]),
        "dk_parquet_row_groups": (C.c_int, [C.c_char_p, C.POINTER(I64), I32, C.POINTER(I32)]),
        "dk_parquet_open_sel": (C.c_int, [P, C.POINTER(C.c_char_p), I32, C.POINTER(C.c_char_p), I32, P, P,
                                          C.POINTER(P)]),
        "dk_parquet_prune_row_groups": (C.c_int, [C.c_char_p, P, P, I32, C.POINTER(I32)]),
        "dk_parquet_nonnull_row_groups": (C.c_int, [C.c_char_p, C.c_char_p, P, I32, C.POINTER(I32)]),
        "dk_parquet_row_offset": (I64, [P, I32]),
        "dk_replay_ckpt_selection_bits": (C.c_int, [P, I32, P, I64, I32]),
        "dk_replay_ckpt_selection_bits_all": (C.c_int, [P, P, P, I32]),
        "dk_replay_ckpt_selection_host": (C.c_int, [P, I32, C.POINTER(P)]),
        "dk_parquet_open_ms": (C.c_int, [P, C.POINTER(C.c_double)]),
        "dk_replay_attach_checkpoint": (C.c_int, [P, P]),
        "dk_parquet_decode": (C.c_int, [P]), "dk_parquet_sync": (C.c_int, [P]),
        "dk_parquet_num_rows": (I64, [P, I32]),
        "dk_parquet_column": (C.c_int, [P, I32, I32, C.POINTER(dk_column)]),
        "dk_parquet_first_row": (C.c_int, [P, I32, I32, I32, C.POINTER(I64)]),
        "dk_parquet_column_rows": (C.c_int, [P, I32, I32, I64, I64, C.POINTER(dk_column)]),
        "dk_parquet_traffic": (C.c_int, [P, C.POINTER(I64), C.POINTER(I64)]),
        "dk_parquet_kernel_traffic": (C.c_int, [P, C.c_char_p, C.POINTER(I64), C.POINTER(I64)]),
        "dk_parquet_close": (None, [P]),
        "dk_json_tail_parse": (C.c_int, [P, C.POINTER(C.c_char_p), C.POINTER(I64), I32, I32, C.POINTER(P)]),
        "dk_json_tail_rows": (I64, [P]),
        "dk_json_tail_parse_parts": (C.c_int, [P, C.POINTER(C.c_char_p), C.POINTER(I64), I32, I32, I32, C.POINTER(P)]),
        "dk_json_tail_checkpoint_row0": (I64, [P]),
        "dk_replay_set_exchange": (C.c_int, [P, I32, I32]),
        "dk_json_pm_decode": (C.c_int, [C.c_char_p, I64, I64, I32, C.c_char_p, I64, C.POINTER(I64)]),
        "dk_ckpt_writer_open": (C.c_int, [P, C.c_char_p, I32, C.POINTER(P)]),
        "dk_ckpt_writer_add_json": (C.c_int, [P, C.c_char_p, I64]),
        "dk_ckpt_writer_add_checkpoint_adds": (C.c_int, [P, P, I32, I64, I64, C.POINTER(I64)]),
        "dk_ckpt_writer_close": (C.c_int, [P, C.POINTER(I64), C.POINTER(I64)]),
        "dk_replay_exchange_counts": (C.c_int, [P, C.POINTER(I64)]),
        "dk_replay_exchange_pack": (C.c_int, [P, P]),
        "dk_replay_exchange_filter": (C.c_int, [P, P, I64, P]),
        "dk_replay_exchange_finish": (C.c_int, [P, P]),
        "dk_json_tail_column": (C.c_int, [P, C.c_char_p, C.POINTER(dk_column)]),
        "dk_json_tail_free": (None, [P]),
        "dk_replay_create": (C.c_int, [P, P, P, C.POINTER(P)]),
        "dk_replay_set_skipping": (C.c_int, [P, P]),
        "dk_replay_set_partition_filter": (C.c_int, [P, P]),
        "dk_replay_run": (C.c_int, [P]), "dk_replay_sync": (C.c_int, [P]),
        "dk_replay_run_grouped": (C.c_int, [P, C.c_int32]), "dk_replay_wait_file": (C.c_int, [P, C.c_int32]),
        "dk_replay_prefetch_leaf": (C.c_int, [P, C.c_char_p]),
        "dk_parquet_open_async": (C.c_int, [P, C.POINTER(C.c_char_p), I32, C.POINTER(C.c_char_p), I32, P, P, C.POINTER(P)]),
        "dk_replay_counters": (C.c_int, [P, C.POINTER(I64)]),
        "dk_replay_counters_split": (C.c_int, [P, C.POINTER(I64), C.POINTER(I64)]),
        "dk_replay_json_selection": (C.c_int, [P, P, I64]),
        "dk_replay_ckpt_selection": (C.c_int, [P, I32, P, I64]),
        "dk_replay_kernel_stats": (C.c_int, [P, I32, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(I64)]),
        "dk_replay_free": (None, [P]),
        "dk_reader_open": (C.c_int, [P, C.POINTER(C.c_char_p), I32, C.POINTER(C.c_char_p), I32,
                                     C.POINTER(dk_read_options), C.POINTER(P)]),
        "dk_reader_next": (C.c_int, [P, C.POINTER(C.POINTER(dk_batch))]),
        "dk_reader_num_rows": (I64, [P, I32]),
        "dk_batch_release": (None, [C.POINTER(dk_batch)]),
        "dk_reader_close": (None, [P]),
        "dk_dv_load": (C.c_int, [P, C.c_char_p, C.POINTER(dk_dv_descriptor), I32, C.POINTER(P)]),
        "dk_dv_num_bits": (I64, [P, I32]),
        "dk_dv_bitmap": (C.c_int, [P, I32, P, I64, I32]),
        "dk_dv_selection": (C.c_int, [P, I32, P, I64, P]),
        "dk_dv_free": (None, [P]),
        "dk_replay_stats_parsed_files": (C.c_int, [P]),
        "dk_log_pm_scan": (C.c_int, [C.POINTER(C.c_char_p), I32] + [C.POINTER(I64)] * 6 + [C.POINTER(I32)]),
        "dk_json_tail_file_steps": (C.c_int, [P, C.POINTER(I32)]),
        "dk_json_tail_file_row0": (C.c_int, [P, C.POINTER(I64)]),
        "dk_json_tail_rebase_steps": (C.c_int, [P, C.POINTER(I32)]),
        "dk_replay_set_owner": (C.c_int, [P, I32, I32]),
        "dk_replay_owner_begin": (C.c_int, [P]),
        "dk_replay_owner_tail_counts": (C.c_int, [P, C.POINTER(I64), C.POINTER(I64)]),
        "dk_replay_owner_tail_pack": (C.c_int, [P, P, P]),
        "dk_replay_owner_tail_resolve": (C.c_int, [P, P, I64, P, I64, P, C.POINTER(I32)]),
        "dk_replay_owner_reseed": (C.c_int, [P]),
        "dk_replay_owner_tail_finish": (C.c_int, [P, P]),
        "dk_replay_owner_ckpt_counts": (C.c_int, [P, C.POINTER(I64)]),
        "dk_replay_owner_ckpt_pack": (C.c_int, [P, P]),
        "dk_replay_owner_ckpt_lookup": (C.c_int, [P, P, I64, P]),
        "dk_replay_owner_ckpt_apply": (C.c_int, [P, P]),
        "dk_replay_owner_cand_counts": (C.c_int, [P, C.POINTER(I64), C.POINTER(I64)]),
        "dk_replay_owner_cand_pack": (C.c_int, [P, P, P]),
        "dk_replay_owner_cand_verify": (C.c_int, [P, P, I64, P, I64, P]),
        "dk_replay_owner_cand_finish": (C.c_int, [P, P]),
        "dk_skip_compile": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(P)]),
        "dk_part_compile": (C.c_int, [C.c_char_p, C.POINTER(P)]),
        "dk_program_describe": (I64, [P, C.c_char_p, I64]),
        "dk_program_free": (None, [P]),
        "dk_json_parse": (C.c_int, [P, C.c_char_p, I64, P, P, P, P, I32, C.POINTER(P)]),
        "dk_parsed_num_leaves": (I32, [P]),
        "dk_parsed_leaf_path": (I64, [P, I32, C.c_char_p, I64]),
        "dk_parsed_column_get": (C.c_int, [P, I32, C.POINTER(dk_parsed_column)]),
        "dk_parsed_eval": (C.c_int, [P, P, P]),
        "dk_parsed_free": (None, [P]),
        "dk_comm_unique_id": (C.c_int, [P]),
        "dk_comm_create": (C.c_int, [P, I32, I32, I32, C.POINTER(P)]),
        "dk_comm_create_callbacks": (C.c_int, [C.POINTER(dk_comm_callbacks), I32, I32, C.POINTER(P)]),
        "dk_comm_create_local": (C.c_int, [I32, I32, C.POINTER(P)]),
        "dk_comm_world": (I32, [P]), "dk_comm_rank": (I32, [P]),
        "dk_comm_allreduce_i64": (C.c_int, [P, C.POINTER(I64), I32, I32]),
        "dk_comm_alltoallv": (C.c_int, [P, P, C.POINTER(I64), P, C.POINTER(I64), I32]),
        "dk_comm_abort": (C.c_int, [P]),
        "dk_comm_last_run": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(I64), C.POINTER(I64)]),
        "dk_comm_last_steps": (C.c_int, [P, C.POINTER(C.c_double)]),
        "dk_comm_destroy": (None, [P]),
        "dk_replay_owner_run": (C.c_int, [P, P]),
        "dk_owner_protocol_run": (C.c_int, [C.POINTER(dk_owner_side), P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise DkError(lib().dk_last_error().decode("utf-8", "replace"))


def _arr(ptr, n, dtype):
    if not ptr or n <= 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,)).copy()


def _view(ptr, n, dtype):
    if not ptr or n <= 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,))


class Column:
    """A dk_column on the host (same field names as the oracle's Column, by design). copy=False
    wraps the library's pinned mirror without copying: valid until the owning set decodes again or
    closes (scan-file batches, consumed before their scan closes)."""

    def __init__(self, c: dk_column, path: str, copy: bool = True):
        _arr = globals()["_arr"] if copy else _view
        self.path = path
        self.present = bool(c.present)
        self.n_rows = c.n_rows
        self.phys, self.width, self.max_def, self.max_rep, self.rep_def = c.phys, c.width, c.max_def, c.max_rep, c.rep_def
        n_val = c.n_entries if c.max_rep > 0 else c.n_rows
        self.row_def = _arr(c.row_def, c.n_rows, np.uint8) if c.present else np.zeros(c.n_rows, np.uint8)
        self.row_offs = _arr(c.row_offs, c.n_rows + 1, np.int64) if c.max_rep > 0 else None
        self.entry_def = _arr(c.entry_def, n_val, np.uint8) if c.max_rep > 0 else None
        if c.present and c.phys == 6:
            self.offs = _arr(c.offs, n_val + 1, np.int64)
            self.chars = _arr(c.chars, c.n_chars, np.uint8)
            self.fixed = None
        elif c.present:
            self.fixed = _arr(c.fixed, n_val * c.width, np.uint8)
            self.offs = self.chars = None
        else:
            self.fixed = self.offs = self.chars = None

    def string(self, i):
        return bytes(self.chars[self.offs[i]:self.offs[i + 1]])

    def slice_rows(self, a, b):
        """Rows [a, b) as a column of their own (views; entry- and char-level arrays are shared:
        the row-level offsets keep pointing into them)."""
        import copy
        c = copy.copy(self)
        c.n_rows = b - a
        c.row_def = self.row_def[a:b]
        if self.max_rep > 0:
            c.row_offs = self.row_offs[a:b + 1]
        elif self.offs is not None:
            c.offs = self.offs[a:b + 1]
        elif self.fixed is not None:
            c.fixed = self.fixed[a * self.width:b * self.width]
        return c
