"""The C-ABI boundary (include/dkgpu.h) on the CPU: the library loads, exports every entry point
the header declares (the symbols a JNI / FFM binding would bind), and refuses to
run without a HIP device instead of falling back to the CPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(ROOT, "include", "dkgpu.h")) as f:
        text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    return sorted(set(re.findall(r"\b(dk_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = _declared()
    for must in ("dk_engine_create", "dk_parquet_open", "dk_parquet_open_rg", "dk_json_tail_parse",
                 "dk_replay_create", "dk_replay_run", "dk_replay_counters", "dk_replay_ckpt_selection_bits",
                 "dk_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from delta_amd import _lib
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(so, n)]
    assert not missing, missing
    assert set(_lib.EXPORTS) <= set(_declared()) | {"dk_debug_snap_stats"}


def test_no_cpu_fallback_without_a_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from delta_amd import kernel as K
    from delta_amd._lib import DkError
    with pytest.raises(DkError, match="no HIP device"):
        K.GpuEngine()


def test_footer_only_entry_point_runs_on_the_host(tmp_path):
    """dk_parquet_row_groups reads a footer without touching a device."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from delta_amd import kernel as K
    p = str(tmp_path / "x.parquet")
    pq.write_table(pa.table({"a": list(range(10))}), p, row_group_size=4)
    assert K.row_group_rows(p) == [4, 4, 2]
