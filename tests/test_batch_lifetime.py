"""Scan-file batches outlive their iterator and their scan (FilteredColumnarBatch semantics of the
reference: ScanImpl.getScanFiles' batches are plain objects the caller keeps). The product hands out
zero-copy views of pinned blocks the library recycles on a rerun and frees on close; a batch still
referenced then gets its own copies (GpuScan._detach_batches)."""
import gc

import numpy as np
import pytest

from delta_amd import synth


@pytest.mark.gpu
def test_batches_survive_rerun_and_close(tmp_path):
    from delta_amd import kernel as K
    from oracle import ref
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=30_000, n_parts=4, n_commits=5, dv_frac=0.1))
    eng = K.GpuEngine()
    snap = K.Table.forPath(eng, str(tmp_path)).getLatestSnapshot(eng)
    scan = snap.getScanBuilder().build()
    first = list(scan.getScanFiles(eng))
    ckpt = [b for b in first if b.file_index >= 0]
    assert len(ckpt) == 4
    # one leaf read now (its mirror is a zero-copy view), the others only after close
    sizes = [b.data["add.size"].fixed.copy() for b in ckpt]
    sels = [None if b.selection is None else b.selection.copy() for b in ckpt]
    second = list(scan.getScanFiles(eng))              # a rerun: recycles the pinned blocks
    assert len(second) == len(first)
    del second
    gc.collect()
    scan.close()
    gc.collect()
    for b, sz, sl in zip(ckpt, sizes, sels):
        assert np.array_equal(b.data["add.size"].fixed, sz)
        assert (b.selection is None and sl is None) or np.array_equal(b.selection, sl)
    full = ref.replay(str(tmp_path))
    rows = [ref.canon_add_from_cols(b.data, int(i)) + (b.table_root,) for b in first for i in b.selected_rows()]
    assert rows == full.scan_files()                   # every leaf, read after the scan closed
    eng.close()
