"""The asynchronous checkpoint open (dk_parquet_open_async, the default for plain scans): the
consumer takes the first files' batches while the later files still cross PCIe.

Its parity is the default GPU suite's (every plain scan runs through it). Here: an error in the
middle of the open's sliced loop (a test hook, DK_INJECT_SLICE_FAULT) reaches the consumer as an
error instead of leaving it waiting (a sticky fault made the polling loop spin and
every consumer block in wait_files), and DK_ASYNC_OPEN=0 gives the same answer as the default.
Each case runs in a child process (the switches are read once per process)."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _child(table, env):
    code = ("import sys, json; sys.path.insert(0, %r)\n"
            "from tests.parity_util import product_scan\n"
            "from delta_amd._lib import DkError\n"
            "try:\n"
            "    import hashlib\n"
            "    v, files, counters = product_scan(%r, 1024)[:3]\n"
            "    digest = hashlib.sha256(repr(files).encode()).hexdigest()\n"
            "    print(json.dumps({'ok': True, 'n': len(files), 'rows': digest, 'counters': list(counters)}))\n"
            "except DkError as e:\n"
            "    print(json.dumps({'ok': False, 'err': str(e)}))\n" % (ROOT, table))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_async_open_error_reaches_consumer(tmp_path):
    from delta_amd import synth
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=40_000, n_parts=6, compression="snappy", n_commits=4))
    got = _child(str(tmp_path), {"DK_INJECT_SLICE_FAULT": "0"})
    assert not got["ok"] and "injected fault in checkpoint open slice 0" in got["err"], got
    ok = _child(str(tmp_path), {})
    sync = _child(str(tmp_path), {"DK_ASYNC_OPEN": "0"})
    assert ok["ok"] and sync["ok"] and ok == sync          # the same rows (digest), counters
    import hashlib
    from tests.parity_util import oracle_scan
    v, files, counters = oracle_scan(str(tmp_path), 1024)
    assert ok["rows"] == hashlib.sha256(repr(files).encode()).hexdigest()
    assert tuple(ok["counters"]) == counters


def _early_close_child(table):
    """Close a scan right after its first checkpoint batch (the asynchronous open still reading and
    decoding), then scan again on the same engine: the closed open is released on the library's
    reaper thread while the next open allocates (a cache miss on the opener's thread
    used to wait for that very release)."""
    from delta_amd import kernel as K
    from tests.parity_util import assert_same, oracle_scan, product_scan
    eng = K.GpuEngine()
    for _ in range(3):
        snap = K.Table.forPath(eng, table).getLatestSnapshot(eng)
        scan = snap.getScanBuilder().build()
        it = iter(scan.getScanFiles(eng))
        first = next(it)
        while first.file_index < 0:               # past the commit tail: a checkpoint batch
            first = next(it)
        assert scan.ckpt.async_open
        scan.close()
    assert_same(product_scan(table, engine=eng), oracle_scan(table))
    eng.close()
    print("ok")


@pytest.mark.gpu
def test_async_open_early_close(tmp_path):
    from delta_amd import synth
    synth.write_table(str(tmp_path), synth.TableSpec(n_adds=200_000, n_parts=16, compression="snappy", n_commits=3))
    code = ("import sys; sys.path.insert(0, %r); from tests.test_async_open import _early_close_child; "
            "_early_close_child(%r)" % (ROOT, str(tmp_path)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]
