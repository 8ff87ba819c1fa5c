"""bench.py's multi-rank path on the CPU: `python bench.py --gpus N --dry-run` must start N ranks by
itself (no torchrun, no WORLD_SIZE in the caller's environment), plan the checkpoint row groups with
the product's planner (delta_amd/shard.plan_units over footers read by libdkgpu's host parser) and
run the one-collective exchange (shard.SelectionExchange) over gloo; rank 0 checks that every
checkpoint row came back exactly once, in replay order."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launcher_reaches_world_n(tmp_path, n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run",
                          "--rows", "6400", "--workdir", str(tmp_path / "t")],
                         env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 prints exactly one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks"] == n and d["backend"] == "gloo"
    assert d["ok"] is True
    assert d["checkpoint_rows"] == 6402 and d["checkpoint_files"] == 64


def test_bench_refuses_world_mismatch(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run",
                          "--rows", "6400", "--workdir", str(tmp_path / "t")],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "--gpus 3 but WORLD_SIZE=2" in out.stderr
