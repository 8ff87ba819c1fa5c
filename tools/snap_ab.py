"""Time k_snap_frag / k_snap_walk_link on one table for several configurations (A/B of snappy
variants), each in a subprocess. Arguments after TABLE: a library path (DK_LIB_PATH) or
"exp=<flags>" (DK_SNAP_EXP: a correct decode plus the experiment instance; compare with exp=16).
Usage: python tools/snap_ab.py TABLE [lib.so | exp=N] ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json
sys.path.insert(0, %r)
from delta_amd import kernel as K
eng = K.GpuEngine(timing=True)
snap = K.Table.forPath(eng, %r).getLatestSnapshot(eng)
scan = snap.getScanBuilder().build(); scan.prepare(eng)
scan.run(); scan.sync()
s0 = scan.kernel_stats()
for _ in range(3): scan.run(); scan.sync()
s1 = scan.kernel_stats()
out = {k: round((a1 * c1 - s0.get(k, (0, 0))[0] * s0.get(k, (0, 0))[1]) / (c1 - s0.get(k, (0, 0))[1]), 1)
       for k, (a1, c1) in s1.items() if c1 > s0.get(k, (0, 0))[1]}
print(json.dumps(out))
'''
table = sys.argv[1]
for so in sys.argv[2:]:
    if so.startswith("exp="):
        env = dict(os.environ, DK_SNAP_EXP=so[4:])
    else:
        env = dict(os.environ, DK_LIB_PATH=os.path.abspath(so))
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, table)], env=env, capture_output=True, text=True, timeout=300)
    try:
        d = json.loads(r.stdout.strip().splitlines()[-1])
        print("%-28s frag %9.1f  walk %8.1f  fix %7.1f  step %9.1f" % (os.path.basename(so), d.get("k_snap_frag", 0),
              d.get("k_snap_walk_link", 0), d.get("k_snap_fix", 0), d.get("step_total", 0)), flush=True)
    except Exception:
        print(os.path.basename(so), "failed", r.stderr[-500:], flush=True)
