"""k_snap_link walk-length statistics (needs a DK_LINK_STATS build loaded via DK_LIB_PATH:
DK_VARIANT_FLAGS=-DDK_LINK_STATS python tools/build_variant.py variants/link_stats.so).
Usage: DK_LIB_PATH=variants/link_stats.so python tools/link_stats.py TABLE_DIR"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_amd import kernel as K  # noqa: E402
from delta_amd._lib import lib  # noqa: E402

NAMES = ["lanes", "merged", "tags", "max_tags", "gt16", "gt64", "gt256", "tags_gt64", "past_last_rec",
         "max_cycles", "sum_cycles", "short_walkers", "entry_past_end"]
eng = K.GpuEngine()
snap = K.Table.forPath(eng, sys.argv[1]).getLatestSnapshot(eng)
z = (C.c_int64 * 24)()
lib().dk_debug_snap_stats(z)
base = list(z)
scan = snap.getScanBuilder().build()
scan.prepare(eng)
scan.run(); scan.sync()
lib().dk_debug_snap_stats(z)
d = {n: z[i] - base[i] for i, n in enumerate(NAMES)}
d["max_tags"] = z[3]; d["max_cycles"] = z[9]
print(d)
n = max(1, d["lanes"])
print("merged %.3f  tags/lane %.2f  >16 %.4f  >64 %.4f  >256 %.4f  past-last-record %.4f  cycles/lane %.0f max %d"
      % (d["merged"] / n, d["tags"] / n, d["gt16"] / n, d["gt64"] / n, d["gt256"] / n, d["past_last_rec"] / n,
         d["sum_cycles"] / n, d["max_cycles"]))
