"""k_snap_frag batch statistics on a bench table (needs a DK_SNAP_STATS build loaded via DK_LIB_PATH:
DK_VARIANT_FLAGS=-DDK_SNAP_STATS python tools/build_variant.py stats_lib/libdk_stats.so).
Usage: DK_LIB_PATH=build/libdk_stats.so python tools/snap_stats.py TABLE_DIR"""
import ctypes as C
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_amd import kernel as K  # noqa: E402
from delta_amd._lib import lib  # noqa: E402

NAMES = ["batches", "batch_tags", "dep_tags", "far_tags", "win_copies", "big_literals", "refills",
         "resolve_rounds", "sum_CH", "fragments", "ring_tags", "literal_tags", "cand_rounds",
         "cy_top", "cy_discovery", "cy_parse_scan", "cy_resolve", "cy_farq", "cy_bytes", "cy_dep", "cy_flush",
         "fix_corrections", "fix_cycles", "fix_correction_cycles"]
eng = K.GpuEngine()
snap = K.Table.forPath(eng, sys.argv[1]).getLatestSnapshot(eng)
scan = snap.getScanBuilder().build()
z = (C.c_int64 * 24)()
lib().dk_debug_snap_stats(z)
base = list(z)
scan.prepare(eng)          # the prepare pass decodes the snappy pages (the first run reuses them)
scan.run(); scan.sync()
lib().dk_debug_snap_stats(z)
d = {n: z[i] - base[i] for i, n in enumerate(NAMES)}
print(d)
b = max(1, d["batches"])
print("cycles per batch (per wave): " + "  ".join("%s %.0f" % (k[3:], d[k] / b) for k in NAMES if k.startswith("cy_")))
print("tags/batch %.1f  dep %.3f far %.3f win-copies %.3f ring %.3f lit %.3f  rounds/batch %.2f  CH %.2f  cand/batch %.2f"
      % (d["batch_tags"] / b, d["dep_tags"] / max(1, d["batch_tags"]), d["far_tags"] / max(1, d["batch_tags"]),
         d["win_copies"] / max(1, d["batch_tags"]), d["ring_tags"] / max(1, d["batch_tags"]),
         d["literal_tags"] / max(1, d["batch_tags"]), d["resolve_rounds"] / b, d["sum_CH"] / b, d["cand_rounds"] / b))
