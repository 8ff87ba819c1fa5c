"""Bin a rocprofv3 kernel + memory-copy trace over one step's window (the [dk] open start on the same
CLOCK_MONOTONIC): per 10 ms bin, busy ms per kernel family and copy ms per direction.

    python tools/trace_window.py gpurun_out/<tag>/tr OPEN_START_MS [SPAN_MS]
"""
import collections
import csv
import glob
import sys

root, t0 = sys.argv[1], float(sys.argv[2]) * 1e6
span = float(sys.argv[3]) if len(sys.argv) > 3 else 210.0
BIN = 10.0
FAM = [("k_snap_frag", "frag"), ("k_snap_", "snapsz"), ("k_tile_decode", "tdec"), ("k_tile_", "tsz"),
       ("k_pos_", "pos"), ("k_string_copy", "scopy"), ("k_page_", "pghdr"), ("k_probe", "probe"),
       ("k_copy_zc", "zc"), ("k_json", "json"), ("k_table", "table")]
def fam(n):
    n = n.replace("void ", "").replace("dk::", "")
    for p, f in FAM:
        if n.startswith(p):
            return f
    return "other"
bins = collections.defaultdict(lambda: collections.defaultdict(float))
first = {}
def add(kind, s, e):
    s, e = (s - t0) / 1e6, (e - t0) / 1e6
    if e < 0 or s > span:
        return
    first.setdefault(kind, [s, e]); first[kind][0] = min(first[kind][0], s); first[kind][1] = max(first[kind][1], e)
    b = int(max(s, 0) // BIN)
    while b * BIN < e:
        lo, hi = max(s, b * BIN), min(e, (b + 1) * BIN)
        if hi > lo:
            bins[b][kind] += hi - lo
        b += 1
for f in glob.glob(root + "/*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        add(fam(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
for f in glob.glob(root + "/*memory_copy_trace.csv"):
    for r in csv.DictReader(open(f)):
        add("H2D" if "HOST_TO_DEVICE" in r["Direction"] else ("D2H" if "DEVICE_TO_HOST" in r["Direction"] else "D2D"),
            int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
kinds = sorted({k for b in bins.values() for k in b})
print("bin(ms)  " + " ".join(k.rjust(6) for k in kinds))
for b in sorted(bins):
    print(("%4d-%-4d" % (b * BIN, (b + 1) * BIN)) + " ".join(("%6.1f" % bins[b][k]) if bins[b][k] else "     ." for k in kinds))
print("first start / last end (ms):")
for k in kinds:
    print("  %-7s %7.1f %7.1f" % (k, first[k][0], first[k][1]))
