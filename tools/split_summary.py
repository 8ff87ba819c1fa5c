"""Summarise a rocprofv3 kernel-trace CSV: average duration per (kernel, grid size).
Usage: python tools/split_summary.py gpurun_out/<tag>/split/k_kernel_trace.csv [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 16
d = collections.defaultdict(list)
for r in rows:
    d[(r["Kernel_Name"].split("(")[0], r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]) / len(kv[1]))[:top]:
    print("  ", k, len(v), round(sum(v) / len(v) / 1000, 1), "us")
