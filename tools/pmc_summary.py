"""Summarise tools/pmc.sh output: per kernel, the counters averaged per dispatch (FETCH_SIZE and
WRITE_SIZE in KB as rocprofv3 reports them). Usage: python tools/pmc_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in acc.values() for c in k})
print("kernel".ljust(28), " ".join(n[:14].rjust(14) for n in names))
for k, d in sorted(acc.items()):
    row = []
    for n in names:
        v = d.get(n)
        # each dispatch may report one value per (dimension) instance; sum per dispatch is not
        # recoverable here, so report the mean of all samples times samples-per-dispatch
        row.append(("%.4g" % (sum(v) / max(1, len(v)))).rjust(14) if v else "-".rjust(14))
    print(k[:28].ljust(28), " ".join(row))
