"""Summarise tools/pmc.sh output: per kernel, each counter averaged over the kernel's dispatches.

    python tools/pmc_summary.py gpurun_out/<tag>                      # table
    python tools/pmc_summary.py gpurun_out/<tag> --json OUT --rows N --compression none --profile NAME

--json writes the per-launch HBM traffic bench.py reports as roofline.traffic:
    bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced
reads (MI355X_MICROARCH.md, HBM), hence the factor 2 (an upper estimate for narrower loads).
"""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--json")
ap.add_argument("--rows", type=int)
ap.add_argument("--compression", default="none")
ap.add_argument("--profile", default="")
args = ap.parse_args()

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(args.root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("dk::", "").replace("void ", "")
        name = name.split("<")[0].replace("k_snap_frag_t", "k_snap_frag")      # template instances
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))

def big_mean(v):
    # the bench's full-size launches: the snapshot-load P&M pass launches the same kernels over a few
    # row groups; averaging those in would hide the per-step figure (HIP events time only the steps)
    top = max(v)
    big = [x for x in v if x >= 0.5 * top] or v
    return sum(big) / len(big)


mean = {k: {c: big_mean(v) for c, v in d.items()} for k, d in acc.items()}
names = sorted({c for d in mean.values() for c in d})
print("kernel".ljust(26), " ".join(n[:14].rjust(14) for n in names))
for k, d in sorted(mean.items()):
    print(k[:26].ljust(26), " ".join(("%.4g" % d[n]).rjust(14) if n in d else "-".rjust(14) for n in names))
if args.json:
    ker = {k: int((2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024) for k, d in mean.items()
           if "FETCH_SIZE" in d and "WRITE_SIZE" in d}
    entry = {"rows": args.rows, "compression": args.compression, "profile": args.profile,
             "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch, launches >= 50% of the largest",
             "kernels": ker}
    try:
        old = json.load(open(args.json))
        old = old if isinstance(old, list) else [old]
    except (OSError, ValueError):
        old = []
    old = [e for e in old if not (e.get("rows") == args.rows and e.get("compression") == args.compression)]
    with open(args.json, "w") as f:
        json.dump(old + [entry], f, indent=1, sort_keys=True)
    print("wrote", args.json)
