"""Summarise tools/pmc.sh output: per kernel, each counter averaged over the kernel's dispatches.

    python tools/pmc_summary.py gpurun_out/<tag>                      # table
    python tools/pmc_summary.py gpurun_out/<tag> --json OUT --rows N --compression none --profile NAME

--json writes the per-launch HBM traffic bench.py reports as roofline.traffic:
    bytes = (FETCH_SIZE / fetch_ratio[width] + WRITE_SIZE / write_ratio[width]) * 1024
FETCH_SIZE / WRITE_SIZE are in KiB. The counters' ratio to the bytes moved depends on the access
width (MI355X_MICROARCH.md, HBM: exactly 1/2 for 16-byte-per-lane streaming reads; other widths
uncalibrated there), so each kernel is corrected by the ratio measured for its dominant access width
(tools/pmc_calib.sh on a known byte count, profiles/r03/pmc_calib.json). Kernels whose width is not
listed are reported raw (ratio 1) and marked so.
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
        name = name.split("<")[0].replace("k_snap_frag_t", "k_snap_frag")      # (round-4 profiles: a template)
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))

def big_mean(v):
    # the bench's full-size launches: the snapshot-load P&M pass launches the same kernels over a few
    # row groups; averaging those in would hide the per-step figure (HIP events time only the steps)
    top = max(v)
    big = [x for x in v if x >= 0.5 * top] or v
    return sum(big) / len(big)


mean = {k: {c: big_mean(v) for c, v in d.items()} for k, d in acc.items()}

# dominant global-load width per kernel (bytes per lane per load), from the kernel source
WIDTH = {"k_string_copy": 16, "k_pos_count": 16, "k_pos_verify": 16, "k_copy_zc": 16,
         "k_snap_walk": 16, "k_snap_walk_lds": 16, "k_snap_recheck": 4, "k_snap_link": 4, "k_snap_fix": 4, "k_snap_frag": 4, "k_tile_decode": 4,
         "k_tile_count": 4, "k_tile_chars": 4, "k_probe_fast_all": 8, "k_snappy_serial": 1}
CALIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r03", "pmc_calib.json")
try:
    cal = json.load(open(CALIB))           # {"fetch": {"16": r, "8": r, "4": r, "1": r}, "write": {...}}
except (OSError, ValueError):
    cal = {"fetch": {"16": 0.5}, "write": {"16": 1.0}}


def ratio(kind, kernel):
    w = WIDTH.get(kernel)
    r = cal[kind].get(str(w)) if w else None
    return (r, w) if r else (1.0, None)
names = sorted({c for d in mean.values() for c in d})
print("kernel".ljust(26), " ".join(n[:14].rjust(14) for n in names))
for k, d in sorted(mean.items()):
    print(k[:26].ljust(26), " ".join(("%.4g" % d[n]).rjust(14) if n in d else "-".rjust(14) for n in names))
if args.json:
    ker, raw, how = {}, {}, {}
    for k, d in mean.items():
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        fr, fw = ratio("fetch", k)
        wr, ww = ratio("write", k)
        ker[k] = int((d["FETCH_SIZE"] / fr + d["WRITE_SIZE"] / wr) * 1024)
        raw[k] = int((d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024)
        how[k] = "width %s B/lane: fetch / %.3f, write / %.3f" % (fw, fr, wr) if fw else "raw (width uncalibrated)"
    entry = {"rows": args.rows, "compression": args.compression, "profile": args.profile,
             "formula": "(FETCH_SIZE / fetch ratio + WRITE_SIZE / write ratio) * 1024 per launch, ratios per "
                        "access width from profiles/r03/pmc_calib.json; launches >= 50% of the largest",
             "kernels": ker, "kernels_raw": raw, "correction": how}
    try:
        old = json.load(open(args.json))
        old = old if isinstance(old, list) else [old]
    except (OSError, ValueError):
        old = []
    old = [e for e in old if not (e.get("rows") == args.rows and e.get("compression") == args.compression)]
    with open(args.json, "w") as f:
        json.dump(old + [entry], f, indent=1, sort_keys=True)
    print("wrote", args.json)
