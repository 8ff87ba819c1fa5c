#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per known byte count for 16 / 8 / 4 / 1-byte-per-lane streams (gfx950).
# Usage (via gpurun): bash tools/pmc_calib.sh TAG      (tools/calib/pmc_calib built beforehand)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/tools/calib/pmc_calib
timeout -k 10 60 $B > $OUT/run.txt 2>&1 || { echo "calib run failed"; cat $OUT/run.txt; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o k -- $B > $OUT/f.log 2>&1 || { echo "fetch pass failed"; tail -5 $OUT/f.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o k -- $B > $OUT/w.log 2>&1 || { echo "write pass failed"; tail -5 $OUT/w.log; exit 1; }
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("$OUT/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
B = 2 << 30
for (k, c), v in sorted(acc.items()):
    print("%-40s %-11s KiB/launch %12.0f  ratio to bytes %.3f" % (k, c, v[-1], v[-1] * 1024 / B))
PY
