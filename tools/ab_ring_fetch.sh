#!/bin/bash
# k_snap_frag output-ring size: step time and FETCH/WRITE of the kernel per variant (C3 table)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab_ring; mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VARIANTS:-vA vR8 vR16}; do
  DK_LIB_PATH=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > $OUT/$v.json 2> $OUT/$v.err || { echo "bench $v failed"; tail $OUT/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); k=d['kernels_us']; print('$v', round(d['ms_per_step'],2), {x: round(k[x]) for x in list(k)[:4]})"
  (cd /tmp && DK_LIB_PATH=$GRAFT_REPO_ROOT/variants/$v.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f_$v -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > $OUT/f_$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
  python3 - <<PY
import csv, glob
v = [float(r["Counter_Value"]) for f in glob.glob("$OUT/f_$v/*counter_collection.csv") for r in csv.DictReader(open(f)) if "snap_frag" in r["Kernel_Name"]]
print("$v FETCH_SIZE KB (largest launch):", max(v) if v else None)
PY
done
