#!/bin/bash
# snappy mode comparison on the C3 bench table: frag mode, page mode + bitmap, page mode without bitmap
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "frag 1" "page 1" "page 0"; do
  set -- $cfg
  DK_SNAPPY_MODE=$1 DK_SNAP_BITS=$2 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > gpurun_out/ab_$1$2.json 2> gpurun_out/ab_$1$2.err || { echo bench $cfg failed; tail gpurun_out/ab_$1$2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$1$2.json')); k=d['kernels_us']; print('$cfg', round(d['ms_per_step'],2), {x: k[x] for x in list(k)[:5]})"
done
