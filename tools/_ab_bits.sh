#!/bin/bash
# A/B of the snappy tag-start bitmap on the C3 bench (same table), after the GPU parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export DK_SNAPPY_MODE=page
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/gpu_all.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
unset DK_SNAPPY_MODE
for b in 1 0; do
  DK_SNAP_BITS=$b timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > gpurun_out/ab_bits$b.json 2> gpurun_out/ab_bits$b.err || { echo bench $b failed; tail gpurun_out/ab_bits$b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_bits$b.json')); k=d['kernels_us']; print('bits=$b', round(d['ms_per_step'],2), {x: k[x] for x in list(k)[:6]})"
done
