#!/bin/bash
# Same-box interleaved A/B of one environment switch on a bench config: base, variant, base, variant.
# Usage (via gpurun): bash tools/ab_interleave.sh TAG "ENV=1" [bench args...]
set -o pipefail
TAG=$1; E=$2; shift 2
for rep in ${REPS:-1 2}; do
  bash tools/quick_bench.sh $TAG/base_$rep --steps ${STEPS:-4} --warmup 1 --device-steps 4 --full-row-steps 1 --jmh-ops 0 "$@" || exit 1
  env $E bash tools/quick_bench.sh $TAG/var_$rep --steps ${STEPS:-4} --warmup 1 --device-steps 4 --full-row-steps 1 --jmh-ops 0 "$@" || exit 1
done
echo done
