#!/bin/bash
# A/B of environment switches on the C3 bench (and the GPU parity suite under the first switch).
# Usage (via gpurun): bash tools/ab_env.sh TAG "ENV=1 ENV2=x" ["ENV=..."...]
#   runs pytest -m gpu under the FIRST environment, then quick_bench for the baseline and each one.
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
env $1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed ($1)"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/quick_bench.sh $TAG/base --steps 4 --warmup 1 --device-steps 6 || exit 1
i=0
for e in "$@"; do
  i=$((i+1))
  echo "== $e"
  env $e bash tools/quick_bench.sh $TAG/v$i --steps 4 --warmup 1 --device-steps 6 || exit 1
done
echo done
