#!/bin/bash
# GPU parity suite (optionally a -k selection) into gpurun_out/TAG/pytest_gpu.log
# Usage (via gpurun): bash tools/gpu_tests.sh TAG [pytest -k expression]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=()
[ -n "$1" ] && K=(-k "$1")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -n 25 $OUT/pytest_gpu.log
exit $rc
