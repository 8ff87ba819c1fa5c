#!/bin/bash
# slices shrinking toward the end of the image: the sliced-open tests, then a same-box interleaved
# A/B against every slice >= 1/8 of the bytes (DK_SLICE_TAIL=0)
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_async_open.py tests/test_configs.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
STEPS=10 REPS="1 2 3" bash tools/ab_interleave.sh $TAG "DK_SLICE_TAIL=0"
