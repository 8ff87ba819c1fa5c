#!/bin/bash
# round 4, call J: k_snap_lds correctness (snappy modes, plain strings and the snappy parity cases
# with DK_SNAP_LDS=1), then a same-box A/B of the C3 bench with DK_SNAP_LDS=0 / 1
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_snappy_modes.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_modes.log 2>&1 || { echo "modes failed"; grep -E "^E |FAILED|Error" $OUT/pytest_modes.log | head -30; tail -5 $OUT/pytest_modes.log; exit 1; }
tail -1 $OUT/pytest_modes.log
DK_SNAP_LDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_plain_strings.py tests/test_reader.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_lds.log 2>&1 || { echo "lds parity failed"; grep -E "^E |FAILED|Error" $OUT/pytest_lds.log | head -30; tail -5 $OUT/pytest_lds.log; exit 1; }
tail -1 $OUT/pytest_lds.log
bash tools/r04_ab.sh $TAG "DK_SNAP_LDS=0" "DK_SNAP_LDS=1"
