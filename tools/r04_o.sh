#!/bin/bash
# round 4, call O: deferred far copies in k_snap_frag (DK_SNAP_DEFER, default on): snappy tests,
# parity, then a same-box A/B of the C3 bench
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_snappy_modes.py tests/test_plain_strings.py tests/test_gpu_parity.py tests/test_reader.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/r04_ab.sh $TAG "DK_SNAP_DEFER=1" "DK_SNAP_DEFER=0"
for f in $OUT/b_*_2.json; do python -c "import json; d=json.load(open('$f')); k=d['kernels_us']; print('$f'.split('/')[-1], {x: round(k[x]) for x in ('k_snap_frag','k_snap_walk_link','k_snap_fix','k_snappy_serial') if x in k})"; done
