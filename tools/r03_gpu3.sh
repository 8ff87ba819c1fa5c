#!/bin/bash
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_checkpoint_write.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_ckw.log 2>&1 || { echo "ckpt write tests failed"; grep -E "Error|error|assert" $OUT/pytest_ckw.log | head -20; tail -40 $OUT/pytest_ckw.log; exit 1; }
tail -1 $OUT/pytest_ckw.log
timeout -k 10 400 python -u tools/ckpt_write_bench.py 2000000 4 > $OUT/ckw_2M.json 2> $OUT/ckw_2M.err || { echo "ckw 2M failed"; tail -20 $OUT/ckw_2M.err; cat $OUT/ckw_2M.json; exit 1; }
cat $OUT/ckw_2M.json
timeout -k 10 600 python -u tools/ckpt_write_bench.py 12500000 8 > $OUT/ckw_12M.json 2> $OUT/ckw_12M.err || { echo "ckw 12.5M failed"; tail -20 $OUT/ckw_12M.err; cat $OUT/ckw_12M.json; exit 1; }
cat $OUT/ckw_12M.json
echo done
