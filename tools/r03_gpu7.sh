#!/bin/bash
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg/typed_diff2.py > $OUT/d1.log 2>&1 || { echo "d1 failed"; tail -30 $OUT/d1.log; exit 1; }
cat $OUT/d1.log
timeout -k 10 600 python -u -m pytest tests/test_skipping.py tests/test_partitions.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_skip.log 2>&1 || { echo "skipping tests failed"; grep -E "^E " $OUT/pytest_skip.log | head -20; tail -5 $OUT/pytest_skip.log; exit 1; }
tail -1 $OUT/pytest_skip.log
for i in 1 2; do
for m in 1 0; do
DK_OPEN_ADAPTIVE=$m timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 > $OUT/b_${m}_$i.json 2> $OUT/b_${m}_$i.err || { echo "bench failed"; tail -20 $OUT/b_${m}_$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${m}_$i.json')); p=d['getScanFiles_phases_ms']; print('adaptive=$m', round(d['ms_per_step'],1), p['open_read_h2d'], p['prep_device_sizing'], p['consume'], p['close'])"
done
done
timeout -k 10 500 rocprofv3 --runtime-trace --memory-copy-trace --kernel-trace --output-format csv -d $OUT/rt -o run -- python -u bench.py --steps 2 --warmup 1 > $OUT/brt.json 2> $OUT/brt.err || { echo "runtime trace failed"; tail -20 $OUT/brt.err; exit 1; }
ls $OUT/rt
