#!/bin/bash
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg/typed_diff2.py > $OUT/d1.log 2>&1 || { echo "d1 failed"; tail -30 $OUT/d1.log; exit 1; }
cat $OUT/d1.log
DK_NO_STATS_PARSED=1 timeout -k 10 300 python -u tools/dbg/typed_diff2.py > $OUT/d2.log 2>&1 || { echo "d2 failed"; tail -30 $OUT/d2.log; exit 1; }
echo "--- json only"; cat $OUT/d2.log
timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 > $OUT/b_adapt.json 2> $OUT/b_adapt.err || { echo "bench failed"; tail -20 $OUT/b_adapt.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_adapt.json')); print('adaptive', d['value'], d['ms_per_step'], d['getScanFiles_phases_ms'])"
DK_OPEN_ADAPTIVE=0 timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 > $OUT/b_fixed.json 2> $OUT/b_fixed.err || { echo "bench failed"; tail -20 $OUT/b_fixed.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_fixed.json')); print('fixed8', d['value'], d['ms_per_step'], d['getScanFiles_phases_ms'])"
DK_OPEN_SLICES=4 timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 > $OUT/b_a4.json 2> $OUT/b_a4.err || { echo "bench failed"; tail -20 $OUT/b_a4.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_a4.json')); print('adaptive4', d['value'], d['ms_per_step'], d['getScanFiles_phases_ms'])"
