#!/bin/bash
# open timeline (DK_VERBOSE): one bench run, the slice / landing log of its timed steps
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DK_VERBOSE=1 timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { echo "bench failed"; tail -20 $OUT/b.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b.json')); p=d['getScanFiles_phases_ms']; print(round(d['ms_per_step'],1), p)"
grep "\[dk\]" $OUT/b.err | tail -40
