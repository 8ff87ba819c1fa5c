#!/bin/bash
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg/typed_diff.py us > $OUT/diff.log 2>&1 || { echo "diff failed"; tail -30 $OUT/diff.log; exit 1; }
head -c 6000 $OUT/diff.log
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $OUT/b.json 2> $OUT/b.err || { echo "bench failed"; tail -20 $OUT/b.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b.json')); print(d['value'], d['ms_per_step'], d['getScanFiles_phases_ms'])"
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run -- python -u bench.py --steps 2 --warmup 1 > $OUT/bt.json 2> $OUT/bt.err || { echo "trace failed"; tail -20 $OUT/bt.err; exit 1; }
find $OUT/trace -name "*.csv" | head
echo done
