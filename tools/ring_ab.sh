#!/bin/bash
# default bench line (no CPU baseline) under environment variants: bash tools/ring_ab.sh TAG "ENV=a" "ENV=b" ...
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
k=0
for v in "$@"; do
  k=$((k+1))
  env $v timeout -k 10 600 python -u bench.py --no-cpu-baseline --full-row-steps 0 --jmh-ops 0 > $OUT/bench_$k.json 2> $OUT/bench_$k.err || { echo "bench $v failed"; tail -30 $OUT/bench_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$k.json')); p=d['getScanFiles_phases_ms']; print('$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],1), 'ms p50', d.get('step_ms_p50'), 'p90', d.get('step_ms_p90'), 'open', p.get('checkpoint_open'), 'rd', p.get('open_read_h2d'), 'prep', p.get('open_prepare'), 'consume', p.get('consume'))"
done
