#!/bin/bash
# One short bench run (no CPU baseline) with extra environment for A/B: bash tools/quick_bench.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --no-cpu-baseline --workdir /tmp/dk_c3 "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.load(open('$OUT/bench.json'))
print('value %.1f M/s  ms/step %.1f  device %.1f ms' % (d['value']/1e6, d['ms_per_step'], d['device_step']['ms']))
print(json.dumps(d['getScanFiles_phases_ms']))
print(json.dumps(d['kernels_us']))"
