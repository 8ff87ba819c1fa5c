#!/bin/bash
# interleaved A/B of open settings (env per config), open timeline of each
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFGS=${CFGS:-"DK_IO_THREADS=16 DK_IO_THREADS=8"}
for i in 1 2; do
for cfg in $CFGS; do
name=$(echo $cfg | tr ',=' '__')
env DK_VERBOSE=1 $(echo $cfg | tr ',' ' ') timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/b_${name}_$i.json 2> $OUT/b_${name}_$i.err || { echo "bench failed"; tail -20 $OUT/b_${name}_$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${name}_$i.json')); p=d['getScanFiles_phases_ms']; print('$cfg', round(d['ms_per_step'],1), 'open', p['checkpoint_open'], 'io', p['open_read_h2d'], 'sizing', p['prep_device_sizing'], 'consume', p['consume'], 'close', p['close'])"
grep -E "sizing slice 0|sizing slice 7|images read" $OUT/b_${name}_$i.err | tail -3
done
done
