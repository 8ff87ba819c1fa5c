#!/bin/bash
# default GPU suite; the scan/parity/error tests again with the per-slice decode + async open; A/B bench
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
true
DK_SLICE_DECODE=1 DK_ASYNC_OPEN=1 timeout -k 10 900 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py tests/test_errors.py tests/test_snappy_modes.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_async.log 2>&1 || { echo "async gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_gpu_async.log | head -20; tail -5 $OUT/pytest_gpu_async.log; exit 1; }
tail -1 $OUT/pytest_gpu_async.log
CFGS=${CFGS:-"DK_SLICE_DECODE=1,DK_ASYNC_OPEN=1 DK_SLICE_DECODE=0 DK_SLICE_DECODE=1"}
for i in 1 2; do
for cfg in $CFGS; do
name=$(echo $cfg | tr ',=' '__')
env DK_CONSUME_PROFILE=1 DK_VERBOSE=1 $(echo $cfg | tr ',' ' ') timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/b_${name}_$i.json 2> $OUT/b_${name}_$i.err || { echo "bench failed"; tail -20 $OUT/b_${name}_$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${name}_$i.json')); p=d['getScanFiles_phases_ms']; print('$cfg', round(d['ms_per_step'],1), round(d['value']/1e6,1), 'open', p['checkpoint_open'], 'run', p['device_run'], 'consume', round(p['consume'],1), 'wait', round(p.get('consume_wait',0),1), 'close', p['close'], 'dev', round(d['device_step']['ms'],1))"
done
done
