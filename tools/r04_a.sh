#!/bin/bash
# round 4, call A: owner-mode GPU tests, then the async-open A/B (default vs DK_SLICE_DECODE+DK_ASYNC_OPEN)
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_owner.py tests/test_exchange.py tests/test_batch_lifetime.py tests/test_shard.py tests/test_gpu_parity.py tests/test_skipping.py tests/test_dv.py tests/test_handlers.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_owner.log 2>&1 || { echo "owner gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_owner.log | head -30; tail -5 $OUT/pytest_owner.log; exit 1; }
tail -1 $OUT/pytest_owner.log
for i in 1 2; do
for cfg in "DK_SLICE_DECODE=0" "DK_SLICE_DECODE=1,DK_ASYNC_OPEN=1"; do
name=$(echo $cfg | tr ',=' '__')
env DK_CONSUME_PROFILE=1 $(echo $cfg | tr ',' ' ') timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --workdir /tmp/dk_c3 > $OUT/b_${name}_$i.json 2> $OUT/b_${name}_$i.err || { echo "bench failed"; tail -20 $OUT/b_${name}_$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${name}_$i.json')); p=d['getScanFiles_phases_ms']; print('$cfg', round(d['ms_per_step'],1), round(d['value']/1e6,1), 'open', p['checkpoint_open'], 'run', p['device_run'], 'consume', round(p['consume'],1), 'wait', round(p.get('consume_wait',0),1), 'close', p['close'], 'dev', round(d['device_step']['ms'],1))"
done
done
