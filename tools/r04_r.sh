#!/bin/bash
# round 4, call R: the asynchronous open for filtered scans (data skipping, partition pruning,
# row-group predicate; DK_ASYNC_FILTERED=1): their GPU tests, then a C4 A/B with consume profile
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
#DK_ASYNC_FILTERED=1 timeout -k 10 700 python -u -m pytest tests/test_skipping.py tests/test_partitions.py tests/test_configs.py tests/test_gpu_parity.py tests/test_handlers.py tests/test_dv.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
#tail -1 $OUT/pytest.log
for rep in 1 2; do
for cfg in "DK_ASYNC_FILTERED=0" "DK_ASYNC_FILTERED=1"; do
name=$(echo $cfg | tr ',=' '__')_$rep
env DK_VERBOSE=1 DK_CONSUME_PROFILE=1 $cfg timeout -k 10 500 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --full-row-steps 0 --workdir /tmp/dk_c4 > $OUT/b_${name}.json 2> $OUT/b_${name}.err || { echo "bench failed"; tail -20 $OUT/b_${name}.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${name}.json')); p=d['getScanFiles_phases_ms']; print('$cfg', $rep, round(d['ms_per_step'],1), 'dev', round(d['device_step']['ms'],1), {k: round(p[k],1) for k in ('checkpoint_open','commit_tail','replay_create_tail','device_run','consume','consume_wait','consume_column','consume_sum','close') if k in p})"
done
done
