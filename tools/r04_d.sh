#!/bin/bash
# round 4, call D: GPU tests over the tail parse / replay create, then the default and async opens'
# tail timings (DK_VERBOSE) and phases
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_plain_strings.py tests/test_snapshot_pm.py tests/test_gpu_parity.py tests/test_golden_fixtures.py tests/test_owner.py tests/test_batch_lifetime.py tests/test_reader.py tests/test_snappy_modes.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in "DK_SLICE_DECODE=0" "DK_SLICE_DECODE=1,DK_ASYNC_OPEN=1"; do
name=$(echo $cfg | tr ',=' '__')
env DK_VERBOSE=1 DK_CONSUME_PROFILE=1 $(echo $cfg | tr ',' ' ') timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --full-row-steps 0 --workdir /tmp/dk_c3 > $OUT/b_${name}.json 2> $OUT/b_${name}.err || { echo "bench failed"; tail -20 $OUT/b_${name}.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${name}.json')); p=d['getScanFiles_phases_ms']; print('$cfg', round(d['ms_per_step'],1), {k: p[k] for k in ('checkpoint_open','commit_tail','replay_create_tail','device_run','consume','consume_wait','consume_sum','close','close_detach','close_replay','close_inputs') if k in p})"
grep -E "commit tail|replay create" $OUT/b_${name}.err | tail -2
grep -E "decode of files|group .* issued|file .* ready|sizing slice|sizing done" $OUT/b_${name}.err | tail -40 > $OUT/timeline_${name}.txt || true
done
