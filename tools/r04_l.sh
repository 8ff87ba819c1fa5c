#!/bin/bash
# round 4, call L: the whole GPU suite + smoke at HEAD (asynchronous open by default), then the C3
# bench line (default knobs) with DK_VERBOSE timelines
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -30; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
DK_VERBOSE=1 DK_CONSUME_PROFILE=1 timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --workdir /tmp/dk_c3 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); p=d['getScanFiles_phases_ms']; print(round(d['ms_per_step'],1), round(d['value']/1e6,1), 'dev', round(d['device_step']['ms'],1), {k: round(p[k],1) for k in ('checkpoint_open','commit_tail','replay_create_tail','consume','consume_wait','consume_sum','close') if k in p}, d.get('full_row_consume'))"
