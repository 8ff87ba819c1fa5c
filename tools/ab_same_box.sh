#!/bin/bash
# same-box A/B of bench configurations (env settings, comma-separated per config), each run
# twice interleaved; prints ms_per_step and the main phases
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
for cfg in "$@"; do
name=$(echo $cfg | tr ',=/' '___')_$rep
env DK_VERBOSE=1 DK_CONSUME_PROFILE=1 $(echo $cfg | tr ',' ' ') timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --full-row-steps 0 --workdir /tmp/dk_c3 > $OUT/b_${name}.json 2> $OUT/b_${name}.err || { echo "bench failed"; tail -20 $OUT/b_${name}.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b_${name}.json')); p=d['getScanFiles_phases_ms']; print('$cfg', $rep, round(d['ms_per_step'],1), 'dev', round(d['device_step']['ms'],1), {k: round(p[k],1) for k in ('checkpoint_open','commit_tail','replay_create_tail','consume','consume_wait','consume_sum','close') if k in p})"
done
done
