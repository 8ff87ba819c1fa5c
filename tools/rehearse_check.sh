#!/bin/bash
# one-GPU rehearsal of every rank of an N=8 owner-mode C3 scan at the head
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/rehearse_rank.py --world 8 --config c3 --workdir /tmp/dk_c3 > $OUT/warm.json 2> $OUT/rehearse.err || { tail -30 $OUT/rehearse.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/warm.json')); print(d['rehearsed_step_ms'], d['rehearsed_actions_per_s'], d['counters_match'])"
