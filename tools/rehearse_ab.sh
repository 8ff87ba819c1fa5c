#!/bin/bash
# same-box A/B of the 8-rank rehearsal: the head's library against a variant (DK_LIB_PATH)
set -o pipefail
TAG=$1; LIB=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in head var; do
    if [ $v = var ]; then L="DK_LIB_PATH=$GRAFT_REPO_ROOT/$LIB"; else L="DK_VERBOSE="; fi
    env $L timeout -k 10 600 python3 -u tools/rehearse_rank.py --world 8 --config c3 --workdir /tmp/dk_c3 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail -30 $OUT/${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); pr=d['per_rank']; pr=pr if isinstance(pr,list) else list(pr.values()); print('$v', d['rehearsed_step_ms'], d['counters_match'], 'open', sorted(round(r['open_ms'],1) for r in pr), 'prepare', sorted(round(r['prepare_ms'],1) for r in pr))"
  done
done
