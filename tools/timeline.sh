#!/bin/bash
# one C3 step timeline: the open's [dk] events and the consumer's batch arrivals on one clock
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DK_VERBOSE=1 DK_CONSUME_PROFILE=1 timeout -k 10 600 python3 -u bench.py --config c3 --steps 3 --warmup 1 \
  --no-cpu-baseline --full-row-steps 0 --workdir /tmp/dk_c3 "$@" > $OUT/bench.json 2> $OUT/bench.err
