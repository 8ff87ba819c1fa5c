#!/bin/bash
# one C3 timeline under a kernel + memory-copy trace, with the [dk] events on the same clock
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline --full-row-steps 0 \
  --workdir /tmp/dk_c3 > /dev/null 2> $OUT/gen.err
cd /tmp
DK_VERBOSE=1 DK_CONSUME_PROFILE=1 timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/tr -o run \
  --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline \
  --full-row-steps 0 --workdir /tmp/dk_c3 "$@" > $OUT/bench.json 2> $OUT/bench.err
