#!/bin/bash
# One GPU call: default bench line, rocprofv3 kernel stats of the same bench, then FETCH_SIZE and
# WRITE_SIZE passes (one rocprofv3 run each) over a short run of the same table.
# Usage (via gpurun): bash tools/prof_round.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
WORK=/tmp/dk_prof_table
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --workdir $WORK "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --workdir $WORK "$@" > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --device-steps 2 --no-cpu-baseline --workdir $WORK "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i ($pass) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*.csv" -size +30M -delete
echo done
