#!/bin/bash
# round-3 final profile: PMC passes (tools/pmc.sh) + kernel stats of the default bench
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/pmc.sh ${TAG}_pmc || { echo "pmc failed"; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*stats*"
find $OUT/prof -name "*kernel_trace.csv" -size +20M -delete
echo done
