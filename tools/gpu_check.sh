#!/bin/bash
# One GPU round trip: parity suite, bench line, rocprofv3 kernel stats (+ optional per-column split).
# Usage (via gpurun): bash tools/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 500 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
if [ -n "$SPLIT" ]; then
  DK_SPLIT_LAUNCH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/split -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/split.log 2>&1 || { echo "split rocprof failed"; exit 1; }
fi
find $OUT -name "*kernel_trace.csv" -size +20M -delete
echo done
