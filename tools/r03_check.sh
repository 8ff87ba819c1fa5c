#!/bin/bash
# One GPU call: parity suite, smoke, default bench line (C3), rocprofv3 kernel stats of a short bench.
# Usage (via gpurun): bash tools/r03_check.sh TAG [skip-tests]
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 600 python -u bench.py --workdir /tmp/dk_c3 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --workdir /tmp/dk_c3 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*stats*"
find $OUT/prof -name "*kernel_trace*" -size +20M -delete
echo done
