#!/bin/bash
# One GPU call: parity suite, smoke, default (C3 100M) bench line, rocprofv3 kernel stats of the same
# bench on the same table, then FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 run each).
# Usage (via gpurun): bash tools/r02_check.sh TAG [--skip-tests]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
WORK=/tmp/dk_c3_table
if [ "$1" != "--skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -n 2 $OUT/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -n 1 $OUT/smoke.log
fi
timeout -k 10 700 python -u bench.py --workdir $WORK > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --workdir $WORK > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --workdir $WORK > $OUT/p$i.log 2>&1 || { echo "pass $i ($pass) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*.csv" -size +30M -delete
echo done
