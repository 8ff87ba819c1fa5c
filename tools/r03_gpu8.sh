#!/bin/bash
# full GPU suite + smoke + C3 bench + rocprofv3 kernel stats of the bench
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['device_step']['ms'], d['getScanFiles_phases_ms'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python -u bench.py --steps 3 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*stats*" | head
echo done
