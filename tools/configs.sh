#!/bin/bash
# GPU parity suite + one bench line per BASELINE.json config.
# Usage (via gpurun): bash tools/configs.sh TAG c1 c4 c5 ...
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
for c in "$@"; do
  timeout -k 10 900 python -u bench.py --config $c --steps 10 --warmup 2 $BENCH_ARGS > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', '%.3g actions/s' % d['value'], round(d['ms_per_step'],3), 'ms/step', 'snapshot', round(d['snapshot_load_ms'],1), 'ms', d['counters'], {k: round(x) for k, x in list(d['kernels_us'].items())[:6]})"
done
