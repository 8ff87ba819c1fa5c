#!/bin/bash
# the whole -m gpu suite + smoke, then the default bench line (the driver's command) twice
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -30; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for k in 1 2; do
  timeout -k 10 600 python -u bench.py > $OUT/bench_default_$k.json 2> $OUT/bench_default_$k.err || { echo "bench failed"; tail -30 $OUT/bench_default_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_default_$k.json')); print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],1), 'ms p50', d.get('step_ms_p50'), 'p90', d.get('step_ms_p90'), 'dev', round(d['device_step']['ms'],1), 'roof', round(d['roofline']['frac'],4), 'parity', json.dumps((d.get('cpu_baseline') or {}).get('parity'))[:200])"
done
