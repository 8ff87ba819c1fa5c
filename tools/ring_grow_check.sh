#!/bin/bash
# lazily grown pinned ring: reader / async-open / lifetime tests, then two short default-config bench
# lines (engine creation and the e2e step)
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_async_open.py tests/test_reader.py tests/test_batch_lifetime.py tests/test_configs.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for k in 1 2; do
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --workdir /tmp/dk_c3 > $OUT/bench_$k.json 2> $OUT/bench_$k.err || { tail -20 $OUT/bench_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$k.json')); print(round(d['ms_per_step'],1), 'ms p50', d['step_ms_p50'], 'p90', d['step_ms_p90'], 'engine_create_ms', round(d['engine_create_ms'],1), 'jmh', round(d['jmh_op']['ms_per_op'],1), 'dev', round(d['device_step']['ms'],1))"
done
