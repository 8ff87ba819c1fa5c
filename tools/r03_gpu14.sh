#!/bin/bash
# consume-phase split (DK_CONSUME_PROFILE) + open timeline, two bench runs
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_configs.py tests/test_errors.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
DK_CONSUME_PROFILE=1 DK_VERBOSE=1 timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench failed"; tail -20 $OUT/b$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b$i.json')); p=d['getScanFiles_phases_ms']; print(round(d['ms_per_step'],1), {k: round(v,1) for k,v in p.items()})"
grep -E "\[dk\]|consume waits" $OUT/b$i.err | tail -14
done
