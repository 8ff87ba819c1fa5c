#!/bin/bash
# full GPU suite, then two profiled bench runs (consume split + open timeline)
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
DK_CONSUME_PROFILE=1 DK_VERBOSE=1 timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench failed"; tail -20 $OUT/b$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b$i.json')); p=d['getScanFiles_phases_ms']; print(round(d['ms_per_step'],1), round(d['value']/1e6,1), {k: round(v,1) for k,v in p.items()})"
grep -E "consume waits" $OUT/b$i.err | tail -2 | cut -c1-300
done
