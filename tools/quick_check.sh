#!/bin/bash
# targeted GPU tests (-k expression) + a short C3 bench on a reused table
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/quick; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${1:-parity or configs or shard}" > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); k=d['kernels_us']; print(round(d['ms_per_step'],2), {x: round(v) for x, v in list(k.items())[:9]})"
