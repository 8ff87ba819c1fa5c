#!/bin/bash
# snappy modes on the C3 table: page (default), hybrid (fragments + bitmap), frag; hybrid with the
# smaller-LDS variant; then the snappy parity tests in hybrid mode
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_hybrid; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail $OUT/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); k=d['kernels_us']; print('$n', round(d['ms_per_step'],2), d['counters'], {x: round(v) for x, v in list(k.items())[:6]})"
}
run page DK_SNAPPY_MODE=page || exit 1
run hybrid DK_SNAPPY_MODE=hybrid || exit 1


DK_SNAPPY_MODE=hybrid timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "snappy or v2 or c5 or C3 or c3 or repeated or reader" > $OUT/pt_hybrid.log 2>&1 || { echo "hybrid tests failed"; tail -20 $OUT/pt_hybrid.log; exit 1; }
echo "hybrid tests: $(tail -n 1 $OUT/pt_hybrid.log)"
