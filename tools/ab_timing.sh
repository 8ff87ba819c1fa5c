#!/bin/bash
# Timing-only A/B of kernel variants (no parity: for diagnostic variants that skip work).
# Usage (via gpurun): bash tools/ab_timing.sh TAG so1 so2 ...
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'.')
from delta_amd import synth
synth.write_table('/tmp/abt', synth.TableSpec(n_adds=10_000_000, pv_keys=2, with_stats_parsed=True, n_commits=100, adds_per_commit=50, removes_per_commit=50, seed=20250218))
" > $OUT/gen.log 2>&1 || { echo gen failed; exit 1; }
for so in "$@"; do
  v=$(basename $so .so)
  DK_LIB_PATH=$GRAFT_REPO_ROOT/$so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --workdir /tmp/abt > $OUT/b_$v.json 2> $OUT/b_$v.err || { echo "bench failed: $v"; tail $OUT/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', round(d['ms_per_step'],3), {k: round(x) for k, x in list(d['kernels_us'].items())[:8]})"
done
