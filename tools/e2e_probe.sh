#!/bin/bash
# C3 bench line + a DK_VERBOSE end-to-end run (host I/O / metadata / prepare split of checkpoint_open)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/e2e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --workdir /tmp/c3w --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(round(d['ms_per_step'],2), d['end_to_end']['getScanFiles_ms'], d['end_to_end']['phases_ms'], {k: round(v) for k, v in list(d['kernels_us'].items())[:8]})"
DK_VERBOSE=1 timeout -k 10 300 python -u bench.py --workdir /tmp/c3w --no-cpu-baseline --steps 1 --warmup 0 --e2e-reps 1 > $OUT/verbose.json 2> $OUT/verbose.err || { echo "verbose failed"; tail $OUT/verbose.err; exit 1; }
grep "\[dk\]" $OUT/verbose.err | tail -n 8
