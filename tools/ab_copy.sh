#!/bin/bash
# A/B the string copy kernel variants (DK_COPY_DBG bits: 1 no output, 2 no hash, 4 no staging loads)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
python -u -c "
import sys; sys.path.insert(0,'.')
from delta_amd import synth
synth.write_table('/tmp/abt', synth.TableSpec(n_adds=10_000_000, pv_keys=2, with_stats_parsed=True, n_commits=100, adds_per_commit=50, removes_per_commit=50, seed=20250218))
" > $OUT/gen.log 2>&1 || exit 1
for v in 0 1 2; do
  DK_COPY_DBG=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --workdir /tmp/abt > $OUT/b$v.json 2>$OUT/b$v.err || { echo fail $v; tail $OUT/b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$v.json')); print($v, d['kernels_us'].get('k_string_copy'), d['ms_per_step'])"
done
