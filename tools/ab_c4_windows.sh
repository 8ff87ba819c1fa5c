#!/bin/bash
# same-box A/B of the whole-window image copies (DK_OPEN_WINDOWS) on C4, two interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04c4w; export TMPDIR=/tmp
for rep in 1 2; do for w in 0 1; do
DK_OPEN_WINDOWS=$w timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --full-row-steps 0 --workdir /tmp/dk_c4 > gpurun_out/r04c4w/b_${w}_${rep}.json 2> gpurun_out/r04c4w/b_${w}_$rep.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r04c4w/b_${w}_${rep}.json')); print('windows=$w', $rep, round(d['ms_per_step'],1))"
done; done
