#!/bin/bash
# k_snap_frag experiment instances (DK_SNAP_EXP flags, SX_NOWRITE): how much of the kernel the far
# references / byte stage cost. Kernel stats per instance via rocprofv3.
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --workdir /tmp/dk_c3 > $OUT/gen.json 2> $OUT/gen.err || { echo gen failed; tail $OUT/gen.err; exit 1; }
for e in 0 1 2 4; do
  DK_SNAP_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e$e -o r -- python -u bench.py --steps 1 --warmup 0 --device-steps 4 --no-cpu-baseline --workdir /tmp/dk_c3 > $OUT/e$e.json 2> $OUT/e$e.err || { echo "exp $e failed"; tail $OUT/e$e.err; exit 1; }
  grep -h "k_snap_frag" $OUT/e$e/*kernel_stats.csv | cut -d, -f1-4 | sed "s/^/exp=$e /"
done
