#!/bin/bash
# k_snap_frag per-batch cycle breakdown (DK_SNAP_STATS build) on a 12.5M-row C3-shaped table
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W=/tmp/dk_snapstats
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, '.')
from delta_amd import synth
synth.write_table('$W', synth.TableSpec(n_adds=12_500_000, n_parts=8, compression='snappy', n_commits=50, adds_per_commit=100, removes_per_commit=100))
" > $OUT/gen.log 2>&1 || { echo gen failed; tail $OUT/gen.log; exit 1; }
DK_LIB_PATH=${DK_STATS_LIB:-stats_lib/libdk_stats.so} timeout -k 10 300 python3 -u tools/snap_stats.py $W > $OUT/snap_stats.txt 2>&1 || { echo stats failed; tail -20 $OUT/snap_stats.txt; exit 1; }
cat $OUT/snap_stats.txt
