#!/bin/bash
# snappy batch statistics on an 8-part C3-shaped table (12.5M rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -c "
from delta_amd import synth
synth.write_table('/tmp/c3s', synth.TableSpec(n_adds=12_500_000, seed=20250218, n_parts=8, compression='snappy', n_commits=100, adds_per_commit=100, removes_per_commit=100, readd_frac=0.1, dup_frac=0.05))
" > gpurun_out/ss_gen.log 2>&1 || { echo gen failed; tail gpurun_out/ss_gen.log; exit 1; }
DK_LIB_PATH=build/libdk_stats.so timeout -k 10 200 python3 tools/snap_stats.py /tmp/c3s > gpurun_out/snapstats.txt 2>&1 || { echo stats failed; tail gpurun_out/snapstats.txt; exit 1; }
cat gpurun_out/snapstats.txt
