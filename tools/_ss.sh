#!/bin/bash
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
timeout -k 10 300 bash tools/_snapstats_run.sh > $OUT/snapstats.txt 2>&1 || { echo "snapstats failed"; tail -5 $OUT/snapstats.txt; exit 1; }
cat $OUT/snapstats.txt
