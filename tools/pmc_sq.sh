#!/bin/bash
# SQ instruction-mix / stall passes (one rocprofv3 run per pass) over a short bench run.
# Usage (via gpurun): bash tools/pmc_sq.sh TAG [bench args...]
set -o pipefail
TAG=${1:-sq}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
WORK=/tmp/dk_sq_table
timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --workdir $WORK "$@" > $OUT/gen.json 2> $OUT/gen.err || { echo "table gen failed"; tail $OUT/gen.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
            "SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --workdir $WORK "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
find $OUT -name "*.csv" -size +30M -delete
echo done
