#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per pass, as the gfx950 slot limits require):
#   FETCH_SIZE | WRITE_SIZE | SQ instruction/wait mix | TCC hit/miss.
# Usage (via gpurun): bash tools/pmc.sh TAG [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
WORK=/tmp/dk_pmc_table
timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --workdir $WORK "$@" > $OUT/gen.json 2> $OUT/gen.err || { echo "table gen failed"; tail $OUT/gen.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
            "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --workdir $WORK "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i ($pass) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*.csv" -size +30M -delete
echo done
