#!/bin/bash
# full bench lines with CPU baseline + full-size parity for C3 / C4 / C5, and a
# rocprofv3 kernel-trace summary of each (same command without the CPU baseline)
set -o pipefail
TAG=$1; shift
CFGS=${CFGS:-"c3 c4 c5"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in $CFGS; do
  W=/tmp/dk_$c
  case $c in c3) ST="--steps 10 --warmup 2";; *) ST="--steps 5 --warmup 2";; esac
  timeout -k 10 900 python3 -u bench.py --config $c $ST --workdir $W > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -30 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); cb=d.get('cpu_baseline') or {}; print('$c', round(d['ms_per_step'],1), 'ms', round(d['value']/1e6,1), 'M/s dev', round(d['device_step']['ms'],1), 'roof', d['roofline']['kernel'], round(d['roofline']['frac'] or 0,4), 'parity', json.dumps(cb.get('parity'))[:300])"
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --full-row-steps 0 --workdir $W > $OUT/bench_prof_$c.json 2> $OUT/bench_prof_$c.err || { echo "rocprof $c failed"; tail -20 $OUT/bench_prof_$c.err; exit 1; }
  cd $GRAFT_REPO_ROOT
  find $OUT/prof_$c -name "*.csv" -size +20M -delete
done
echo done
