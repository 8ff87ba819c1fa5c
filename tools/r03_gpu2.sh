#!/bin/bash
# GPU call: full parity suite, k_snap_frag stage breakdown (DK_SNAP_STATS build), C4 / C5 bench lines
# with rocprofv3 kernel stats. Usage (via gpurun): bash tools/r03_gpu2.sh TAG
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
# libdkgpu on torch's HIP runtime (the import order of bench.py's multi-GPU ranks): C3 bench
timeout -k 10 600 python -u -c "
import sys, runpy, torch
torch.zeros(1, device='cuda')
sys.argv = ['bench.py', '--steps', '3', '--warmup', '1', '--device-steps', '3', '--no-cpu-baseline', '--workdir', '/tmp/dk_c3']
runpy.run_path('bench.py', run_name='__main__')" > $OUT/bench_torchfirst.json 2> $OUT/bench_torchfirst.err || { echo "torch-first bench failed"; tail -20 $OUT/bench_torchfirst.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_torchfirst.json'))
print('torch-first c3 value %.1f M/s ms/step %.1f device %.1f ms' % (d['value']/1e6, d['ms_per_step'], d['device_step']['ms']), d['device_step']['counters'])"
if [ -f build/libdk_stats.so ]; then
  timeout -k 10 300 bash tools/_snapstats_run.sh > $OUT/snapstats.txt 2>&1 || { echo "snapstats failed"; tail -5 $OUT/snapstats.txt; }
  tail -3 $OUT/snapstats.txt
fi
for c in c5 c4; do
  timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --workdir /tmp/dk_$c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$c.json'))
print('$c', 'value %.1f M/s ms/step %.1f device %.1f ms' % (d['value']/1e6, d['ms_per_step'], d['device_step']['ms']), d['roofline']['kernel'], d['roofline']['frac'])"
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --workdir /tmp/dk_$c > $OUT/bench_prof_$c.json 2> $OUT/bench_prof_$c.err || { echo "rocprof $c failed"; tail -20 $OUT/bench_prof_$c.err; exit 1; }
  find $OUT/prof_$c -name "*kernel_trace*" -delete
  cd $GRAFT_REPO_ROOT
done
echo done
