#!/bin/bash
# A/B of snappy kernel variants (tools/build_variant.py builds) on C3: snappy parity subset per variant,
# then the C3 bench per variant, interleaved twice. Usage (via gpurun): bash tools/ab_snap.sh TAG so1 so2 ...
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for so in "$@"; do
  v=$(basename $so .so)
  DK_LIB_PATH=$GRAFT_REPO_ROOT/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_errors.py -k "snappy or c3 or c5 or sidecar or damaged" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t_$v.log 2>&1 || { echo "parity failed: $v"; tail -15 $OUT/t_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/t_$v.log)"
done
for rep in 1 2; do
  for so in "$@"; do
    v=$(basename $so .so)
    DK_LIB_PATH=$GRAFT_REPO_ROOT/$so timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --device-steps 8 --no-cpu-baseline --workdir /tmp/dk_c3 > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { echo "bench failed: $v"; tail $OUT/b_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$rep.json')); print('$v', 'e2e %.1f ms' % d['ms_per_step'], 'dev %.2f ms' % d['device_step']['ms'], {k: round(x) for k, x in list(d['kernels_us'].items())[:6]})"
  done
done
