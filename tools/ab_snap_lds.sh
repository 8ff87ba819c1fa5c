#!/bin/bash
# A/B of k_snap_frag LDS sizings (variants/v*.so built by tools/build_variant.py) on the C3 bench
# table, then the snappy parity tests on each variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_lds; mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VARIANTS:-vA vB vC vD}; do
  DK_LIB_PATH=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > $OUT/$v.json 2> $OUT/$v.err || { echo "bench $v failed"; tail $OUT/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); k=d['kernels_us']; print('$v', round(d['ms_per_step'],2), {x: round(k[x]) for x in list(k)[:5]})"
done
for v in ${VARIANTS:-vA vB vC vD}; do
  DK_LIB_PATH=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${KEXPR:-snappy or v2 or c5 or C3 or c3 or reader}" > $OUT/pt_$v.log 2>&1 || { echo "tests $v failed"; tail -20 $OUT/pt_$v.log; exit 1; }
  echo "$v tests: $(tail -n 1 $OUT/pt_$v.log)"
done
