set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab5; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'.')
import bench
from delta_amd import synth
synth.write_table('/tmp/abt5', bench.table_spec(bench.CONFIGS['c5'], 10_000_000, 20250218))
" > $OUT/gen.log 2>&1 || { echo gen failed; exit 1; }
for so in ${VARIANTS:-variants/v_cur.so}; do
  v=$(basename $so .so)
  DK_LIB_PATH=$GRAFT_REPO_ROOT/$so timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --workdir /tmp/abt5 > $OUT/b_$v.json 2> $OUT/b_$v.err || { echo "bench failed: $v"; tail $OUT/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', round(d['ms_per_step'],3), {k: round(x) for k, x in list(d['kernels_us'].items())[:4]})"
done
