#!/bin/bash
# kernel-trace A/B of libdkgpu variants (DK_LIB_PATH) on the 12.5M-row C3-shaped snappy table, one
# synchronous single-slice open per decode (one k_snap_frag launch over every fragment).
# Usage (via gpurun): bash tools/snap_variants.sh TAG LIB1 [LIB2 ...]   ("default" = the in-tree build)
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W=/tmp/dk_snapstats
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, '.')
from delta_amd import synth
synth.write_table('$W', synth.TableSpec(n_adds=12_500_000, n_parts=8, compression='snappy', n_commits=50, adds_per_commit=100, removes_per_commit=100))
" > $OUT/gen.log 2>&1 || { echo gen failed; tail $OUT/gen.log; exit 1; }
cat > /tmp/snap_run.py <<PY
import sys, hashlib; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from delta_amd import kernel as K
eng = K.GpuEngine()
for i in range(3):
    snap = K.Table.forPath(eng, '$W').getLatestSnapshot(eng)
    sc = snap.getScanBuilder().build()
    h = hashlib.sha256(); n = 0
    for b in sc.getScanFiles(eng):
        c = b.data['add.path']; n += b.size
        h.update(bytes(c.chars[:int(c.offs[b.size])]))
    sc.close()
print('rows', n, h.hexdigest()[:16])
PY
cd /tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = default ]; then L="DK_VERBOSE="; else L="DK_LIB_PATH=$GRAFT_REPO_ROOT/$lib"; fi
  env $L DK_ASYNC_OPEN=0 DK_OPEN_SLICES=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$i -o k -- python3 /tmp/snap_run.py > $OUT/v$i.log 2>&1 || { echo "run $i failed"; tail -5 $OUT/v$i.log; exit 1; }
  python3 - $OUT/v$i "$lib" <<PY
import csv, glob, sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'snap' in r['Name'] and 'serial' not in r['Name']:
            print(sys.argv[2], r['Name'][:24], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3), [l for l in open(sys.argv[1] + '.log').read().splitlines() if l.startswith('rows')])
PY
done
