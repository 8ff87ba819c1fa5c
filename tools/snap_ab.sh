#!/bin/bash
# k_snap_pipe vs k_snap_frag on a 12.5M-row C3-shaped snappy table: kernel trace + one SQ PMC pass
# per variant (DK_SNAP_PIPE=1 / 0: a switch of the profiles/r05/snap_pipe_ab patch only; without
# the patch both passes run the same kernel). Usage (via gpurun): bash tools/snap_ab.sh TAG
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W=/tmp/dk_snapstats
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, '.')
from delta_amd import synth
synth.write_table('$W', synth.TableSpec(n_adds=12_500_000, n_parts=8, compression='snappy', n_commits=50, adds_per_commit=100, removes_per_commit=100))
" > $OUT/gen.log 2>&1 || { echo gen failed; tail $OUT/gen.log; exit 1; }
cat > /tmp/snap_run.py <<PY
import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from delta_amd import kernel as K
eng = K.GpuEngine()
for i in range(3):
    snap = K.Table.forPath(eng, '$W').getLatestSnapshot(eng)
    sc = snap.getScanBuilder().build()
    n = sum(b.size for b in sc.getScanFiles(eng))
    sc.close()
print('rows', n)
PY
cd /tmp
for pipe in 1 0; do
  DK_SNAP_PIPE=$pipe timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$pipe -o k -- python3 /tmp/snap_run.py > $OUT/kt$pipe.log 2>&1 || { echo "trace $pipe failed"; tail -5 $OUT/kt$pipe.log; exit 1; }
  DK_SNAP_PIPE=$pipe timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/pmc$pipe -o k -- python3 /tmp/snap_run.py > $OUT/pmc$pipe.log 2>&1 || { echo "pmc $pipe failed"; tail -5 $OUT/pmc$pipe.log; exit 1; }
done
find $OUT -name "*.csv" -size +30M -delete
cd $GRAFT_REPO_ROOT
python3 - <<PY
import csv, glob, collections
for pipe in (1, 0):
    for f in glob.glob('$OUT/kt%d/**/*kernel_stats.csv' % pipe, recursive=True):
        for r in csv.DictReader(open(f)):
            if 'snap' in r['Name']:
                print(pipe, r['Name'][:40], r['Calls'], r['AverageNs'])
    for f in glob.glob('$OUT/kt%d/**/*kernel_trace.csv' % pipe, recursive=True):
        for r in csv.DictReader(open(f)):
            if 'snap_pipe' in r['Kernel_Name'] or 'snap_frag' in r['Kernel_Name']:
                print(pipe, {k: r[k] for k in r if k in ('LDS_Block_Size', 'VGPR_Count', 'Arch_VGPR_Count', 'SGPR_Count', 'Scratch_Size', 'Workgroup_Size', 'Grid_Size', 'Lds_Size', 'Accum_VGPR_Count')})
                break
    agg = collections.defaultdict(float)
    for f in glob.glob('$OUT/pmc%d/**/*counter_collection.csv' % pipe, recursive=True):
        for r in csv.DictReader(open(f)):
            if 'snap_pipe' in r['Kernel_Name'] or 'snap_frag' in r['Kernel_Name']:
                agg[r['Counter_Name']] += float(r['Counter_Value'])
    print(pipe, dict(agg))
PY
