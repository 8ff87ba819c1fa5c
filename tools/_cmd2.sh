set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "snappy or v2 or multipart or c5" > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
python -c "
from delta_amd import synth
synth.write_table('/tmp/t10', synth.TableSpec(n_adds=10_000_000, n_parts=8, compression='snappy', n_commits=20, adds_per_commit=100, removes_per_commit=100))
" || exit 1
DK_SNAPPY_MODE=frag DK_LIB_PATH=$GRAFT_REPO_ROOT/build/libdk_stats.so timeout -k 10 200 python -u tools/snap_stats.py /tmp/t10
DK_SNAPPY_MODE=frag timeout -k 10 500 python tools/snap_ab.py /tmp/t10 delta_amd/libdkgpu.so exp=16 exp=24
