set -o pipefail
python -c "
from delta_amd import synth
synth.write_table('/tmp/t10', synth.TableSpec(n_adds=10_000_000, n_parts=8, compression='snappy', n_commits=20, adds_per_commit=100, removes_per_commit=100))
" || exit 1
DK_SNAPPY_MODE=frag timeout -k 10 500 python tools/snap_ab.py /tmp/t10 delta_amd/libdkgpu.so build/lib_NO_FAR.so build/lib_NO_BYTES.so build/lib_NO_RESOLVE.so build/lib_ONLY_DISCOVERY.so
