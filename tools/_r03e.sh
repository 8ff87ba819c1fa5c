set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03h; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash tools/quick_bench.sh r03h --steps 6 --warmup 2 || exit 1
cd /tmp
timeout -k 10 600 rocprofv3 --hip-trace --stats -d $OUT/hip -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --workdir /tmp/dk_c3 --device-steps 0 > $OUT/hip.json 2> $OUT/hip.err || { echo "rocprof failed"; tail -5 $OUT/hip.err; exit 1; }
find $OUT/hip -name "*trace*" -size +20M -delete
echo done
