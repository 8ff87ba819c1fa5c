#!/bin/bash
# GPU parity tests that exercise the checkpoint probe (DVs), then the C4 line with its
# full-size oracle parity and a kernel-trace summary
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_configs.py tests/test_owner.py > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
CFGS=c4 bash tools/bench_lines.sh $TAG/b
